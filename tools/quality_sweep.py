"""Attribution sweep of the bf16 (C3) training-quality gap: the 1000-step C3 run of
tests/test_gpu_quality.py in four arms over several sample streams, one JSON line per run and a summary.

  arms  bf16        the product mode: bf16 operand images, σ recovered from the bf16 activation image
        bf16_sig32  the same images as GEMM operands, σ from an fp32 copy of the activation (fields.SIGMA_FP32)
        bf16_noimg  no operand images: fp32 operands rounded while staging (the same products), σ and the
                    second-order term's s, u̇ from fp32 (fields.BF16_IMAGES off)
        bf16x6      the fp32-class GEMMs
The two attribution arms run the layer-by-layer composition (renderer.RENDER_NATIVE / fields.MLP_NATIVE off),
which honours the switches; the other two the C entry points (bitwise that composition).

    python tools/quality_sweep.py OUT.json [--arms a,b] [--seeds none,12345,...]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "cope-nerf_amd"), ROOT, os.path.join(ROOT, "tests")]

ARMS = {"bf16": ("bf16", {}), "bf16_sig32": ("bf16", {"SIGMA_FP32": True}),
        "bf16_noimg": ("bf16", {"BF16_IMAGES": False}), "bf16x6": ("bf16x6", {})}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("out")
    ap.add_argument("--arms", default="bf16,bf16_sig32,bf16_noimg,bf16x6")
    ap.add_argument("--seeds", default="none,12345,777,4242,31337,9001")
    args = ap.parse_args()
    from copenerf import fields, renderer
    import test_gpu_quality as Q
    seeds = [None if s == "none" else int(s) for s in args.seeds.split(",")]
    runs = []
    for sd in seeds:
        for arm in args.arms.split(","):
            mode, sw = ARMS[arm]
            composed = bool(sw)
            saved = {k: getattr(fields, k) for k in sw}
            for k, v in sw.items():
                setattr(fields, k, v)
            renderer.RENDER_NATIVE = fields.MLP_NATIVE = not composed
            t0 = time.time()
            try:
                r = Q._train(mode, sd)
            finally:
                for k, v in saved.items():
                    setattr(fields, k, v)
                renderer.RENDER_NATIVE = fields.MLP_NATIVE = True
            r.update(arm=arm, composed=composed, s=round(time.time() - t0, 1))
            runs.append(r)
            print(json.dumps({k: v for k, v in r.items() if not k.endswith("_curve")}), flush=True)
    summary = {}
    for arm in args.arms.split(","):
        rs = [r for r in runs if r["arm"] == arm]
        summary[arm] = {"psnr_mean": sum(r["psnr"] for r in rs) / len(rs),
                        "l1_mean": sum(r["l1_final"] for r in rs) / len(rs),
                        "psnr": [round(r["psnr"], 2) for r in rs]}
    print(json.dumps(summary), flush=True)
    with open(args.out, "w") as f:
        json.dump({"steps": Q.STEPS, "rays": 4096, "workload": "c3 (skateboard stage 1) on the textured room",
                   "seeds": [None if s is None else s for s in seeds], "arms": {a: ARMS[a][1] for a in summary},
                   "summary": summary, "runs": runs}, f)


if __name__ == "__main__":
    main()
