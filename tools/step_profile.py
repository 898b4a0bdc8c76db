"""Per-launch GEMM table of one C2 train step (shape-keyed HIP-event timer)."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "cope-nerf_amd"), ROOT]
from copenerf import ops  # noqa: E402
from copenerf.train_step import SyntheticTrainer  # noqa: E402


def main():
    steps = int(os.environ.get("STEPS", 5))
    tr = SyntheticTrainer("cuda:0", rays=int(os.environ.get("RAYS", 4096)), mfma_dtype=os.environ.get("MODE", "bf16x6"))
    for _ in range(3):
        tr.step()
    torch.cuda.synchronize()
    timer = ops.KernelTimer(detail=True)
    ops.set_kernel_timer(timer)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(steps):
        tr.step()
    e1.record()
    ops.set_kernel_timer(None)
    agg = timer.summary()
    step_ms = e0.elapsed_time(e1) / steps
    tot_ms = sum(a["ms"] for a in agg.values()) / steps
    tot_fl = sum(a["flops"] for a in agg.values()) / steps
    print(f"step {step_ms:.3f} ms, GEMM {tot_ms:.3f} ms, GEMM {tot_fl / 1e12:.3f} TFLOP/step "
          f"({tot_fl / tot_ms / 1e9:.1f} TFLOP/s avg)")
    for k, a in sorted(agg.items(), key=lambda kv: -kv[1]["ms"]):
        ms = a["ms"] / steps
        print(f"{str(k):60s} n={a['launches'] // steps:3d} {ms:8.3f} ms  {a['flops'] / a['ms'] / 1e9:7.1f} TF/s")


if __name__ == "__main__":
    main()
