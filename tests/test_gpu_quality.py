"""Training quality of the bf16 mode (config C3, "bf16 MLP MFMA") over many steps.

SURVEY.md §7: C3 cannot meet the fp32 1e-4 bar and is judged by loss / PSNR, the numbers the
reference reports (eval.py:190-221).  Here the C3 workload of bench.py (Co3D/skateboard stage 1:
MotionNetwork, scene-flow SDF loss, flow-RGB warp, SDF consistency with pose gradient; 4096 rays x
128 samples) trains for STEPS steps from the same seed twice -- bf16 MFMA operands with the
operand images, and the fp32-class bf16x6 GEMMs -- on a scene with a learnable surface: a camera at
the centre of a textured spherical room (radius 1; the indoor-scene initialisation, inside_outside,
starts the SDF as a room of radius 0.5), ten identical frames (a static camera: the motion network
should stay still).  Each mode runs over six sample streams; every run must have learned the scene
and the modes' mean final photometric loss and mean PSNR of a held-out eval render must agree within
the stated tolerances (PSNR 12.1 dB at the start; see the tolerances below for the measured runs).
COPENERF_QUALITY_LOG receives the loss curves (profiles/r5_bf16_quality.json)."""
import json
import math
import os

import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"
STEPS = 1000
ROOM_RADIUS = 1.0
EVAL_HW = (135, 240)
# Tolerances between the modes (bf16 vs bf16x6) from the round-6 attribution sweep over these six sample streams
# (profiles/r6_bf16_quality_sweep.json, tools/quality_sweep.py): eval PSNR bf16 30.5 / 31.1 / 35.3 / 37.8 /
# 38.4 / 33.5, bf16x6 42.3 / 36.4 / 35.9 / 38.1 / 31.4 / 35.5 dB -- paired differences -11.8 .. +7.0 (training
# is chaotic: bf16x6 runs among themselves span 31.4 .. 42.3) -- means 34.4 vs 36.6: a 2.15 dB gap, so
# PSNR_TOL_DB = 2.15 + 1.35 dB of margin; photometric loss (L1 rgb, mean of the last 100 steps) means 0.0111 vs
# 0.0101 (ratio 1.10): L1_RATIO_TOL = 1.10 + 0.15; every run gains >= 18.4 dB over the initial 12.1 --
# MIN_PSNR_GAIN_DB.  The runs are bitwise reproducible for a build, so these bars hold exactly for this one; a
# change to any GEMM's summation order re-draws every stream (the six-stream mean moves by ~2.7 dB std), and
# a failure after such a change calls for a wider sweep (tools/quality_sweep.py --seeds ...), not a wider bar.
# The sweep's attribution arms: sigma recovered from an fp32 copy of the activation 35.3 dB mean (images stay
# the GEMM operands), no operand images at all 32.8 dB (L1 0.0180) -- the operand images do not cost quality.
L1_RATIO_TOL = 1.25
PSNR_TOL_DB = 3.5
MIN_PSNR_GAIN_DB = 15.0


def room_texture(d):
    """Colour of the room wall in unit direction d [..., 3] (smooth: about 1.5 periods across the view)."""
    ph = torch.tensor([0.3, 1.9, 4.1], device=d.device)
    return 0.5 + 0.35 * torch.sin(6.0 * d[..., 0:1] + 4.0 * d[..., 1:2] + 2.0 * d[..., 2:3] + ph)


def room_image(K, H, W):
    """The frame of a camera at the room's centre with the identity pose: [3, H, W]."""
    from copenerf.rays import world_rays
    ys, xs = torch.meshgrid(torch.arange(H, device=DEV), torch.arange(W, device=DEV), indexing="ij")
    pixn = torch.stack([2.0 * xs.flatten().float() / (W - 1) - 1.0, 2.0 * ys.flatten().float() / (H - 1) - 1.0], -1)
    I = torch.eye(4, device=DEV)
    _, d, _ = world_rays(pixn, K, I, I)
    return room_texture(d).t().reshape(3, H, W).contiguous()


def _train(mode, sample_seed=None):
    from bench import C3_TRAIN
    from copenerf.inference import render_image
    from copenerf.train_step import SDF_CFG, SyntheticTrainer
    tr = SyntheticTrainer(DEV, rays=4096, stage1=True, mfma_dtype=mode, start_it=30000, train_cfg=dict(C3_TRAIN),
                          sdf_cfg=dict(SDF_CFG, inside_outside=True), depth_range=(0.01, 3.0), seed=678)
    if sample_seed is not None:  # same initial weights and frames, other patches and jitter
        tr.gen.manual_seed(sample_seed)
    tr.images = room_image(tr.K, tr.H, tr.W).expand(tr.n_images, 3, tr.H, tr.W).contiguous()
    target = room_image(tr.K, *EVAL_HW)
    t0 = torch.full((1,), -1.0, device=DEV)  # frame 0's time step

    def psnr():
        with torch.no_grad():
            out = render_image(tr.renderer, tr.K, tr.I, tr.I, EVAL_HW, t0, depth_range=(0.01, 3.0), chunk=32400)
        rgb = out["rgb"].reshape(*EVAL_HW, 3).permute(2, 0, 1)
        return -10.0 * math.log10(((rgb - target) ** 2).mean().item())

    p0 = psnr()
    losses, l1s = [], []
    for _ in range(STEPS):
        tr.begin_iteration()
        batch = tr.make_batch()
        loss, out = tr.iteration(batch, return_out=True)
        losses.append(loss.detach())
        l1s.append((out["color_fine"].detach() - batch["rgb_gt"]).abs().mean())  # the photometric (L1 rgb) term
        del out
    tr.check_finite()
    losses, l1s = torch.stack(losses).float().cpu(), torch.stack(l1s).float().cpu()
    return {"mode": mode, "sample_seed": sample_seed, "psnr_init": p0, "psnr": psnr(),
            "l1_final": l1s[-100:].mean().item(), "loss_final": losses[-100:].mean().item(),
            "l1_curve": [round(v, 5) for v in l1s.view(-1, 50).mean(1).tolist()],
            "loss_curve": [round(v, 5) for v in losses.view(-1, 50).mean(1).tolist()]}


SEEDS = [None, 12345, 777, 4242, 31337, 9001]  # the trainer's own sample stream, then others (same weights and frames)
RUNS = {}


@pytest.mark.parametrize("mode,seed", [(m, sd) for sd in SEEDS for m in ("bf16", "bf16x6")])
def test_quality_run(mode, seed):
    """One 1000-step training run (17 s bf16, 38 s bf16x6): it learns the room."""
    r = _train(mode, seed)
    RUNS[(mode, seed)] = r
    print(json.dumps({k: v for k, v in r.items() if not k.endswith("_curve")}))
    assert r["psnr"] - r["psnr_init"] >= MIN_PSNR_GAIN_DB, r["psnr"]


def test_bf16_training_tracks_fp32_class_training():
    """bf16 and bf16x6 from the same weights over the same six sample streams (training is chaotic: one
    stream's pair can differ by as much as two fp32-class streams, so the modes are compared on means)."""
    if len(RUNS) != 2 * len(SEEDS):
        pytest.skip("the runs did not all complete")
    mean = lambda mode, k: sum(RUNS[(mode, sd)][k] for sd in SEEDS) / len(SEEDS)  # noqa: E731
    summary = {f"{m}/{sd}": {k: v for k, v in RUNS[(m, sd)].items() if not k.endswith("_curve")}
               for (m, sd) in RUNS}
    print(json.dumps(summary))
    logp = os.environ.get("COPENERF_QUALITY_LOG")
    if logp:
        with open(logp, "w") as f:
            json.dump({"steps": STEPS, "rays": 4096, "workload": "c3 (skateboard stage 1) on the textured room",
                       "tolerances": {"l1_ratio": L1_RATIO_TOL, "psnr_db": PSNR_TOL_DB, "min_gain_db": MIN_PSNR_GAIN_DB},
                       "runs": {f"{m}/{sd}": r for (m, sd), r in RUNS.items()}}, f)
    lb, lx = mean("bf16", "l1_final"), mean("bf16x6", "l1_final")
    assert lb <= L1_RATIO_TOL * lx and lx <= L1_RATIO_TOL * lb, summary
    assert abs(mean("bf16", "psnr") - mean("bf16x6", "psnr")) <= PSNR_TOL_DB, summary
