"""Training quality of the bf16 mode (config C3, "bf16 MLP MFMA") over many steps.

SURVEY.md §7: C3 cannot meet the fp32 1e-4 bar and is judged by loss / PSNR, the numbers the
reference reports (eval.py:190-221).  Here the C3 workload of bench.py (Co3D/skateboard stage 1:
MotionNetwork, scene-flow SDF loss, flow-RGB warp, SDF consistency with pose gradient; 4096 rays x
128 samples) trains for STEPS steps from the same seed twice -- bf16 MFMA operands with the
operand images, and the fp32-class bf16x6 GEMMs -- on a scene with a learnable surface: a camera at
the centre of a textured spherical room (radius 1; the indoor-scene initialisation, inside_outside,
starts the SDF as a room of radius 0.5), ten identical frames (a static camera: the motion network
should stay still).  The final photometric loss and the PSNR of a held-out eval render must agree
between the modes within the stated tolerances, and both must have learned the scene (a first run:
PSNR 12.1 dB at the start, 41.4 (bf16) and 36.6 dB (bf16x6) after 1000 steps).
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
# tolerances between the modes (bf16 vs bf16x6), from the measured runs (profiles/r5_bf16_quality.json):
# eval PSNR 41.4 (bf16) / 36.6 (bf16x6) / 40.9 dB (bf16x6, other patches): the two fp32-class runs differ
# by 4.3 dB, the modes by 4.8 -- PSNR_TOL_DB; the photometric loss (L1 rgb, mean of the last 100 steps)
# 0.0174 / 0.0086 / 0.0066: bf16's noise floor is ~2x the fp32-class one at 1000 steps -- L1_RATIO_TOL
L1_RATIO_TOL = 3.0
PSNR_TOL_DB = 6.0
MIN_PSNR_GAIN_DB = 20.0


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


def test_bf16_training_tracks_fp32_class_training():
    """bf16 and bf16x6 from the same seed; a second bf16x6 run with other patches / jitter (the seed
    spread: two fp32-class runs differ by about as much as the modes, training being chaotic)."""
    runs = {"bf16": _train("bf16"), "bf16x6": _train("bf16x6"), "bf16x6_seed2": _train("bf16x6", 12345)}
    b, x, x2 = runs["bf16"], runs["bf16x6"], runs["bf16x6_seed2"]
    summary = {m: {k: v for k, v in r.items() if not k.endswith("_curve")} for m, r in runs.items()}
    print(json.dumps(summary))
    logp = os.environ.get("COPENERF_QUALITY_LOG")
    if logp:
        with open(logp, "w") as f:
            json.dump({"steps": STEPS, "rays": 4096, "workload": "c3 (skateboard stage 1) on the textured room",
                       "tolerances": {"l1_ratio": L1_RATIO_TOL, "psnr_db": PSNR_TOL_DB}, "runs": runs}, f)
    for r in runs.values():
        assert r["psnr"] - r["psnr_init"] >= MIN_PSNR_GAIN_DB, summary
    assert b["l1_final"] <= L1_RATIO_TOL * max(x["l1_final"], x2["l1_final"]), summary
    assert x["l1_final"] <= L1_RATIO_TOL * b["l1_final"], summary
    assert abs(b["psnr"] - x["psnr"]) <= PSNR_TOL_DB, summary
