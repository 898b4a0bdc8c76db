"""The oracle's stage-1 losses (oracle.stage1_losses: scene-flow SDF loss, flow-RGB warp,
SDF consistency at the world camera) against tests/golden/stage1.npz, which
tests/golden/make_golden.py wrote by executing the reference's own stage-1 block of
train.py (467-517) and warp_pixel (235-244): losses and their gradients with respect to
the renderer outputs the block reads, the motion network and the SDF network, for frames
before / at / after the world camera and the last frame, reference intervals (1, 2, 3)
and (1, 5, 10), with and without sdf_consistency_enable_pose_grad.  CPU only."""
import os

import numpy as np
import pytest
import torch

from helpers import check_grad
from oracle import neus_oracle as O

FX = os.path.join(os.path.dirname(__file__), "golden", "stage1.npz")
CASES = ("before", "world", "after", "last", "iv1510", "posegrad_before", "posegrad_after")


def _fixture():
    d = np.load(FX)
    return {k: torch.from_numpy(d[k]) for k in d.files}


def _nets(fx):
    from copenerf.fields import SDFNetwork
    from copenerf.motion import MotionNetwork
    from copenerf.train_step import MOTION_CFG, SDF_CFG
    motion = MotionNetwork(**MOTION_CFG)
    motion.load_state_dict({k[7:]: v for k, v in fx.items() if k.startswith("motion.")}, strict=True)
    sdf = SDFNetwork(**dict(SDF_CFG, d_hidden=64))
    sdf.load_state_dict({k[7:]: v for k, v in fx.items() if k.startswith("sdfnet.")}, strict=True)
    leaves, W, b = {}, [], []
    for l in range(sdf.num_layers - 1):
        lin = getattr(sdf, f"lin{l}")
        for nm in ("weight_g", "weight_v", "bias"):
            leaves[f"lin{l}.{nm}"] = getattr(lin, nm).detach().clone().requires_grad_(True)
        W.append(torch._weight_norm(leaves[f"lin{l}.weight_v"], leaves[f"lin{l}.weight_g"], 0))
        b.append(leaves[f"lin{l}.bias"])
    P = O.SDFParams(W, b, skip=sdf.skip_in[0], multires=sdf.multires, scale=sdf.scale)
    return motion, P, leaves


@pytest.mark.parametrize("case", CASES)
def test_stage1_losses_match_reference_block(case):
    fx = _fixture()
    motion, P, sdf_leaves = _nets(fx)
    c = case + "."
    n, world, H, W = int(fx["n_images"]), int(fx["world"]), int(fx["H"]), int(fx["W"])
    out = {k: fx[c + "in." + k].clone().requires_grad_(k != "sampled_points")
           for k in ("sampled_points", "weights", "normals", "sdf_flows", "sdf")}
    intervals = tuple(int(j) for j in fx[c + "intervals"])
    l_sdf, l_flow, l_cons = O.stage1_losses(
        out, motion, lambda x: O.sdf_mlp(P, x)[:, :1], image_idx=int(fx[c + "image"]), n_images=n,
        world_cam_idx=world, nb_sample_timestep=10, rgb_gt=fx[c + "rgb_gt"], sampled_pixel=fx[c + "pix"],
        normalized_pixel=fx[c + "pixn"], camera_mats=fx["K"].expand(n, 4, 4), ref_images=fx["frames"],
        scale_mat=torch.eye(4)[None], img_hw=(H, W), ref_intervals=intervals,
        consistency_pose_grad=bool(int(fx[c + "pose_grad"])))
    for name, got in (("sdf_loss", l_sdf), ("flow_rgb_loss", l_flow), ("sdf_consistency_loss", l_cons)):
        ref = fx[c + name].item()
        assert abs(float(got) - ref) <= 1e-6 * abs(ref) + 1e-8, (name, float(got), ref)
    total = 0.1 * l_sdf + 7.5 * l_flow + 0.3 * l_cons
    wrt = ([("out." + k, v) for k, v in out.items() if v.requires_grad] +
           [("motion." + k, p) for k, p in motion.named_parameters()] +
           [("sdfnet." + k, v) for k, v in sdf_leaves.items()])
    grads = torch.autograd.grad(total, [v for _, v in wrt], allow_unused=True)
    checked = 0
    for (k, v), g in zip(wrt, grads):
        key = c + k
        if ("grad." + key) in fx and fx["grad." + key].numel() == 0:  # no gradient in the reference
            assert g is None or not g.any(), key
            continue
        assert g is not None, key
        scale = (fx["grad." + key] if "grad." + key in fx else fx["gradval." + key]).abs().max().item()
        check_grad(key, g, fx, rtol=1e-5, atol=1e-6 * scale + 1e-12)
        checked += 1
    assert checked > 10
    if case == "world":
        assert float(l_cons) == 0.0
    if case == "last":
        assert float(l_flow) == 0.0
    if case.startswith("posegrad"):  # the consistency term reaches the motion network
        mg = grads[[k for k, _ in wrt].index("motion.lin0.weight_v")]
        assert mg is not None and mg.abs().max() > 0
