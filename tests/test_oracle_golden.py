"""The CPU oracle against golden vectors produced by the reference itself
(tests/golden/make_golden.py).  These pin the oracle before it is trusted as
the checker of the HIP path."""
import pytest
import torch

import os

from helpers import REN_CFG, build_modules, check_grad, fixture, load_pretrained_sdf, named_params, oracle_params
from oracle import neus_oracle as O


def _render(fx, P, Pc, var):
    return O.render(P, Pc, var, fx["rays_o"], fx["rays_d"], fx["rays_d_norm"], fx["t"], fx["near"], fx["far"],
                    n_samples=REN_CFG["n_samples"], n_importance=REN_CFG["n_importance"],
                    up_steps=REN_CFG["up_sample_steps"], car=float(fx["car"]), t_rand=fx["t_rand"],
                    eval_mode=bool(fx["eval"]))


@pytest.mark.parametrize("name", ["render_small_train", "render_small_eval", "render_full_train"])
def test_seeded_modules_match_reference_weights(name):
    fx = fixture(name)
    mods = build_modules(int(fx["seed"]), int(fx["dh_sdf"]), int(fx["dh_col"]))
    for k, p in named_params(*mods):
        assert torch.allclose(p.detach().double().sum(), fx["psum." + k].double(), rtol=1e-5, atol=1e-5), k
        assert torch.allclose((p.detach().double() ** 2).sum(), fx["psq." + k].double(), rtol=1e-5), k


@pytest.mark.parametrize("name", ["render_small_train", "render_small_eval", "render_full_train"])
def test_oracle_render_matches_reference(name):
    fx = fixture(name)
    torch.set_num_threads(4)
    mods = build_modules(int(fx["seed"]), int(fx["dh_sdf"]), int(fx["dh_col"]))
    P, Pc, var, leaves = oracle_params(*mods)
    out = _render(fx, P, Pc, var)
    torch.testing.assert_close(out["z_vals"], fx["z_vals"], rtol=0, atol=1e-6)
    for k in ("color_fine", "depth_pred", "weights", "sdf", "normals", "sdf_flows", "cdf_fine", "s_val",
              "sampled_points"):
        torch.testing.assert_close(out[k].detach(), fx["out_" + k], rtol=1e-5, atol=1e-6, msg=lambda m: f"{k}: {m}")
    if not bool(fx["eval"]):
        loss = O.train_loss(out, fx["rgb_gt"])
        torch.testing.assert_close(loss.detach(), fx["loss"], rtol=1e-6, atol=1e-7)
        names = list(leaves)
        grads = torch.autograd.grad(loss, [leaves[n] for n in names])
        for n, g in zip(names, grads):
            check_grad(n, g, fx, rtol=1e-4, atol=1e-6)


def test_oracle_up_sample_matches_reference():
    fx = fixture("seams")
    for n in (64, 80, 96, 112):
        nz = O.up_sample(fx[f"up{n}_z"], fx[f"up{n}_sdf"], 16, float(fx[f"up{n}_invs"]))
        torch.testing.assert_close(nz, fx[f"up{n}_new"], rtol=0, atol=1e-6)
        zc, _ = O.cat_z_vals(fx[f"up{n}_z"], nz, None)
        torch.testing.assert_close(zc, fx[f"up{n}_cat"], rtol=0, atol=1e-6)


def test_oracle_sdf_field_and_double_backward_match_reference():
    fx = fixture("seams")
    sdf, col, dev = build_modules(7)
    P, Pc, var, leaves = oracle_params(sdf, col, dev)
    x = fx["mlp_x"]
    out = O.sdf_mlp(P, x)
    g = O.sdf_gradient(P, x)
    torch.testing.assert_close(out[:, :1].detach(), fx["mlp_sdf"], rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(out[:, 1:].detach(), fx["mlp_feat"], rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(g.detach(), fx["mlp_grad"], rtol=1e-4, atol=1e-5)
    L = (fx["mlp_a"] * out[:, :1]).sum() + (fx["mlp_B"] * out[:, 1:]).sum() + (fx["mlp_C"] * g).sum()
    names = [n for n in leaves if n.startswith("sdf.")]
    grads = torch.autograd.grad(L, [leaves[n] for n in names])
    for n, gr in zip(names, grads):
        check_grad("mlp." + n[4:], gr, fx, rtol=1e-4, atol=1e-5)


def test_oracle_color_field_matches_reference():
    fx = fixture("seams")
    sdf, col, dev = build_modules(7)
    P, Pc, var, leaves = oracle_params(sdf, col, dev)
    feat = fx["col_feat"].clone().requires_grad_(True)
    gg = fx["col_g"].clone().requires_grad_(True)
    rgb = O.color_mlp(Pc, fx["col_pts"], gg, fx["col_dirs"], feat)
    torch.testing.assert_close(rgb.detach(), fx["col_rgb"], rtol=1e-5, atol=1e-6)
    names = [n for n in leaves if n.startswith("col.")]
    grads = torch.autograd.grad((fx["col_D"] * rgb).sum(), [leaves[n] for n in names] + [feat, gg])
    for n, gr in zip(names, grads[:-2]):
        check_grad("colnet." + n[4:], gr, fx, rtol=1e-4, atol=1e-6)
    torch.testing.assert_close(grads[-2], fx["col_dfeat"], rtol=1e-4, atol=1e-6)
    torch.testing.assert_close(grads[-1], fx["col_dg"], rtol=1e-4, atol=1e-6)


def test_oracle_matches_reference_with_pretrained_sdf():
    """A trained surface (the reference's pretrained_sdf/model.pt, weights carried by
    the fixture), rendered from the origin with near/far 0.01/5.0."""
    fx = fixture("render_pretrained")
    torch.set_num_threads(8)
    sdf, col, dev = build_modules(int(fx["seed"]))
    load_pretrained_sdf(sdf, fx)
    P, Pc, var, leaves = oracle_params(sdf, col, dev)
    out = _render(fx, P, Pc, var)
    torch.testing.assert_close(out["z_vals"], fx["z_vals"], rtol=0, atol=1e-5)
    for k in ("color_fine", "depth_pred", "weights", "sdf", "normals"):
        torch.testing.assert_close(out[k].detach(), fx["out_" + k], rtol=1e-4, atol=1e-5, msg=lambda m: f"{k}: {m}")
    loss = O.train_loss(out, fx["rgb_gt"])
    torch.testing.assert_close(loss.detach(), fx["loss"], rtol=1e-5, atol=1e-6)


def test_checkpoint_keys_match_reference_pretrained_sdf():
    """State-dict compatibility (§8(f) rank 3): the reference's checkpoint loads
    strictly into the build's SDFNetwork, from the fixture and, when the reference
    checkout is present (this container only), from the file itself (weights_only)."""
    sdf, col, dev = build_modules(690)
    load_pretrained_sdf(sdf, fixture("render_pretrained"))
    path = "/root/reference/pretrained_sdf/model.pt"
    if os.path.exists(path):
        sd = torch.load(path, map_location="cpu", weights_only=True)
        sdf.load_state_dict(sd, strict=True)
        for k, v in sd.items():
            assert torch.equal(sdf.state_dict()[k], v), k
    from copenerf import NeuSRenderer
    from copenerf.motion import MotionNetwork
    from copenerf.train_step import MOTION_CFG
    r = NeuSRenderer(None, sdf, dev, col, MotionNetwork(**MOTION_CFG), **REN_CFG)
    keys = set(r.state_dict())
    for prefix in ("sdf_network.lin0.weight_g", "color_network.lin0.weight_v", "deviation_network.variance",
                   "motion_network.lin0.bias"):
        assert prefix in keys, prefix
