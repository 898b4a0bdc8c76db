"""Shared test helpers: fixtures, seeded modules, oracle parameters."""
from __future__ import annotations

import os

import numpy as np
import torch

from oracle import neus_oracle as O

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")

SDF_CFG = dict(d_in=4, d_out=257, d_hidden=256, n_layers=8, skip_in=[4], multires=6, bias=0.5, scale=1.0,
               geometric_init=True, weight_norm=True)
COL_CFG = dict(d_feature=256, mode="idr", d_in=11, d_out=3, d_hidden=256, n_layers=4, weight_norm=True,
               multires_view=4, squeeze_out=True, use_negative_ray_vector=False)
REN_CFG = dict(n_samples=64, n_importance=64, n_outside=0, up_sample_steps=4, perturb=1.0,
               n_max_network_queries=64000, importance_sampling_start=0, naive_render=False)


def fixture(name):
    with np.load(os.path.join(GOLDEN, name + ".npz")) as f:
        return {k: torch.from_numpy(f[k]) if f[k].ndim else torch.tensor(f[k]) for k in f.files}


def build_modules(seed, dh_sdf=256, dh_col=256, var=0.3, device="cpu"):
    """The copenerf modules, seeded exactly like tests/golden/make_golden.py builds the reference's."""
    from copenerf.fields import RenderingNetwork, SDFNetwork, SingleVarianceNetwork
    torch.manual_seed(seed)
    sdf = SDFNetwork(**dict(SDF_CFG, d_hidden=dh_sdf))
    col = RenderingNetwork(**dict(COL_CFG, d_hidden=dh_col))
    dev = SingleVarianceNetwork(var)
    return sdf.to(device), col.to(device), dev.to(device)


def named_params(sdf, col, dev):
    return ([("sdf." + k, p) for k, p in sdf.named_parameters()] +
            [("col." + k, p) for k, p in col.named_parameters()] + [("dev.variance", dev.variance)])


def oracle_params(sdf, col, dev):
    """Oracle parameters on the CPU whose effective weights are built from (g, v)
    leaves, so gradients come back in the reference's parameterisation."""
    leaves = {}

    def eff(mod, prefix):
        W, b = [], []
        for l in range(mod.num_layers - 1):
            lin = getattr(mod, f"lin{l}")
            g = lin.weight_g.detach().cpu().clone().requires_grad_(True)
            v = lin.weight_v.detach().cpu().clone().requires_grad_(True)
            bb = lin.bias.detach().cpu().clone().requires_grad_(True)
            leaves[f"{prefix}lin{l}.weight_g"] = g
            leaves[f"{prefix}lin{l}.weight_v"] = v
            leaves[f"{prefix}lin{l}.bias"] = bb
            W.append(torch._weight_norm(v, g, 0))
            b.append(bb)
        return W, b

    W, b = eff(sdf, "sdf.")
    P = O.SDFParams(W, b, skip=sdf.skip_in[0], multires=sdf.multires, scale=sdf.scale)
    Wc, bc = eff(col, "col.")
    Pc = O.ColorParams(Wc, bc, multires_view=col.multires_view)
    var = dev.variance.detach().cpu().clone().requires_grad_(True)
    leaves["dev.variance"] = var
    return P, Pc, var, leaves


def check_grad(name, got, fx, rtol, atol):
    """Compare a gradient with a fixture entry (full or sampled)."""
    got = got.detach().cpu().float()
    if "grad." + name in fx:
        ref = fx["grad." + name].float()
        torch.testing.assert_close(got, ref, rtol=rtol, atol=atol, msg=lambda m: f"{name}: {m}")
    else:
        idx = fx["gradidx." + name].long()
        torch.testing.assert_close(got.reshape(-1)[idx], fx["gradval." + name].float(), rtol=rtol, atol=atol,
                                   msg=lambda m: f"{name} (sampled): {m}")
        n = fx["gradnorm." + name].float()
        assert abs(got.norm().item() - n.item()) <= rtol * n.item() + atol, (name, got.norm().item(), n.item())


def load_pretrained_sdf(sdf, fx):
    """Load the reference's pretrained SDF weights carried by a fixture (sdfw.*)
    into an SDFNetwork with strict key matching (checkpoint compatibility)."""
    sd = {k[5:]: v for k, v in fx.items() if k.startswith("sdfw.")}
    sdf.load_state_dict({k: v.to(next(sdf.parameters()).device) for k, v in sd.items()}, strict=True)
    return sdf


def smooth_frames(n, H, W, device="cpu", seed=0):
    """n smooth (low-frequency) RGB frames in (0.1, 0.9): bilinear warps of them have a
    gradient that varies slowly across pixel boundaries, so the flow-RGB term
    (train.py:506-515, grid_sample) is well conditioned for gradient parity; on
    per-pixel noise a last-ulp change of a flow can cross a pixel edge and flip the
    warp's gradient (the bilinear derivative jumps there)."""
    g = torch.Generator().manual_seed(seed)
    f = torch.rand(n, 3, 2, generator=g) * 2.0 + 0.5     # cycles per frame
    ph = torch.rand(n, 3, generator=g) * 6.28
    y = torch.linspace(0, 1, H).view(1, 1, H, 1)
    x = torch.linspace(0, 1, W).view(1, 1, 1, W)
    arg = 6.2831853 * (f[..., 0, None, None] * x + f[..., 1, None, None] * y) + ph[..., None, None]
    return (0.5 + 0.4 * torch.sin(arg)).float().to(device)
