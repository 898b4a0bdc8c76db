"""Ray / pose gradients (eval.py:51-82 test-pose optimisation and joint pose
training): d loss / d rays_o, d rays_d through the HIP backward against the CPU
oracle's autograd on identical sample positions.  The ∇ₓSDF pass runs on
detached points in the reference (neus_renderer.py:356), so the oracle's
sdf_gradient detaches too and the gradients reach the rays through the SDF
forward, the colour network (points and view directions) and true_cos."""
import pytest
import torch

from helpers import REN_CFG, build_modules, named_params, oracle_params
from oracle import neus_oracle as O

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _renderer(mods):
    from copenerf import NeuSRenderer
    sdf, col, dev = mods
    return NeuSRenderer(None, sdf, dev, col, None, **REN_CFG).to(DEV)


def _case(R, seed=55):
    g = torch.Generator().manual_seed(1000 + R)
    mods_cpu = build_modules(seed, 256, 256)
    P, Pc, var, _ = oracle_params(*mods_cpu)
    o = torch.tensor([0.05, -0.03, 1.6]).expand(R, 3).contiguous() + 0.01 * torch.randn(R, 3, generator=g)
    d = torch.cat([(torch.rand(R, 2, generator=g) - 0.5) * 0.6, -torch.ones(R, 1)], -1)
    nrm = d.norm(dim=-1, keepdim=True)
    d = d / nrm
    t = torch.tensor([0.25])
    near, far = torch.full((R, 1), 0.01), torch.full((R, 1), 3.0)
    t_rand = torch.rand(R, 64, generator=g)
    gt = torch.rand(R, 3, generator=g)
    torch.set_num_threads(8)
    z = O.hierarchical_z(P, o, d, t, near, far, 64, 64, 4, t_rand)
    o_, d_ = o.clone().requires_grad_(True), d.clone().requires_grad_(True)
    ref = O.render_core(P, Pc, var, o_, d_, nrm, t, z, (far[0, 0] - near[0, 0]) / 64, 0.5)
    go, gd = torch.autograd.grad(O.train_loss(ref, gt), [o_, d_])
    return (o, d, nrm, t, near, far, z, gt), (go, gd)


def _close(got, ref, name):
    scale = ref.abs().max().item()
    err = (got.detach().cpu() - ref).abs()
    assert err.max().item() <= 2e-3 * scale + 1e-6, (name, err.max().item(), scale)
    assert (err / (ref.abs() + 1e-2 * scale)).mean().item() <= 1e-3, name


@pytest.mark.parametrize("frozen", [False, True])
def test_ray_gradients_match_oracle_on_identical_samples(frozen):
    R = 256
    (o, d, nrm, t, near, far, z, gt), (go, gd) = _case(R)
    mods = build_modules(55, 256, 256, device=DEV)
    if frozen:  # eval.py pose optimisation: networks frozen, only the rays carry gradients
        for m in mods:
            m.requires_grad_(False)
    r = _renderer(mods)
    og, dg = o.to(DEV).requires_grad_(True), d.to(DEV).requires_grad_(True)
    out = r(og, dg, nrm.to(DEV), t.to(DEV), near.to(DEV), far.to(DEV), cos_anneal_ratio=0.5, it=0, eval=False,
            z_vals=z.to(DEV))
    loss = O.train_loss(out, gt.to(DEV))
    if frozen:
        ho, hd = torch.autograd.grad(loss, [og, dg])
    else:  # joint pose training: parameter and ray gradients in one backward
        loss.backward()
        ho, hd = og.grad, dg.grad
        for n, p in named_params(*mods):
            assert p.grad is not None and torch.isfinite(p.grad).all(), n
    _close(ho, go, "rays_o")
    _close(hd, gd, "rays_d")
