"""End-to-end NeuSRenderer on the HIP path against the reference's golden
vectors (tests/golden) and against the CPU oracle at larger ray counts.
Tolerance (BASELINE.json north_star): rendered RGB / depth |Δ| <= 1e-4 in fp32."""
import pytest
import torch

from helpers import REN_CFG, build_modules, check_grad, fixture, named_params, oracle_params
from oracle import neus_oracle as O

pytestmark = pytest.mark.gpu
DEV = "cuda"
TOL_RGB_DEPTH = 1e-4


def _renderer(mods):
    from copenerf import NeuSRenderer
    sdf, col, dev = mods
    return NeuSRenderer(None, sdf, dev, col, None, **REN_CFG).to(DEV)


def _run(r, fx):
    g = lambda k: fx[k].to(DEV)  # noqa: E731
    return r(g("rays_o"), g("rays_d"), g("rays_d_norm"), g("t"), g("near"), g("far"),
             cos_anneal_ratio=float(fx["car"]), it=0, eval=bool(fx["eval"]), t_rand=g("t_rand"))


@pytest.mark.parametrize("name", ["render_small_train", "render_small_eval", "render_full_train"])
def test_render_matches_reference_golden(name):
    fx = fixture(name)
    mods = build_modules(int(fx["seed"]), int(fx["dh_sdf"]), int(fx["dh_col"]), device=DEV)
    r = _renderer(mods)
    out = _run(r, fx)
    for k in ("color_fine", "depth_pred"):
        err = (out[k].detach().cpu() - fx["out_" + k]).abs().max().item()
        assert err <= TOL_RGB_DEPTH, (k, err)
    S = fx["z_vals"].shape[1]
    assert out["weights"].shape[1] == S
    # Per-sample quantities: importance-sample positions come from a searchsorted on
    # the SDF-derived cdf, so GEMM summation-order differences move a few samples
    # (fp32-vs-fp64 reference moves 0.56 % of samples > 1e-4).  Require
    # 99 % of entries within 1e-4 and every entry within 2e-3; RGB/depth above are strict.
    for k, tol in (("weights", 1e-4), ("sdf", 1e-4), ("normals", 1e-3), ("sampled_points", 1e-4)):
        a, b = out[k].detach().cpu(), fx["out_" + k]
        diff = (a - b).abs()
        assert (diff <= tol + 1e-3 * b.abs()).float().mean().item() >= 0.99, (k, diff.max().item())
        assert diff.max().item() <= 2e-3 + 2e-3 * b.abs().max().item(), (k, diff.max().item())
    if not bool(fx["eval"]):
        loss = O.train_loss({k: v for k, v in out.items()}, fx["rgb_gt"].to(DEV))
        assert abs(loss.item() - fx["loss"].item()) <= 1e-4 * abs(fx["loss"].item()) + 1e-5
        params = named_params(*mods)
        grads = torch.autograd.grad(loss, [p for _, p in params])
        for (n, _), gr in zip(params, grads):
            check_grad(n, gr, fx, rtol=2e-2, atol=2e-4 * (gr.abs().max().item() + 1e-3))


@pytest.mark.parametrize("R,dh", [(256, 256), (1024, 256)])
def test_render_matches_oracle(R, dh):
    g = torch.Generator().manual_seed(R)
    mods_cpu = build_modules(55, dh, dh)
    P, Pc, var, leaves = oracle_params(*mods_cpu)
    o = torch.tensor([0.05, -0.03, 1.6]).expand(R, 3).contiguous()
    d = torch.cat([(torch.rand(R, 2, generator=g) - 0.5) * 0.6, -torch.ones(R, 1)], -1)
    nrm = d.norm(dim=-1, keepdim=True)
    d = d / nrm
    t = torch.tensor([0.25])
    near, far = torch.full((R, 1), 0.01), torch.full((R, 1), 3.0)
    t_rand = torch.rand(R, 64, generator=g)
    torch.set_num_threads(8)
    ref = O.render(P, Pc, var, o, d, nrm, t, near, far, car=0.5, t_rand=t_rand)
    mods = build_modules(55, dh, dh, device=DEV)
    r = _renderer(mods)
    out = r(o.to(DEV), d.to(DEV), nrm.to(DEV), t.to(DEV), near.to(DEV), far.to(DEV), cos_anneal_ratio=0.5, it=0,
            eval=False, t_rand=t_rand.to(DEV))
    for k in ("color_fine", "depth_pred"):
        err = (out[k].detach().cpu() - ref[k].detach()).abs().max().item()
        assert err <= TOL_RGB_DEPTH, (k, err)


def test_render_large_batch_properties():
    """C2 size (4096 rays x 128 samples): invariants that need no oracle."""
    R = 4096
    mods = build_modules(56, device=DEV)
    r = _renderer(mods)
    g = torch.Generator(device=DEV).manual_seed(3)
    o = torch.tensor([0.05, -0.03, 1.6], device=DEV).expand(R, 3).contiguous()
    d = torch.cat([(torch.rand(R, 2, device=DEV, generator=g) - 0.5) * 0.6, -torch.ones(R, 1, device=DEV)], -1)
    nrm = d.norm(dim=-1, keepdim=True)
    d = d / nrm
    args = (o, d, nrm, torch.tensor([0.0], device=DEV), torch.full((R, 1), 0.01, device=DEV),
            torch.full((R, 1), 3.0, device=DEV))
    t_rand = torch.rand(R, 64, device=DEV, generator=g)
    out1 = r(*args, cos_anneal_ratio=0.5, it=0, eval=False, t_rand=t_rand)
    out2 = r(*args, cos_anneal_ratio=0.5, it=0, eval=False, t_rand=t_rand)
    for k in ("color_fine", "depth_pred", "weights", "normals"):
        assert torch.isfinite(out1[k]).all(), k
        assert torch.equal(out1[k], out2[k]), k  # deterministic (no atomics on the path)
    w = out1["weights"]
    assert w.shape == (R, 128)
    assert (w >= 0).all() and (w.sum(-1) <= 1 + 1e-5).all()
    pts = out1["sampled_points"]
    zz = ((pts - o[:, None, :]) * d[:, None, :]).sum(-1)
    assert (zz[:, 1:] >= zz[:, :-1] - 1e-5).all()  # samples sorted along each ray
    loss = O.train_loss(out1, torch.rand(R, 3, device=DEV, generator=g))
    loss.backward()
    for n, p in named_params(*mods):
        assert p.grad is not None and torch.isfinite(p.grad).all(), n
