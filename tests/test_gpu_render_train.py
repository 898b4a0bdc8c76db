"""cn_render_train_fwd / cn_render_bwd (ABI v14): render_core under autograd (neus_renderer.py:307-450) as two C
calls -- the points, the SDF field with ∇ₓSDF, the colour network with the folded feature head, the compositing,
and the backward of all of them with autograd's gradient sums between the pieces -- against copenerf's
composition of the same kernels (_PointsFn, _SDFFieldFn, _ColorFieldFn, _CompositeFn: RENDER_NATIVE off):
every output and every gradient (both networks' parameters through weight norm and the fold, the variance, the
rays' pose gradient) bitwise equal in each GEMM mode, with and without the pose gradient and with upstream
gradients on every output; and whole training steps (C2's and C3's workloads at a small batch) bitwise equal.
The composition is pinned to the reference by the golden tests (test_gpu_render.py and the stage-1 tests)."""
import pytest
import torch

from helpers import REN_CFG, build_modules

pytestmark = pytest.mark.gpu
DEV = "cuda"
MODES = ["fp32", "bf16x6", "bf16"]
KEYS = ["color_fine", "depth_pred", "weights", "cdf_fine", "sdf", "normals", "sdf_flows", "sampled_points"]


def _run(native, mode, pose, seed=3, R=384):
    from copenerf import NeuSRenderer, ops
    from copenerf import renderer as rmod
    saved = rmod.RENDER_NATIVE
    rmod.RENDER_NATIVE = native
    calls = []
    fwd = ops.render_train_fwd
    ops.render_train_fwd = lambda *a, **k: calls.append(1) or fwd(*a, **k)
    try:
        sdf, col, dev = build_modules(seed, device=DEV)
        r = NeuSRenderer(None, sdf, dev, col, None, **REN_CFG).to(DEV).set_mfma_dtype(mode)
        gen = torch.Generator(device=DEV).manual_seed(seed)
        rays_o = ((torch.rand(R, 3, device=DEV, generator=gen) - 0.5) * 0.3).requires_grad_(pose)
        rays_d = torch.nn.functional.normalize(torch.randn(R, 3, device=DEV, generator=gen), dim=-1)
        rays_d = rays_d.requires_grad_(pose)
        nrm = torch.ones(R, 1, device=DEV)
        near = torch.full((R, 1), 0.1, device=DEV)
        far = torch.full((R, 1), 1.9, device=DEV)
        t = torch.full((1,), 0.4, device=DEV)
        t_rand = torch.rand(R, r.n_samples, device=DEV, generator=gen)
        out = r(rays_o, rays_d, nrm, t, near, far, cos_anneal_ratio=0.6, it=0, eval=False, t_rand=t_rand)
        # an upstream gradient on every differentiable output (fixed random weights)
        loss = 0.0
        for i, k in enumerate(KEYS):
            v = out[k]
            if not v.requires_grad:
                continue
            w = torch.randn(v.shape, device=DEV, generator=torch.Generator(device=DEV).manual_seed(100 + i))
            loss = loss + (v * w).sum()
        loss.backward()
        torch.cuda.synchronize()
        grads = {n: p.grad.clone() for n, p in list(r.named_parameters()) if p.grad is not None}
        if pose:
            grads["rays_o"], grads["rays_d"] = rays_o.grad.clone(), rays_d.grad.clone()
        return {k: out[k].detach().clone() for k in KEYS}, grads, len(calls)
    finally:
        rmod.RENDER_NATIVE = saved
        ops.render_train_fwd = fwd


@pytest.mark.parametrize("pose", [False, True])
@pytest.mark.parametrize("mode", MODES)
def test_render_train_equals_composition(mode, pose):
    out_c, g_c, n_c = _run(False, mode, pose)
    out_n, g_n, n_n = _run(True, mode, pose)
    assert n_c == 0 and n_n == 1  # the C calls ran (once), and only in the native run
    for k in KEYS:
        assert torch.equal(out_n[k], out_c[k]), k
    assert g_n.keys() == g_c.keys() and len(g_c) >= 30
    for k, v in g_c.items():
        assert torch.equal(g_n[k], v), (k, (g_n[k] - v).abs().max().item())


@pytest.mark.parametrize("R", [1, 3, 65])
def test_render_train_ragged_batches(R):
    """Ragged and tiny ray batches (one ray, a partial wave, a partial tile) with the pose gradient, bf16."""
    out_c, g_c, _ = _run(False, "bf16", True, seed=8, R=R)
    out_n, g_n, n_n = _run(True, "bf16", True, seed=8, R=R)
    assert n_n == 1
    for k in KEYS:
        assert torch.equal(out_n[k], out_c[k]), k
    for k, v in g_c.items():
        assert torch.equal(g_n[k], v), (k, (g_n[k] - v).abs().max().item())


@pytest.mark.parametrize("cfg", ["c2", "c3"])
def test_training_steps_equal_composition(cfg):
    """Two training steps of SyntheticTrainer (C2: fixed poses, fp32-class; C3: stage 1 with the motion network,
    joint pose and the consistency re-query, bf16) with and without the C calls: losses and every parameter
    bitwise equal."""
    from copenerf import renderer as rmod
    from copenerf.train_step import SyntheticTrainer
    kw = dict(rays=512, H=96, W=128, n_images=6, start_it=30000)
    kw.update(dict(mfma_dtype="bf16x6") if cfg == "c2" else dict(mfma_dtype="bf16", stage1=True, joint_pose=True))
    res = []
    saved = rmod.RENDER_NATIVE
    try:
        for native in (False, True):
            rmod.RENDER_NATIVE = native
            tr = SyntheticTrainer(DEV, **kw)
            losses = [tr.step().item() for _ in range(2)]
            res.append((losses, [p.detach().clone() for p in tr.all_params]))
    finally:
        rmod.RENDER_NATIVE = saved
    assert res[0][0] == res[1][0]
    for a, b in zip(res[0][1], res[1][1]):
        assert torch.equal(a, b)
