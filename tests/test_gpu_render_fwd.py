"""cn_render_fwd (ABI v13): the rendering forward of NeuSRenderer (neus_renderer.py:453-584, render_core
307-450) in one C call -- sampler, midpoints, SDF field with ∇ₓSDF, colour network with the folded feature
head, compositing -- against copenerf's renderer run with the same packs and inputs: the same launches
with the same descriptors, so every output bitwise equal, in each GEMM mode; and through the renderer to
the reference's own outputs (test_gpu_render holds those bars) by transitivity."""
import pytest
import torch

from helpers import REN_CFG, build_modules, fixture

pytestmark = pytest.mark.gpu
DEV = "cuda"
MODES = ["fp32", "bf16x6", "bf16"]


def _renderer(mods, mode):
    from copenerf import NeuSRenderer
    sdf, col, dev = mods
    return NeuSRenderer(None, sdf, dev, col, None, **REN_CFG).to(DEV).set_mfma_dtype(mode)


def _c_render(r, rays_o, rays_d, t, near, far, car, t_rand=None, z_in=None):
    from copenerf import ops
    sdf_packed = r.sdf_network.params_and_pack()
    col_packed = r.color_network.params_and_pack(fold_feature=(sdf_packed[0][-1], sdf_packed[1][-1]))
    sn, k1 = ops.sdf_net(r.sdf_network.layout(), sdf_packed[2])
    cn, k2 = ops.color_net(r.color_network.layout(), col_packed[2])
    inv_s = r.deviation_network(torch.zeros([1, 3], device=DEV))[:, :1].clip(1 / 1e3, 1 / 1e-3).contiguous()
    out = ops.render_fwd(sn, cn, rays_o, rays_d, near, far, t, inv_s, ops.device_scalar(car, DEV), r.n_samples,
                         r.n_importance, r.up_sample_steps, t_rand=t_rand, z_in=z_in)
    torch.cuda.synchronize()
    del k1, k2
    return out


def _python_forward(r, *args, **kw):
    """The renderer's launch-by-launch forward (RENDER_NATIVE off), the reference of the C call."""
    from copenerf import renderer as rmod
    saved = rmod.RENDER_NATIVE
    rmod.RENDER_NATIVE = False
    try:
        with torch.no_grad():
            return r(*args, **kw)
    finally:
        rmod.RENDER_NATIVE = saved


def _compare_dicts(a, b):
    for k, v in b.items():
        assert torch.equal(a[k], v), (k, (a[k] - v).abs().max().item() if a[k].shape == v.shape else a[k].shape)


def _compare(out, ref, R, S):
    pairs = [("color", ref["color_fine"]), ("weights", ref["weights"]), ("cdf", ref["cdf_fine"]),
             ("sdf", ref["sdf"].reshape(-1)), ("depth", ref["weighted_z_vals"].reshape(-1))]
    for k, v in pairs:
        assert torch.equal(out[k].reshape(v.shape), v), (k, (out[k].reshape(v.shape) - v).abs().max().item())
    assert torch.equal(out["grad"][:, :3].reshape(R, S, 3), ref["normals"])
    assert torch.equal(out["grad"][:, 3:].reshape(R, S, 1), ref["sdf_flows"])
    assert torch.equal(out["pts"][:, :3].reshape(R, S, 3), ref["sampled_points"])


@pytest.mark.parametrize("mode", MODES)
@pytest.mark.parametrize("name", ["render_small_eval", "render_full_train"])
def test_render_fwd_equals_renderer(name, mode):
    fx = fixture(name)
    mods = build_modules(int(fx["seed"]), int(fx["dh_sdf"]), int(fx["dh_col"]), device=DEV)
    r = _renderer(mods, mode)
    if not r._can_fold():
        pytest.skip("cn_render_fwd takes the folded feature head (d_hidden == d_feature)")
    g = lambda k: fx[k].to(DEV).float().contiguous()  # noqa: E731
    ev = bool(fx["eval"])
    t_rand = None if ev else g("t_rand")
    t = g("t").reshape(-1)[:1].contiguous()
    car = float(fx["car"])
    args = (g("rays_o"), g("rays_d"), g("rays_d_norm"), t, g("near"), g("far"))
    kw = dict(cos_anneal_ratio=car, it=0, eval=ev, t_rand=t_rand)
    ref = _python_forward(r, *args, **kw)
    with torch.no_grad():
        out = _c_render(r, g("rays_o"), g("rays_d"), t, g("near"), g("far"), car, t_rand=t_rand)
        native = r(*args, **kw)  # the renderer's own no-grad forward: the C call
    R, S = ref["weights"].shape
    _compare(out, ref, R, S)
    _compare_dicts(native, ref)


@pytest.mark.parametrize("mode", MODES)
def test_render_fwd_given_samples_and_larger_batch(mode):
    """1536 rays with the caller's sample positions (the z_vals hook) and with the sampler, at the
    full-width networks."""
    mods = build_modules(11, device=DEV)
    r = _renderer(mods, mode)
    gen = torch.Generator(device=DEV).manual_seed(5)
    R = 1536
    rays_o = (torch.rand(R, 3, device=DEV, generator=gen) - 0.5) * 0.3
    rays_d = torch.nn.functional.normalize(torch.randn(R, 3, device=DEV, generator=gen), dim=-1)
    nrm = rays_d.norm(dim=-1, keepdim=True)
    near = torch.full((R, 1), 0.1, device=DEV)
    far = torch.full((R, 1), 1.9, device=DEV)
    t = torch.full((1,), 0.4, device=DEV)
    t_rand = torch.rand(R, r.n_samples, device=DEV, generator=gen)
    args = (rays_o, rays_d, nrm, t, near, far)
    ref = _python_forward(r, *args, cos_anneal_ratio=0.7, it=0, eval=False, t_rand=t_rand)
    with torch.no_grad():
        out = _c_render(r, rays_o, rays_d, t, near, far, 0.7, t_rand=t_rand)
        _compare(out, ref, *ref["weights"].shape)
        _compare_dicts(r(*args, cos_anneal_ratio=0.7, it=0, eval=False, t_rand=t_rand), ref)
        # eval: no jitter, depth_pred divided by the ray norm
        ref_e = _python_forward(r, *args, cos_anneal_ratio=0.7, it=0, eval=True)
        _compare_dicts(r(*args, cos_anneal_ratio=0.7, it=0, eval=True), ref_e)
        z = torch.sort(torch.rand(R, 96, device=DEV, generator=gen) * 1.8 + 0.1, dim=-1)[0]
        ref2 = _python_forward(r, *args, cos_anneal_ratio=0.7, it=0, eval=False, z_vals=z)
        out2 = _c_render(r, rays_o, rays_d, t, near, far, 0.7, z_in=z)
        _compare(out2, ref2, R, 96)
        assert torch.equal(out2["z"], z)


def test_render_fwd_refuses_inputs_the_c_side_would_overrun():
    """ops.render_fwd / render_train_fwd check what cn_render_fwd assumes (R from rays_o, S from z) before the
    call: a short t_rand or z, near / far of another length, a non-fp32 or strided input raise RuntimeError."""
    from copenerf import ops
    R = 64
    f = lambda *s: torch.zeros(*s, device=DEV)  # noqa: E731
    good = dict(rays_o=f(R, 3), rays_d=f(R, 3), near=f(R, 1), far=f(R, 1), time_step=f(1), inv_s=f(1, 1), car=f(1))

    def call(**kw):
        a = dict(good, **kw)
        t_rand, z = a.pop("t_rand", None), a.pop("z", None)
        return ops.render_fwd(None, None, a["rays_o"], a["rays_d"], a["near"], a["far"], a["time_step"], a["inv_s"],
                              a["car"], 64, 64, 4, t_rand=t_rand, z_in=z)

    for bad in (dict(t_rand=f(R - 1, 64)), dict(t_rand=f(R, 32)), dict(z=f(R - 1, 128)), dict(near=f(R - 1, 1)),
                dict(far=f(2 * R, 1)), dict(rays_d=f(R, 4)), dict(rays_o=f(R, 3).double()),
                dict(t_rand=f(64, R).t()), dict(z=f(R, 128).half())):
        with pytest.raises(RuntimeError):
            call(**bad)
    with pytest.raises(RuntimeError):
        ops.render_train_fwd(None, None, good["rays_o"], good["rays_d"], good["near"], good["far"], good["time_step"],
                             good["inv_s"], good["car"], 64, f(R + 1, 128))
