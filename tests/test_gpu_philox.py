"""cn_uniform_philox (ABI v14, the §8(b) device Philox seed): the device generator bitwise equal to the numpy
Philox4x32-10 (pinned to the Random123 known answers, tests/test_philox.py); uniform moments; seed and offset read
on the device (a captured graph replays with the current offset); cn_sample drawing its jitter with it equals
cn_sample given that jitter as t_rand."""
import numpy as np
import pytest
import torch

from helpers import REN_CFG, build_modules
from philox_ref import uniform

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _so(seed, offset):
    return torch.tensor([seed, offset], dtype=torch.uint64, device=DEV)


@pytest.mark.parametrize("n,seed,offset", [(1, 0, 0), (1001, 678, 3), (4096 * 64, 0x1234567890ABCDEF, (7 << 32) + 11)])
def test_uniform_philox_matches_reference(n, seed, offset):
    from copenerf import ops
    out = ops.uniform_philox(n, _so(seed, offset))
    torch.cuda.synchronize()
    assert np.array_equal(out.cpu().numpy(), uniform(n, seed, offset))


def test_uniform_philox_moments_and_streams():
    from copenerf import ops
    n = 1 << 22
    u = ops.uniform_philox(n, _so(42, 0)).double()
    assert 0.0 <= u.min().item() and u.max().item() < 1.0
    assert abs(u.mean().item() - 0.5) < 1e-3 and abs(u.var().item() - 1.0 / 12.0) < 1e-3
    v = ops.uniform_philox(n, _so(42, n // 4)).double()  # the next disjoint stream
    assert abs(torch.corrcoef(torch.stack([u, v]))[0, 1].item()) < 3e-3


def test_uniform_philox_replays_with_the_current_offset():
    from copenerf import ops
    so = _so(9, 0)
    out = torch.empty(1000, device=DEV)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        ops.uniform_philox(1000, so, out)
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        ops.uniform_philox(1000, so, out)
    for off in (0, 250, 1 << 33):
        so.copy_(_so(9, off))
        g.replay()
        torch.cuda.synchronize()
        assert np.array_equal(out.cpu().numpy(), uniform(1000, 9, off))


def test_sample_draws_its_jitter_on_the_device():
    from copenerf import NeuSRenderer, ops
    sdf, col, dev = build_modules(5, device=DEV)
    r = NeuSRenderer(None, sdf, dev, col, None, **REN_CFG).to(DEV).set_mfma_dtype("bf16x6")
    R = 777
    gen = torch.Generator(device=DEV).manual_seed(1)
    rays_o = (torch.rand(R, 3, device=DEV, generator=gen) - 0.5) * 0.4
    rays_d = torch.nn.functional.normalize(torch.randn(R, 3, device=DEV, generator=gen), dim=-1)
    near, far = torch.full((R, 1), 0.2, device=DEV), torch.full((R, 1), 1.8, device=DEV)
    t = torch.full((1,), 0.1, device=DEV)
    so = _so(1234, 56)
    with torch.no_grad():
        pk = r.sdf_network.params_and_pack()[2]
        net, keep = ops.sdf_net(r.sdf_network.layout(), pk)
        for n_imp in (64, 0):
            k = n_imp // r.up_sample_steps
            S = r.n_samples + r.up_sample_steps * k
            z1 = torch.empty(R, S, device=DEV)
            ops.sample(net, rays_o, rays_d, near, far, None, t, r.n_samples, n_imp, r.up_sample_steps, z1, philox=so)
            t_rand = ops.uniform_philox(R * r.n_samples, so).view(R, r.n_samples)
            z2 = torch.empty(R, S, device=DEV)
            ops.sample(net, rays_o, rays_d, near, far, t_rand, t, r.n_samples, n_imp, r.up_sample_steps, z2)
            torch.cuda.synchronize()
            assert torch.equal(z1, z2), n_imp
    del keep


def test_render_fwd_draws_its_jitter_on_the_device():
    """cn_render_fwd with the philox seed (no t_rand) = cn_render_fwd given that jitter, every output bitwise."""
    from copenerf import NeuSRenderer, ops
    sdf, col, dev = build_modules(6, device=DEV)
    r = NeuSRenderer(None, sdf, dev, col, None, **REN_CFG).to(DEV).set_mfma_dtype("bf16")
    R = 513
    gen = torch.Generator(device=DEV).manual_seed(2)
    rays_o = (torch.rand(R, 3, device=DEV, generator=gen) - 0.5) * 0.3
    rays_d = torch.nn.functional.normalize(torch.randn(R, 3, device=DEV, generator=gen), dim=-1)
    near, far = torch.full((R, 1), 0.1, device=DEV), torch.full((R, 1), 1.9, device=DEV)
    t = torch.full((1,), 0.2, device=DEV)
    so = _so(77, 1 << 20)
    with torch.no_grad():
        sp = r.sdf_network.params_and_pack()
        cp = r.color_network.params_and_pack(fold_feature=(sp[0][-1], sp[1][-1]))
        sn, k1 = ops.sdf_net(r.sdf_network.layout(), sp[2])
        cn, k2 = ops.color_net(r.color_network.layout(), cp[2])
        inv_s = torch.full((1, 1), 20.0, device=DEV)
        car = ops.device_scalar(0.5, DEV)
        a = ops.render_fwd(sn, cn, rays_o, rays_d, near, far, t, inv_s, car, r.n_samples, r.n_importance,
                           r.up_sample_steps, philox=so)
        t_rand = ops.uniform_philox(R * r.n_samples, so).view(R, r.n_samples)
        b = ops.render_fwd(sn, cn, rays_o, rays_d, near, far, t, inv_s, car, r.n_samples, r.n_importance,
                           r.up_sample_steps, t_rand=t_rand)
        torch.cuda.synchronize()
    for k in a:
        assert torch.equal(a[k], b[k]), k
    del k1, k2
