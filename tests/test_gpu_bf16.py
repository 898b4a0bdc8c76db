"""bf16 MFMA mode (config C3, "bf16 MLP MFMA"): cn_linear with mfma_dtype
CN_MFMA_BF16 against torch with the same operand rounding (A and B rounded to
bf16 RNE, products and sums in double), every epilogue, both tiles, the
virtual concat; and the renderer in bf16 mode against the fp32 oracle with the
bf16 tolerance of DESIGN.md §4 (the fp32 path keeps the 1e-4 bar)."""
import pytest
import torch

from helpers import REN_CFG, build_modules, oracle_params
from oracle import neus_oracle as O

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _rnd(*s, scale=1.0, seed=0):
    g = torch.Generator(device="cpu").manual_seed(seed)
    return ((torch.rand(*s, generator=g) * 2 - 1) * scale).to(DEV)


def _ref(A, Bb, N):
    """(A rounded to bf16) @ B^T in double: the exact result the bf16 MFMA path rounds once per sum."""
    return A.bfloat16().double() @ Bb[:N].double().t()


@pytest.mark.parametrize("M,N,K,tile", [(1000, 256, 256, 0), (130, 204, 256, 0), (777, 52, 256, 1),
                                        (64, 256, 64, 0), (4096, 128, 192, 0)])
def test_linear_bf16_store(M, N, K, tile):
    from copenerf import ops
    A = _rnd(M, K, seed=1)
    bn = 64 if tile else 128
    B = torch.zeros(ops.rup(N, bn), K, device=DEV)
    B[:N] = _rnd(N, K, seed=2, scale=0.1)
    Bb = B.bfloat16().contiguous()
    bias = _rnd(N, seed=3)
    ld = ops.rup(N, bn)
    out = torch.full((M, ld), float("nan"), device=DEV)
    ops.linear(A, Bb, N, K, out, ops.EPI_STORE, bias=bias, nzero=ld, tile=tile)
    ref = (_ref(A, Bb, N) + bias.double()).float()
    torch.testing.assert_close(out[:, :N], ref, rtol=1e-5, atol=1e-5)
    assert torch.all(out[:, N:] == 0)


def test_linear_bf16_epilogues_and_concat():
    from copenerf import ops
    M, K1, K2, N = 517, 256, 64, 256
    A, A2 = _rnd(M, K1, seed=4, scale=0.3), _rnd(M, K2, seed=5, scale=0.3)
    Bb = _rnd(N, K1 + K2, seed=6, scale=0.05).bfloat16().contiguous()
    bias = _rnd(N, seed=7, scale=0.3)
    v = (torch.cat([A, A2], 1).bfloat16().double() @ Bb.double().t())
    a = torch.empty(M, N, device=DEV)
    ops.linear(A, Bb, N, K1 + K2, a, ops.EPI_SOFTPLUS, A2=A2, K1=K1, bias=bias)
    z = (v + bias.double()).float()
    torch.testing.assert_close(a, torch.nn.functional.softplus(z, beta=100), rtol=1e-5, atol=2e-5)
    aux0 = torch.nn.functional.softplus(_rnd(M, N, seed=9, scale=0.05), beta=100)
    sg = -torch.expm1(-100.0 * aux0.double())
    aux1, aux2 = _rnd(M, N, seed=8), _rnd(M, N, seed=10)
    o0 = torch.empty(M, N, device=DEV)
    ops.linear(A, Bb, N, K1 + K2, o0, ops.EPI_TANGENT, A2=A2, K1=K1, aux0=aux0, aux_beta=100.0)
    torch.testing.assert_close(o0, (v * sg).float(), rtol=1e-5, atol=1e-5)
    o2 = torch.empty(M, N, device=DEV)
    ops.linear(A, Bb, N, K1 + K2, o2, ops.EPI_BWD_SOFTPLUS, A2=A2, K1=K1, aux0=aux0, aux_beta=100.0, aux1=aux1,
               aux2=aux2, aux2_scale=100.0)
    ref = v * sg + aux1.double() * aux2.double() * 100.0 * (1 - sg) / sg
    torch.testing.assert_close(o2, ref.float(), rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("M,N,K,pairs", [(70000, 256, 256, 2), (1000, 204, 64, 1), (5, 256, 256, 1),
                                         (4097, 256, 320, 1), (300, 52, 192, 2)])
def test_wgrad_bf16(M, N, K, pairs):
    """cn_wgrad with mfma_dtype CN_MFMA_BF16: dW against the bf16-rounded operands
    in double; db is the column sum of the fp32 Y0 (not rounded)."""
    from copenerf import ops
    ldn, ldk = ops.rup(N, 128), ops.rup(K, 128 if K % 128 == 0 else 64)
    Y0, X0 = _rnd(M, ldn, seed=15), _rnd(M, ldk, seed=16)
    Y1, X1 = (_rnd(M, ldn, seed=17), _rnd(M, ldk, seed=18)) if pairs == 2 else (None, None)
    dW = torch.empty(N, K, device=DEV)
    db = torch.empty(N, device=DEV)
    ops.wgrad(Y0, X0, N, K, dW, db=db, Y1=Y1, X1=X1, mode="bf16")
    r = lambda t, n: t[:, :n].bfloat16().double()  # noqa: E731
    ref = r(Y0, N).t() @ r(X0, K)
    if pairs == 2:
        ref = ref + r(Y1, N).t() @ r(X1, K)
    tol = 1e-6 * M ** 0.5 + 1e-5
    torch.testing.assert_close(dW, ref.float(), rtol=1e-4, atol=tol)
    torch.testing.assert_close(db, Y0[:, :N].double().sum(0).float(), rtol=1e-4, atol=tol)
    dW2 = torch.empty_like(dW)
    ops.wgrad(Y0, X0, N, K, dW2, Y1=Y1, X1=X1, mode="bf16")
    assert torch.equal(dW, dW2)


def test_render_bf16_mode_against_fp32_oracle():
    """bf16 operands cannot meet the fp32 1e-4 bar; measured against the fp32
    oracle on identical samples (1024 rays) the bf16 path stays within the bounds
    asserted here, and training gradients stay finite."""
    from copenerf import NeuSRenderer
    R = 1024
    g = torch.Generator().manual_seed(R)
    mods_cpu = build_modules(55, 256, 256)
    P, Pc, var, _ = oracle_params(*mods_cpu)
    o = torch.tensor([0.05, -0.03, 1.6]).expand(R, 3).contiguous()
    d = torch.cat([(torch.rand(R, 2, generator=g) - 0.5) * 0.6, -torch.ones(R, 1)], -1)
    nrm = d.norm(dim=-1, keepdim=True)
    d = d / nrm
    t = torch.tensor([0.25])
    near, far = torch.full((R, 1), 0.01), torch.full((R, 1), 3.0)
    t_rand = torch.rand(R, 64, generator=g)
    torch.set_num_threads(8)
    ref = O.render(P, Pc, var, o, d, nrm, t, near, far, car=0.5, t_rand=t_rand)
    sdf, col, dev = build_modules(55, 256, 256, device=DEV)
    r = NeuSRenderer(None, sdf, dev, col, None, **REN_CFG).to(DEV).set_mfma_dtype("bf16")
    args = tuple(x.to(DEV) for x in (o, d, nrm, t, near, far))
    out = r(*args, cos_anneal_ratio=0.5, it=0, eval=False, z_vals=ref["z_vals"].to(DEV))
    errs = {}
    for k in ("color_fine", "depth_pred"):
        e = (out[k].detach().cpu() - ref[k].detach()).abs()
        errs[k] = (e.max().item(), e.mean().item())
    print("bf16 vs fp32 oracle (max, mean):", errs)
    # measured on MI355X: rgb max 1.8e-3 / mean 2.0e-4, depth max 5.0e-3 / mean 5.6e-4
    assert errs["color_fine"][0] <= 5e-3 and errs["color_fine"][1] <= 5e-4, errs
    assert errs["depth_pred"][0] <= 1.5e-2 and errs["depth_pred"][1] <= 1.5e-3, errs
    loss = O.train_loss(out, torch.rand(R, 3, generator=g).to(DEV))
    loss.backward()
    for p in list(sdf.parameters()) + list(col.parameters()):
        assert p.grad is not None and torch.isfinite(p.grad).all()


def test_sdf_field_bf16_mode_narrow_width():
    """bf16 mode at a hidden width that is not 256-padded (d_hidden = 64: 128-wide buffers): the
    operand images stay off (their weight gradients need the 256x256 ring), fp32 operands are
    rounded on load; the field and a double-backward loss's parameter gradients against the fp32
    mode within bf16 rounding."""
    from copenerf import SDFNetwork, fields
    from helpers import SDF_CFG
    torch.manual_seed(5)
    net = SDFNetwork(**dict(SDF_CFG, d_hidden=64)).to(DEV)
    lay = net.layout()
    x = torch.rand(3001, 4, device=DEV) * 2 - 1
    res = []
    for mode in ("bf16", "fp32"):
        net.mfma_dtype = mode
        if mode == "bf16":
            assert not fields._img_mode(net.params_and_pack()[2], lay)
        sdf, feat, g = net.field(x)
        loss = ((g.norm(dim=-1) - 1) ** 2).mean() + sdf.abs().mean() + 1e-2 * feat.square().mean()
        grads = torch.autograd.grad(loss, list(net.parameters()))
        res.append([sdf.detach(), g.detach()] + list(grads))
    names = ["sdf", "grad"] + [n for n, _ in net.named_parameters()]
    for n, a, b in zip(names, res[0], res[1]):
        assert torch.isfinite(a).all(), n
        rel = ((a - b).norm() / b.norm().clamp_min(1e-30)).item()
        print(f"{n}: relative L2 {rel:.2e}")
        assert rel <= 5e-2, (n, rel)
