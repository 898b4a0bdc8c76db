"""HIP kernels against plain torch fp32 (GEMM family) and against the CPU oracle
(fields, compositing, sampler).  All calls go through the C ABI."""
import math

import pytest
import torch

from helpers import build_modules, fixture, oracle_params
from oracle import neus_oracle as O

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _rnd(*s, scale=1.0, seed=0):
    g = torch.Generator(device="cpu").manual_seed(seed)
    return ((torch.rand(*s, generator=g) * 2 - 1) * scale).to(DEV)


def _ops():
    from copenerf import ops
    return ops


# ----------------------------------------------------------------------------- GEMM family
@pytest.mark.parametrize("M,N,K,tile", [(1000, 256, 256, 0), (130, 204, 224, 0), (777, 52, 256, 1),
                                        (64, 256, 64, 0), (4096, 128, 96, 0)])
def test_linear_store_matches_torch(M, N, K, tile):
    ops = _ops()
    A = _rnd(M, K, seed=1)
    bn = 64 if tile else 128
    Np = ops.rup(N, bn)
    B = torch.zeros(Np, K, device=DEV)
    B[:N] = _rnd(N, K, seed=2, scale=0.1)
    bias = _rnd(N, seed=3)
    ld = ops.rup(N, bn)
    out = torch.full((M, ld), float("nan"), device=DEV)
    ops.linear(A, B, N, K, out, ops.EPI_STORE, bias=bias, nzero=ld, tile=tile)
    ref = (A.double() @ B[:N].double().t() + bias.double()).float()
    torch.testing.assert_close(out[:, :N], ref, rtol=1e-5, atol=1e-5)
    assert torch.all(out[:, N:] == 0)


def test_linear_tile_order_does_not_change_results():
    """cn_linear_desc.flags bit 0 (reverse M-tile walk, alternated launch to launch by
    ops.linear): both walks give bitwise identical outputs, edge tiles included."""
    ops = _ops()
    M, N, K = 70001, 256, 256
    A = _rnd(M, K, seed=51)
    W = _rnd(N, K, seed=52, scale=0.05)
    for B in (W, ops.split_bf16x3(W)):
        outs = []
        for _ in range(2):  # consecutive launches: opposite walks
            o = torch.empty(M, N, device=DEV)
            ops.linear(A, B, N, K, o, ops.EPI_SOFTPLUS, bias=W[0].contiguous(), beta=100.0)
            outs.append(o)
        assert torch.equal(outs[0], outs[1])


def test_linear_virtual_concat_rank1_and_divisor():
    ops = _ops()
    M, K1, K2, N = 333, 256, 64, 256
    A, A2 = _rnd(M, K1, seed=4), _rnd(M, K2, seed=5)
    B = _rnd(N, K1 + K2, seed=6, scale=0.1)
    rowv, colv = _rnd(M, seed=7), _rnd(N, seed=8)
    out = torch.empty(M, N, device=DEV)
    ops.linear(A, B, N, K1 + K2, out, ops.EPI_STORE, A2=A2, K1=K1, rowv=rowv, colv=colv, adiv=ops.SQRT2)
    ref = torch.cat([A, A2], 1).double() @ B.double().t() / ops.SQRT2 + rowv.double()[:, None] * colv.double()
    torch.testing.assert_close(out, ref.float(), rtol=1e-5, atol=1e-5)


def test_linear_softplus_and_derivative():
    ops = _ops()
    M, N, K = 517, 256, 256
    A = _rnd(M, K, seed=9, scale=0.3)
    B = _rnd(N, K, seed=10, scale=0.05)
    bias = _rnd(N, seed=11, scale=0.3)
    a = torch.empty(M, N, device=DEV)
    ops.linear(A, B, N, K, a, ops.EPI_SOFTPLUS, bias=bias, beta=100.0, threshold=20.0)
    z = torch.nn.functional.linear(A, B, bias)
    torch.testing.assert_close(a, torch.nn.functional.softplus(z, beta=100), rtol=1e-5, atol=2e-5)
    # the identity the backward epilogues rely on (ABI v4): softplus' = 1 - exp(-beta a)
    # from the stored activation equals torch's derivative (1 on the linear branch) of the
    # kernel's own pre-activation (the STORE epilogue: same accumulation, same z) to ~1e-7
    zk = torch.empty(M, N, device=DEV)
    ops.linear(A, B, N, K, zk, ops.EPI_STORE, bias=bias)
    sg = -torch.expm1(-100.0 * a.double())
    ref = torch.where(zk * 100 > 20, torch.ones_like(zk), torch.sigmoid(100 * zk)).double()
    assert (sg - ref).abs().max().item() < 5e-7


def _act(M, N, seed, c=1.0):
    """Softplus(beta=100) activations / c of pre-activations in [-0.05, 0.05]
    (softplus' in [0.007, 0.993]), as the SDF forward stores them."""
    z = _rnd(M, N, seed=seed, scale=0.05)
    return (torch.nn.functional.softplus(z, beta=100) / c).contiguous()


def _sg(aux0, aux_beta):
    return -torch.expm1(-aux_beta * aux0.double())


def test_linear_mul_split_tangent_bwd_relu():
    ops = _ops()
    M, N, K = 300, 256, 224
    A = _rnd(M, K, seed=12)
    B = _rnd(N, K, seed=13, scale=0.1)
    aux0 = _act(M, N, 24, c=ops.SQRT2)
    ab = 100.0 * ops.SQRT2
    sg = _sg(aux0, ab)
    aux1, aux2 = _rnd(M, N, seed=14), _rnd(M, N, seed=15)
    v = A.double() @ B.double().t()
    out, split = torch.empty(M, 256, device=DEV), torch.empty(M, 64, device=DEV)
    ops.linear(A, B, N, K, out, ops.EPI_MUL, aux0=aux0, aux_beta=ab, nsplit=204, out_split=split, nzero=256,
               adiv=ops.SQRT2)
    torch.testing.assert_close(out[:, :204], (v / ops.SQRT2 * sg)[:, :204].float(), rtol=1e-5, atol=1e-5)
    assert torch.all(out[:, 204:] == 0)
    torch.testing.assert_close(split[:, :52], (v / ops.SQRT2)[:, 204:].float(), rtol=1e-5, atol=1e-5)
    o0 = torch.empty(M, N, device=DEV)
    ops.linear(A, B, N, K, o0, ops.EPI_TANGENT, aux0=aux0, aux_beta=ab, odiv=ops.SQRT2, beta=100.0)
    torch.testing.assert_close(o0, (v * sg / ops.SQRT2).float(), rtol=1e-5, atol=1e-5)
    o2 = torch.empty(M, N, device=DEV)
    ops.linear(A, B, N, K, o2, ops.EPI_BWD_SOFTPLUS, aux0=aux0, aux_beta=ab)
    torch.testing.assert_close(o2, (v * sg).float(), rtol=1e-5, atol=1e-5)
    # the second-order term beta s (1 - sg) z', z' = u' c / sg, rebuilt from s = aux1, u' = aux2
    ops.linear(A, B, N, K, o2, ops.EPI_BWD_SOFTPLUS, aux0=aux0, aux_beta=ab, aux1=aux1, aux2=aux2,
               aux2_scale=ab)
    ref = v * sg + aux1.double() * aux2.double() * ab * (1 - sg) / sg
    torch.testing.assert_close(o2, ref.float(), rtol=1e-4, atol=1e-4)
    # sg = 0 (a zero activation) carries s = u' = 0: the term is 0, not 0 * inf
    z0 = torch.zeros_like(aux0)
    ops.linear(A, B, N, K, o2, ops.EPI_BWD_SOFTPLUS, aux0=z0, aux_beta=ab, aux1=z0, aux2=z0, aux2_scale=ab)
    assert torch.all(o2 == 0)
    o3 = torch.empty(M, N, device=DEV)
    ops.linear(A, B, N, K, o3, ops.EPI_BWD_RELU, aux0=aux1)
    torch.testing.assert_close(o3, torch.where(aux1 > 0, v, torch.zeros_like(v)).float(), rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("M,N,K,pairs", [(70000, 256, 256, 2), (1000, 204, 64, 1), (5, 256, 256, 1),
                                         (4097, 256, 320, 1)])
def test_wgrad_matches_torch(M, N, K, pairs):
    ops = _ops()
    ldn, ldk = ops.rup(N, 128), ops.rup(K, 128 if K % 128 == 0 else 64)
    Y0, X0 = _rnd(M, ldn, seed=15), _rnd(M, ldk, seed=16)
    Y1, X1 = (_rnd(M, ldn, seed=17), _rnd(M, ldk, seed=18)) if pairs == 2 else (None, None)
    dW = torch.empty(N, K, device=DEV)
    db = torch.empty(N, device=DEV)
    ops.wgrad(Y0, X0, N, K, dW, db=db, Y1=Y1, X1=X1)
    ref = Y0[:, :N].double().t() @ X0[:, :K].double()
    if pairs == 2:
        ref = ref + Y1[:, :N].double().t() @ X1[:, :K].double()
    tol = 1e-6 * math.sqrt(M) + 1e-5
    torch.testing.assert_close(dW, ref.float(), rtol=1e-4, atol=tol)
    torch.testing.assert_close(db, Y0[:, :N].double().sum(0).float(), rtol=1e-4, atol=tol)
    # determinism: the slab reduction has a fixed order
    dW2 = torch.empty_like(dW)
    ops.wgrad(Y0, X0, N, K, dW2, Y1=Y1, X1=X1)
    assert torch.equal(dW, dW2)


def test_row_head_colsum_scale_cols():
    ops = _ops()
    M, K = 5000, 256
    A = _rnd(M, K, seed=19)
    W = _rnd(3, K, seed=20, scale=0.1)
    b = _rnd(3, seed=21)
    out = torch.empty(M, 3, device=DEV)
    ops.row_head(A, K, W, b, 3, 1, out)
    torch.testing.assert_close(out, torch.sigmoid(A @ W.t() + b), rtol=1e-5, atol=1e-6)
    w = _rnd(M, seed=22)
    cs = torch.empty(K, device=DEV)
    ops.colsum(A, K, cs, w=w, wdiv=2.0)
    torch.testing.assert_close(cs, ((w.double()[:, None] * A.double()).sum(0) / 2).float(), rtol=1e-5, atol=1e-4)
    sc = torch.empty(M, K, device=DEV)
    ops.scale_cols(A, K, W[0].contiguous(), sc)
    torch.testing.assert_close(sc, A * W[0], rtol=0, atol=0)
    act = _act(M, K, 25)
    ops.scale_cols(act, K, W[0].contiguous(), sc, act_beta=100.0)
    torch.testing.assert_close(sc, (_sg(act, 100.0) * W[0].double()).float(), rtol=1e-5, atol=1e-7)
    ops.scale_cols(act, K, W[0].contiguous(), sc, act_beta=100.0, rowv=w)
    torch.testing.assert_close(sc, (_sg(act, 100.0) * W[0].double() * w.double()[:, None]).float(), rtol=1e-5,
                               atol=1e-7)


@pytest.mark.parametrize("N,x6", [(128, False), (256, True), (64, False), (256, False)])
def test_softplus_head(N, x6):
    """EPI_SOFTPLUS_HEAD: the last SDF hidden layer with the sdf head and the ∇-pass seed
    in its epilogue -- a = softplus_100(A Bᵀ + b), out1 = colv ⊙ sg(a), head[idx[m]] =
    a[m]·w + c -- against torch in float64; out0 may be absent; N = 256 needs the
    bf16x6 128x256 tile (the fp32 mode's 128-wide tile is rejected)."""
    ops = _ops()
    M, K = 3000, 256
    A = _rnd(M, K, seed=41, scale=0.1)
    W = _rnd(N, K, seed=42, scale=0.05)
    b = _rnd(N, seed=43, scale=0.05)
    hw, hb, cv = _rnd(N, seed=44), _rnd(1, seed=45), _rnd(N, seed=46)
    B = ops.split_bf16x3(W) if x6 else W
    z = A.double() @ W.double().t() + b.double()
    a_ref = torch.nn.functional.softplus(z, beta=100)
    out0, out1 = torch.empty(M, N, device=DEV), torch.empty(M, N, device=DEV)
    head = torch.empty(M, device=DEV)
    kw = dict(bias=b, beta=100.0, threshold=20.0, head_w=hw, head_b=hb, head_out=head)
    if N > 128 and not x6:
        with pytest.raises(RuntimeError, match="SOFTPLUS_HEAD"):
            ops.linear(A, B, N, K, out0, ops.EPI_SOFTPLUS_HEAD, **kw)
        return
    ops.linear(A, B, N, K, out0, ops.EPI_SOFTPLUS_HEAD, out1=out1, colv=cv, aux_beta=100.0, **kw)
    torch.testing.assert_close(out0, a_ref.float(), rtol=1e-5, atol=2e-6)
    sg = _sg(out0, 100.0)
    torch.testing.assert_close(out1, (cv.double() * sg).float(), rtol=1e-5, atol=1e-7)
    h_ref = out0.double() @ hw.double() + hb.double()
    torch.testing.assert_close(head, h_ref.float(), rtol=1e-5, atol=1e-5)
    # scattered, no stored activation: the same head values at the destination rows
    perm = torch.randperm(M, generator=torch.Generator().manual_seed(7)).to(DEV).int()
    head2 = torch.full((M,), float("nan"), device=DEV)
    ops.linear(A, B, N, K, None, ops.EPI_SOFTPLUS_HEAD, **dict(kw, head_out=head2), head_idx=perm)
    assert torch.equal(head2[perm.long()], head)


def test_softplus_adjoint():
    """cn_softplus_adjoint: the adjoint of the last SDF hidden layer when the feature
    head is folded into the colour network -- (D + rowv colv) σ + c2 s1 s2 (1-σ)/σ,
    σ recovered from the stored activation (0 where σ = 0)."""
    ops = _ops()
    M, K = 3000, 256
    act = _act(M, K, 31)
    D = _rnd(M, K, seed=32)
    rv, cv = _rnd(M, seed=33), _rnd(K, seed=34)
    s1, s2 = _rnd(M, K, seed=35), _rnd(M, K, seed=36)
    out = torch.empty(M, K, device=DEV)
    sg = _sg(act, 100.0)
    rr = torch.where(sg > 0, (1 - sg) / sg.clamp_min(1e-300), torch.zeros_like(sg))
    ops.softplus_adjoint(act, K, out, act_beta=100.0, D=D)
    torch.testing.assert_close(out, (D.double() * sg).float(), rtol=1e-5, atol=1e-7)
    ops.softplus_adjoint(act, K, out, act_beta=100.0, D=D, rowv=rv, colv=cv, aux1=s1, aux2=s2, aux2_scale=0.7)
    ref = (D.double() + rv.double()[:, None] * cv.double()) * sg + 0.7 * s1.double() * s2.double() * rr
    torch.testing.assert_close(out, ref.float(), rtol=1e-4, atol=1e-5)
    assert torch.isfinite(out).all()
    # the column-sum form: same out, plus lin8's sdf-row gradient Σ_m rv act + s2, over a ragged M
    for m in (M, 1537, 1):
        out2, cs, rs = torch.full((m, K), float("nan"), device=DEV), torch.empty(K, device=DEV), torch.empty(1, device=DEV)
        ops.softplus_adjoint(act[:m], K, out2, act_beta=100.0, D=D[:m], rowv=rv[:m].contiguous(), colv=cv,
                             aux1=s1[:m], aux2=s2[:m], aux2_scale=0.7, cs_out=cs, rs_out=rs, cs_div=2.0)
        assert torch.equal(out2, out[:m])
        cs_ref = (rv[:m].double()[:, None] * act[:m].double() + s2[:m].double()).sum(0) / 2.0
        torch.testing.assert_close(cs, cs_ref.float(), rtol=1e-5, atol=1e-4)
        torch.testing.assert_close(rs, (rv[:m].double().sum() / 2.0).float().view(1), rtol=1e-5, atol=1e-5)
    cs2 = torch.empty(K, device=DEV)
    ops.softplus_adjoint(act, K, out, act_beta=100.0, D=D, cs_out=cs2)  # no rowv / aux2: zero sums
    assert torch.all(cs2 == 0)


@pytest.mark.parametrize("img", [0, 1, 2, 4, 7])
def test_softplus_adjoint_cs_images_strided(img):
    """The column-sum form (buffer views of a block's rows, four rows in flight per lane) over
    bf16 operand images (in_bf16 mask `img`, bf16 out when img) and column slices of wider
    tensors (leading dimension > N): out bitwise equal to the plain form's, the sums within fp32
    summation error of the fp64 reference, over ragged M (block tails, a lane's tail)."""
    ops = _ops()
    K, W = 256, 264
    for M in (1029, 517, 3):
        def t(seed, b):
            x = _rnd(M, W, seed=seed)[:, 4:4 + K]
            return x.to(torch.bfloat16) if b else x
        act = _act(M, W, 41 + M)[:, 4:4 + K]
        act = act.to(torch.bfloat16) if img & 2 else act
        D, s1, s2 = t(42, img & 1), t(43, img & 4), t(44, img & 4)
        rv, cv = _rnd(M, seed=45), _rnd(K, seed=46)
        dt = torch.bfloat16 if img else torch.float32
        ref_out = torch.full((M, W), float("nan"), device=DEV, dtype=dt)[:, :K]
        out = torch.full((M, W), float("nan"), device=DEV, dtype=dt)[:, :K]
        kw = dict(act_beta=100.0, D=D, rowv=rv, colv=cv, aux1=s1, aux2=s2, aux2_scale=0.7)
        ops.softplus_adjoint(act, K, ref_out, **kw)
        cs, rs = torch.empty(K, device=DEV), torch.empty(1, device=DEV)
        ops.softplus_adjoint(act, K, out, cs_out=cs, rs_out=rs, **kw)
        assert torch.equal(out, ref_out)
        cs_ref = (rv.double()[:, None] * act.double() + s2.double()).sum(0)
        torch.testing.assert_close(cs, cs_ref.float(), rtol=1e-5, atol=1e-4)
        torch.testing.assert_close(rs, rv.double().sum().float().view(1), rtol=1e-5, atol=1e-5)


def test_c_abi_rejects_bad_arguments():
    ops = _ops()
    A = torch.zeros(10, 30, device=DEV)
    B = torch.zeros(128, 30, device=DEV)
    with pytest.raises(RuntimeError, match="multiple of 32"):
        ops.linear(A, B, 16, 30, torch.empty(10, 16, device=DEV), ops.EPI_STORE)
    with pytest.raises(RuntimeError, match="CUDA/HIP tensor"):
        ops.linear(A.cpu(), B, 16, 32, torch.empty(10, 16, device=DEV), ops.EPI_STORE)


# ----------------------------------------------------------------------------- fields vs oracle
def _sdf_points(M, seed):
    g = torch.Generator().manual_seed(seed)
    return torch.cat([(torch.rand(M, 3, generator=g) - 0.5) * 1.6, torch.full((M, 1), 0.25)], -1)


@pytest.mark.parametrize("dh", [256, 64])
def test_sdf_field_forward_gradient_and_double_backward(dh):
    sdf, col, dev = build_modules(31, dh, dh)
    P, Pc, var, leaves = oracle_params(sdf, col, dev)
    M = 3000
    x = _sdf_points(M, 5)
    g = torch.Generator().manual_seed(6)
    a, Bm, C = torch.randn(M, 1, generator=g), torch.randn(M, 256, generator=g) * 0.01, torch.randn(M, 4, generator=g)
    # oracle
    out = O.sdf_mlp(P, x)
    gr = O.sdf_gradient(P, x)
    L = (a * out[:, :1]).sum() + (Bm * out[:, 1:]).sum() + (C * gr).sum()
    names = [n for n in leaves if n.startswith("sdf.")]
    ref_grads = torch.autograd.grad(L, [leaves[n] for n in names])
    # HIP
    sdf_g = sdf.to(DEV)
    s, f, G = sdf_g.field(x.to(DEV), want_feat=True, want_grad=True)
    torch.testing.assert_close(s.cpu(), out[:, :1].detach(), rtol=1e-4, atol=2e-5)
    torch.testing.assert_close(f.cpu(), out[:, 1:].detach(), rtol=1e-4, atol=2e-5)
    torch.testing.assert_close(G.cpu(), gr.detach(), rtol=1e-3, atol=1e-4)
    Lg = (a.to(DEV) * s).sum() + (Bm.to(DEV) * f).sum() + (C.to(DEV) * G).sum()
    params = dict(sdf_g.named_parameters())
    got = torch.autograd.grad(Lg, [params[n[4:]] for n in names])
    for n, r, gg in zip(names, ref_grads, got):
        scale = r.abs().max().item() + 1e-6
        torch.testing.assert_close(gg.cpu(), r, rtol=2e-3, atol=2e-4 * scale, msg=lambda m: f"{n}: {m}")


@pytest.mark.parametrize("want_feat", [False, True])
def test_sdf_first_order_input_and_parameter_gradients(want_feat):
    """First order with dL/dx and the parameter gradients together (e.g. train.py:504's
    SDFNetwork.sdf on pose-dependent points): the input gradient comes out of the
    parameter adjoint chain (fields.sdf_backward want_dx) -- against oracle autograd."""
    sdf, col, dev = build_modules(33)
    P, Pc, var, leaves = oracle_params(sdf, col, dev)
    M = 2500
    x = _sdf_points(M, 7)
    g = torch.Generator().manual_seed(8)
    a, Bm = torch.randn(M, 1, generator=g), torch.randn(M, 256, generator=g) * 0.01
    xr = x.clone().requires_grad_(True)
    out = O.sdf_mlp(P, xr)
    L = (a * out[:, :1]).sum() + ((Bm * out[:, 1:]).sum() if want_feat else 0.0)
    names = [n for n in leaves if n.startswith("sdf.")]
    ref = torch.autograd.grad(L, [xr] + [leaves[n] for n in names])
    sdf_g = sdf.to(DEV)
    xg = x.to(DEV).requires_grad_(True)
    s, f, _ = sdf_g.field(xg, want_feat=want_feat, want_grad=False)
    Lg = (a.to(DEV) * s).sum() + ((Bm.to(DEV) * f).sum() if want_feat else 0.0)
    params = dict(sdf_g.named_parameters())
    got = torch.autograd.grad(Lg, [xg] + [params[n[4:]] for n in names])
    sc = ref[0].abs().max().item() + 1e-6  # dL/d(x, y, z, t): all four embedded inputs
    torch.testing.assert_close(got[0].cpu(), ref[0], rtol=2e-3, atol=2e-4 * sc)
    for n, r, gg in zip(names, ref[1:], got[1:]):
        scale = r.abs().max().item() + 1e-6
        torch.testing.assert_close(gg.cpu(), r, rtol=2e-3, atol=2e-4 * scale, msg=lambda m: f"{n}: {m}")


def test_color_field_forward_backward():
    sdf, col, dev = build_modules(32)
    P, Pc, var, leaves = oracle_params(sdf, col, dev)
    fx = fixture("seams")
    R, S = 16, 16
    M = R * S
    pts = fx["col_pts"][:M]
    dirs_r = fx["col_dirs"][:R]
    dirs = dirs_r[:, None, :].expand(R, S, 3).reshape(M, 3)
    feat = fx["col_feat"][:M].clone().requires_grad_(True)
    gg = fx["col_g"][:M].clone().requires_grad_(True)
    D = fx["col_D"][:M]
    rgb = O.color_mlp(Pc, pts, gg, dirs, feat)
    names = [n for n in leaves if n.startswith("col.")]
    ref = torch.autograd.grad((D * rgb).sum(), [leaves[n] for n in names] + [feat, gg])
    colg = col.to(DEV)
    featg = feat.detach().to(DEV).requires_grad_(True)
    ggg = gg.detach().to(DEV).requires_grad_(True)
    rgbg = colg.color(pts.to(DEV), ggg, dirs_r.to(DEV), S, featg)
    torch.testing.assert_close(rgbg.cpu(), rgb.detach(), rtol=1e-4, atol=1e-5)
    params = dict(colg.named_parameters())
    got = torch.autograd.grad((D.to(DEV) * rgbg).sum(), [params[n[4:]] for n in names] + [featg, ggg])
    for n, r, g in zip(names + ["feat", "g"], ref, got):
        torch.testing.assert_close(g.cpu(), r, rtol=1e-3, atol=1e-5 * (r.abs().max().item() + 1e-3),
                                   msg=lambda m: f"{n}: {m}")


def test_composite_forward_backward():
    from copenerf.renderer import _CompositeFn
    g = torch.Generator().manual_seed(40)
    R, S = 37, 128
    z = torch.sort(torch.rand(R, S, generator=g) * 2.5 + 0.1, -1)[0]
    sdf = (0.9 - z.reshape(-1, 1)) + 0.05 * torch.randn(R * S, 1, generator=g)
    Gm = torch.randn(R * S, 4, generator=g)
    rgb = torch.rand(R * S, 3, generator=g)
    rays_d = torch.nn.functional.normalize(torch.randn(R, 3, generator=g), dim=-1)
    near, far = torch.full((R, 1), 0.1), torch.full((R, 1), 2.6)
    inv_s = torch.tensor([[30.0]])
    car = 0.3
    dcol, ddep, dw = torch.randn(R, 3, generator=g), torch.randn(R, 1, generator=g), torch.randn(R, S, generator=g)
    # oracle
    leaves = [t.clone().requires_grad_(True) for t in (sdf, Gm, rgb, inv_s)]
    sd = (far[0, 0] - near[0, 0]) / 64
    dists = torch.cat([z[:, 1:] - z[:, :-1], sd.expand(R, 1)], -1)
    dirs = rays_d[:, None, :].expand(R, S, 3).reshape(-1, 3)
    c, d, w, pc = O.composite(z, dists, leaves[0], leaves[1][:, :3], leaves[2].reshape(R, S, 3), dirs, leaves[3], car)
    Lr = (dcol * c).sum() + (ddep * d).sum() + (dw * w).sum()
    ref = torch.autograd.grad(Lr, leaves)
    # HIP
    gl = [t.to(DEV).requires_grad_(True) for t in (sdf, Gm, rgb, inv_s)]
    cg, dg, wg, pcg = _CompositeFn.apply(z.to(DEV), gl[0], gl[1], gl[2], rays_d.to(DEV), gl[3], near.to(DEV),
                                         far.to(DEV), 64, car)
    torch.testing.assert_close(cg.cpu(), c, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(dg.cpu(), d, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(wg.cpu(), w, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(pcg.cpu(), pc.reshape(R, S), rtol=1e-5, atol=1e-6)
    Lg = (dcol.to(DEV) * cg).sum() + (ddep.to(DEV) * dg).sum() + (dw.to(DEV) * wg).sum()
    got = torch.autograd.grad(Lg, gl)
    for n, r, gg in zip(("sdf", "G", "rgb", "inv_s"), ref, got):
        torch.testing.assert_close(gg.cpu(), r, rtol=1e-4, atol=1e-5 * (r.abs().max().item() + 1e-3),
                                   msg=lambda m: f"{n}: {m}")


@pytest.mark.parametrize("n", [64, 80, 96, 112])
def test_up_sample_merge_matches_reference_seams(n):
    ops = _ops()
    fx = fixture("seams")
    z, sd = fx[f"up{n}_z"], fx[f"up{n}_sdf"]
    R = z.shape[0]
    z_out, z_new = torch.empty(R, n + 16, device=DEV), torch.empty(R, 16, device=DEV)
    sdf_out = torch.empty(R, n + 16, device=DEV)
    dst = torch.empty(R * 16, dtype=torch.int32, device=DEV)
    ops.up_sample_merge(z.to(DEV), sd.to(DEV), 16, float(fx[f"up{n}_invs"]), z_out, z_new, sdf_out, dst)
    torch.testing.assert_close(z_new.cpu(), fx[f"up{n}_new"], rtol=0, atol=2e-6)
    torch.testing.assert_close(z_out.cpu(), fx[f"up{n}_cat"], rtol=0, atol=2e-6)
    # the scatter map puts every new sample where its z landed and old sdf at the old z positions
    flat = z_out.reshape(-1)
    assert torch.equal(flat[dst.long()], z_new.reshape(-1))
    pos_old = sdf_out.clone().reshape(-1)
    pos_old[dst.long()] = float("nan")
    kept = pos_old[~torch.isnan(pos_old)].reshape(R, n)
    torch.testing.assert_close(kept.cpu(), sd, rtol=0, atol=0)


def test_row_head_edge_cases_and_rgb_head_bwd():
    """row_head with one output scattered through dst_index, K < 256 and a row
    count that is not a multiple of the 8-row pass; rgb_head_bwd (sigmoid + Linear
    256 -> 3 backward, neus_fields.py:367-373) against torch autograd."""
    ops = _ops()
    M, K = 5003, 64
    A = _rnd(M, K, seed=23)
    W = _rnd(1, K, seed=24, scale=0.2)
    b = _rnd(1, seed=25)
    dst = torch.randperm(M, device=DEV).to(torch.int32)
    out = torch.full((M, 1), float("nan"), device=DEV)
    ops.row_head(A, K, W, b, 1, 0, out, dst_index=dst)
    ref = torch.empty(M, 1, device=DEV)
    ref[dst.long()] = A @ W.t() + b
    torch.testing.assert_close(out, ref, rtol=1e-5, atol=1e-6)
    M, K = 3001, 256
    H3 = torch.relu(_rnd(M, K, seed=26))
    W3 = _rnd(3, K, seed=27, scale=0.1).requires_grad_(True)
    b3 = _rnd(3, seed=28).requires_grad_(True)
    Z = _rnd(M, K, seed=29)  # pre-activation whose relu is H3's pattern
    Z = torch.where(H3 > 0, H3, -Z.abs()).requires_grad_(True)
    rgb = torch.sigmoid(torch.relu(Z) @ W3.t() + b3)
    drgb = _rnd(M, 3, seed=30)
    gZ, gW, gb = torch.autograd.grad(rgb, [Z, W3, b3], drgb)
    dZ = torch.empty(M, K, device=DEV)
    dW = torch.empty(3, K, device=DEV)
    db = torch.empty(3, device=DEV)
    ops.rgb_head_bwd(drgb, rgb.detach().contiguous(), torch.relu(Z).detach(), K, W3.detach().contiguous(), dZ, dW, db)
    torch.testing.assert_close(dZ, gZ, rtol=1e-5, atol=1e-7)
    torch.testing.assert_close(dW, gW, rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(db, gb, rtol=1e-4, atol=1e-5)
    # dZ as a bf16 operand image (bf16 mode): the RNE image of the same values, dW / db unchanged
    dZb, dW2, db2 = torch.empty(M, K, device=DEV, dtype=torch.bfloat16), torch.empty_like(dW), torch.empty_like(db)
    ops.rgb_head_bwd(drgb, rgb.detach().contiguous(), torch.relu(Z).detach(), K, W3.detach().contiguous(), dZb, dW2, db2)
    assert torch.equal(dZb, dZ.bfloat16()) and torch.equal(dW2, dW) and torch.equal(db2, db)
    cs = torch.empty(K, device=DEV)
    ops.colsum(H3, K, cs)
    torch.testing.assert_close(cs, H3.double().sum(0).float(), rtol=1e-5, atol=1e-4)


@pytest.mark.parametrize("patch", [4, 2, 1])
def test_train_loss_matches_reference_losses(patch):
    """cn_train_loss (value and input gradients) against the oracle's torch
    statement of training.py:506-509, train.py:519-526 and losses.py:7-38."""
    from copenerf.losses import train_losses
    R, S = 4096, 32
    g = torch.Generator(device=DEV).manual_seed(31)
    color = torch.rand(R, 3, device=DEV, generator=g).requires_grad_(True)
    gt = torch.rand(R, 3, device=DEV, generator=g)
    depth = (torch.rand(R, 1, device=DEV, generator=g) * 3).requires_grad_(True)
    G = torch.randn(R * S, 4, device=DEV, generator=g)
    G[:7, :3] = 0.0  # zero normals: the norm's gradient is 0 there
    G.requires_grad_(True)
    normals = G[:, :3].reshape(R, S, 3)
    w = dict(w_rgb=1.0, w_eik=0.1, w_edge=1.0, w_smooth=1e-4)
    ref = O.train_loss({"color_fine": color, "normals": normals, "depth_pred": depth}, gt, patch=patch, **w)
    r_grads = torch.autograd.grad(ref, [color, depth, G], allow_unused=True)  # patch 1: depth unused
    r_grads = [torch.zeros_like(t) if gr is None else gr for gr, t in zip(r_grads, (color, depth, G))]
    got = train_losses(color, gt, depth, normals, patch=patch, **w)
    g_grads = torch.autograd.grad(got * 2.0, [color, depth, G])  # upstream gradient scales the inputs'
    assert abs(got.item() - ref.item()) <= 1e-6 * abs(ref.item()), (got.item(), ref.item())
    for a, b, n in zip(g_grads, r_grads, ("color", "depth", "G")):
        torch.testing.assert_close(a, 2.0 * b, rtol=1e-5, atol=1e-9, msg=lambda m: f"{n}: {m}")


def test_patch_indices_distinct_whole_patches():
    """cn_patch_indices (device patch sampling, training.py:413-436): whole ps x ps
    patches at distinct corners inside the image, deterministic per key, and the
    corners of many keys spread uniformly over the corner grid."""
    ops = _ops()
    from copenerf.rays import get_patch_indices
    h, w, ps, n_pts = 540, 960, 4, 4096
    n = (h - ps + 1) * (w - ps + 1)
    key = torch.tensor([1, -2, 3, 12345], dtype=torch.int32, device=DEV)
    a = ops.patch_indices(h, w, ps, n_pts // 16, key)
    assert torch.equal(a, ops.patch_indices(h, w, ps, n_pts // 16, key))
    idx = a.view(-1, 16).cpu()
    corners = idx[:, 0]
    assert corners.unique().numel() == corners.numel()
    offs = torch.tensor([r * w + c for r in range(ps) for c in range(ps)])
    assert torch.equal(idx - corners[:, None], offs.expand_as(idx))
    assert int(idx.max()) < h * w and int((corners % w).max()) <= w - ps and int((corners // w).max()) <= h - ps
    # every corner of a tiny grid is reachable: all n corners when n_patches == n
    full = ops.patch_indices(6, 7, 2, 30, key).view(-1, 4)[:, 0].cpu()
    assert sorted(((full // 7) * 6 + full % 7).tolist()) == list(range(30))
    # uniformity over keys: mean corner id ~ n/2, both halves of the grid drawn equally
    g = torch.Generator(device=DEV).manual_seed(3)
    cs = torch.cat([get_patch_indices(h, w, ps, n_pts, generator=g, device=DEV).view(-1, 16)[:, 0] for _ in range(64)])
    cid = (cs // w) * (w - ps + 1) + cs % w
    frac_low = (cid < n // 2).float().mean().item()
    assert abs(frac_low - 0.5) < 0.02, frac_low


def test_weight_norm_batch_matches_torch():
    """cn_weight_norm (every weight-normed Linear of a network in one launch, forward and
    backward) against torch._weight_norm and its autograd, dim 0."""
    from copenerf.fields import _WeightNormFn
    shapes = [(256, 39), (256, 256), (204, 256), (257, 256), (3, 256), (6, 13)]
    vs = [_rnd(o, i, seed=60 + k).requires_grad_(True) for k, (o, i) in enumerate(shapes)]
    gs = [(_rnd(o, 1, seed=70 + k) + 2.0).requires_grad_(True) for k, (o, i) in enumerate(shapes)]
    ref = [torch._weight_norm(v, g, 0) for v, g in zip(vs, gs)]
    got = _WeightNormFn.apply(len(vs), *vs, *gs)
    for a, b in zip(got, ref):
        torch.testing.assert_close(a, b, rtol=2e-6, atol=1e-7)
    dWs = [_rnd(*w.shape, seed=80 + k) for k, w in enumerate(ref)]
    gr = torch.autograd.grad(ref, vs + gs, dWs)
    gg = torch.autograd.grad(got, vs + gs, dWs)
    for a, b in zip(gg, gr):
        torch.testing.assert_close(a, b, rtol=1e-5, atol=1e-6)
