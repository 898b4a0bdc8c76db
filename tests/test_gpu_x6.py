"""fp32 GEMMs on the bf16 MFMA (CN_MFMA_F32_BF16X6): both operands split into
three bf16 terms, the six term products with i + j <= 2 accumulated in fp32.

The bar is the native fp32 MFMA path's own accuracy: against a float64 GEMM of
the unrounded fp32 operands, the split path's error must stay within a small
factor of the exact-product fp32 MFMA's error on the same inputs, every
epilogue and both tiles.  (Renderer-level parity of this mode against the
reference golden vectors and the oracle at |Δ| <= 1e-4 runs in
test_gpu_render.py, parametrized over FP32_MODES.)"""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _rnd(*s, scale=1.0, seed=0):
    g = torch.Generator(device="cpu").manual_seed(seed)
    return ((torch.rand(*s, generator=g) * 2 - 1) * scale).to(DEV)


def test_split_terms_reconstruct():
    from copenerf import ops
    W = _rnd(256, 320, seed=1) * torch.logspace(-6, 3, 320, device=DEV)
    S = ops.split_bf16x3(W)
    assert S.shape == (20, 256, 48) and S.dtype == torch.bfloat16
    T = ops.unsplit_bf16x3(S)
    assert torch.equal(T[0], W.to(torch.bfloat16))
    rec = T[0].double() + T[1].double() + T[2].double()
    rel = ((rec - W.double()).abs() / W.double().abs().clamp_min(1e-30)).max().item()
    assert rel <= 2.0 ** -26, rel


@pytest.mark.parametrize("M,N,K,tile", [(1000, 256, 256, 0), (130, 204, 256, 0), (777, 52, 256, 1),
                                        (64, 256, 64, 0), (4096, 128, 192, 0), (300, 64, 288, 1)])
def test_linear_x6_store_matches_fp32_accuracy(M, N, K, tile):
    from copenerf import ops
    A = _rnd(M, K, seed=2)
    bn = 64 if tile else 128
    B = torch.zeros(ops.rup(N, bn), K, device=DEV)
    B[:N] = _rnd(N, K, seed=3, scale=0.1)
    bias = _rnd(N, seed=4)
    ld = ops.rup(N, bn)
    exact = A.double() @ B[:N].double().t() + bias.double()
    o32 = torch.empty(M, ld, device=DEV)
    ops.linear(A, B, N, K, o32, ops.EPI_STORE, bias=bias, nzero=ld, tile=tile)
    o6 = torch.full((M, ld), float("nan"), device=DEV)
    ops.linear(A, ops.split_bf16x3(B), N, K, o6, ops.EPI_STORE, bias=bias, nzero=ld, tile=tile)
    e32 = (o32[:, :N].double() - exact).abs()
    e6 = (o6[:, :N].double() - exact).abs()
    scale = exact.abs().max().item()
    print(f"fp32 MFMA max {e32.max().item():.3e} mean {e32.mean().item():.3e} | "
          f"bf16x6 max {e6.max().item():.3e} mean {e6.mean().item():.3e} (|C| max {scale:.2f})")
    assert e6.max().item() <= 2.0 * e32.max().item() + 1e-7 * scale
    assert e6.mean().item() <= 1.5 * e32.mean().item() + 1e-8 * scale
    assert torch.all(o6[:, N:] == 0)


def test_linear_x6_epilogues_and_concat():
    from copenerf import ops
    M, K1, K2, N = 517, 256, 64, 256
    A, A2 = _rnd(M, K1, seed=5, scale=0.3), _rnd(M, K2, seed=6, scale=0.3)
    B = _rnd(N, K1 + K2, seed=7, scale=0.05)
    Bs = ops.split_bf16x3(B)
    bias = _rnd(N, seed=8, scale=0.3)
    aux0 = torch.nn.functional.softplus(_rnd(M, N, seed=9, scale=0.05), beta=100)
    aux1, aux2 = _rnd(M, N, seed=10), _rnd(M, N, seed=11)
    sg = dict(aux0=aux0, aux_beta=100.0)
    for epi, kw in ((ops.EPI_SOFTPLUS, dict(bias=bias)), (ops.EPI_TANGENT, dict(sg)),
                    (ops.EPI_BWD_SOFTPLUS, dict(sg, aux1=aux1, aux2=aux2, aux2_scale=100.0)),
                    (ops.EPI_RELU, dict(bias=bias)), (ops.EPI_MUL, dict(sg)), (ops.EPI_BWD_RELU, dict(aux0=aux1))):
        outs = []
        for Bimg in (B, Bs):
            o0 = torch.empty(M, N, device=DEV)
            ops.linear(A, Bimg, N, K1 + K2, o0, epi, A2=A2, K1=K1, **kw)
            outs.append(o0)
        a0, b0 = outs
        torch.testing.assert_close(b0, a0, rtol=2e-5, atol=2e-6 if epi != ops.EPI_BWD_SOFTPLUS else 2e-4)


def test_sdf_field_x6_gradients_match_fp32():
    """SDF forward, ∇ₓSDF and the double backward in bf16x6 mode against the fp32
    mode on the same weights and points."""
    from copenerf import SDFNetwork
    from helpers import SDF_CFG
    torch.manual_seed(3)
    net = SDFNetwork(**SDF_CFG).to(DEV)
    x = (torch.rand(8192, 4, device=DEV) * 2 - 1)
    res = {}
    for mode in ("fp32", "bf16x6"):
        net.mfma_dtype = mode
        sdf, feat, g = net.field(x)
        loss = ((g.norm(dim=-1) - 1) ** 2).mean() + sdf.abs().mean() + 1e-2 * feat.square().mean()
        grads = torch.autograd.grad(loss, list(net.parameters()))
        res[mode] = (sdf.detach(), g.detach(), grads)
    a, b = res["fp32"], res["bf16x6"]
    torch.testing.assert_close(b[0], a[0], rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(b[1], a[1], rtol=1e-4, atol=1e-4)
    for ga, gb in zip(a[2], b[2]):
        torch.testing.assert_close(gb, ga, rtol=1e-3, atol=1e-5 * (ga.abs().max().item() + 1e-6))


@pytest.mark.parametrize("M,N,K,pairs", [(70000, 256, 256, 2), (1000, 204, 64, 1), (5, 256, 256, 1),
                                         (4097, 256, 320, 1), (300, 52, 192, 2), (33, 128, 128, 2),
                                         (2000, 256, 512, 2), (3000, 204, 256, 2), (70001, 256, 64, 2)])
def test_wgrad_x6_matches_fp32_accuracy(M, N, K, pairs):
    """cn_wgrad in bf16x6 mode: dW's error against float64 within a small factor
    of the exact fp32 MFMA kernel's on the same inputs; db (summed from the fp32
    values in both modes) within fp32 rounding; deterministic."""
    from copenerf import ops
    ldn, ldk = ops.rup(N, 128), ops.rup(K, 128 if K % 128 == 0 else 64)
    if (N, K) == (204, 256):  # 256-wide rows: the 256x256 tile with padding columns (set to garbage)
        ldn = 256
    Y0, X0 = _rnd(M, ldn, seed=15), _rnd(M, ldk, seed=16)
    Y1, X1 = (_rnd(M, ldn, seed=17), _rnd(M, ldk, seed=18)) if pairs == 2 else (None, None)
    exact = Y0[:, :N].double().t() @ X0[:, :K].double()
    if pairs == 2:
        exact = exact + Y1[:, :N].double().t() @ X1[:, :K].double()
    res = {}
    for mode in ("fp32", "bf16x6"):
        dW = torch.empty(N, K, device=DEV)
        db = torch.empty(N, device=DEV)
        ops.wgrad(Y0, X0, N, K, dW, db=db, Y1=Y1, X1=X1, mode=mode)
        res[mode] = (dW, db)
    e32 = (res["fp32"][0].double() - exact).abs()
    e6 = (res["bf16x6"][0].double() - exact).abs()
    scale = exact.abs().max().item() + 1e-30
    print(f"wgrad fp32 max {e32.max().item():.3e} | bf16x6 max {e6.max().item():.3e} (|dW| max {scale:.2f})")
    assert e6.max().item() <= 2.0 * e32.max().item() + 1e-7 * scale
    assert e6.mean().item() <= 1.5 * e32.mean().item() + 1e-8 * scale
    tol = 1e-6 * M ** 0.5 + 1e-5
    torch.testing.assert_close(res["bf16x6"][1], Y0[:, :N].double().sum(0).float(), rtol=1e-4, atol=tol)
    dW2 = torch.empty_like(res["bf16x6"][0])
    ops.wgrad(Y0, X0, N, K, dW2, Y1=Y1, X1=X1, mode="bf16x6")
    assert torch.equal(dW2, res["bf16x6"][0])


@pytest.mark.parametrize("nzero", [204, 256])
def test_linear_x6_narrow_n_on_the_wide_tile(nzero):
    """128 < N < 256 (the 204-wide layer before the skip) on the 256x256 tile: columns < N
    equal the exact-fp32 mode's, [N, nzero) are zero-filled and columns >= nzero (the
    skip input's embedding in the real layout) are never written."""
    from copenerf import ops
    M, N, K = 1537, 204, 256
    A = _rnd(M, K, seed=21, scale=0.3)
    B = torch.zeros(256, K, device=DEV)
    B[:N] = _rnd(N, K, seed=22, scale=0.05)
    Bs = ops.split_bf16x3(B)
    bias = _rnd(N, seed=23, scale=0.3)
    aux0 = torch.nn.functional.softplus(_rnd(M, 256, seed=24, scale=0.05), beta=100)
    sg = dict(aux0=aux0, aux_beta=100.0)
    for epi, kw in ((ops.EPI_SOFTPLUS, dict(bias=bias, odiv=ops.SQRT2)), (ops.EPI_STORE, dict(bias=bias)),
                    (ops.EPI_RELU, dict(bias=bias)), (ops.EPI_TANGENT, dict(sg, odiv=ops.SQRT2)),
                    (ops.EPI_MUL, dict(sg)), (ops.EPI_BWD_RELU, dict(aux0=aux0 - 0.005))):
        outs = []
        for Bimg in (B, Bs):
            o = torch.full((M, 256), 7.0, device=DEV)
            ops.linear(A, Bimg, N, K, o, epi, nzero=nzero, **kw)
            outs.append(o)
        ref, got = outs
        torch.testing.assert_close(got[:, :N], ref[:, :N], rtol=2e-5, atol=2e-6, msg=lambda m: f"epi {epi}: {m}")
        assert torch.all(got[:, N:nzero] == 0), epi
        assert torch.all(got[:, nzero:] == 7.0), epi


def test_wgrad_batch_matches_single_calls():
    """cn_wgrad_batch (ops.WgradQueue): the stage-ring jobs share one launch and one slab
    reduction, each with its share of the workgroups; every job's dW / db equals its own
    cn_wgrad call's up to the summation order (fewer, longer M-slices): within fp32
    rounding of the float64 products (longer slices: see the bar), and bitwise repeatable.  Jobs: C2-shape two-pair and
    one-pair 256x256 layers, two output tiles (K = 512), a ragged M, a 204-wide layer on
    256-wide rows and a K = 64 first layer (another tile class: launched at add())."""
    from copenerf import ops
    specs = [(70000, 256, 256, 2, 256), (70000, 256, 256, 1, 256), (5000, 256, 512, 2, 512),
             (1001, 256, 256, 1, 256), (3000, 204, 256, 2, 256), (20000, 256, 64, 2, 64)]
    jobs = []
    for i, (M, N, K, pairs, ldk) in enumerate(specs):
        Y0, X0 = _rnd(M, 256, seed=40 + 4 * i), _rnd(M, ldk, seed=41 + 4 * i)
        Y1, X1 = (_rnd(M, 256, seed=42 + 4 * i), _rnd(M, ldk, seed=43 + 4 * i)) if pairs == 2 else (None, None)
        jobs.append((Y0, X0, Y1, X1, N, K))

    def run_batch():
        q = ops.WgradQueue()
        outs = []
        for Y0, X0, Y1, X1, N, K in jobs:
            dW, db = torch.full((N, K), float("nan"), device=DEV), torch.full((N,), float("nan"), device=DEV)
            q.add(Y0, X0, N, K, dW, db=db, Y1=Y1, X1=X1, mode="bf16x6")
            outs.append((dW, db))
        q.flush()
        return outs

    got = run_batch()
    again = run_batch()
    for (Y0, X0, Y1, X1, N, K), (dW, db), (dW2, db2) in zip(jobs, got, again):
        ref, rb = torch.empty(N, K, device=DEV), torch.empty(N, device=DEV)
        ops.wgrad(Y0, X0, N, K, ref, db=rb, Y1=Y1, X1=X1, mode="bf16x6")
        exact = Y0[:, :N].double().t() @ X0[:, :K].double()
        if Y1 is not None:
            exact = exact + Y1[:, :N].double().t() @ X1[:, :K].double()
        scale = exact.abs().max().item()
        e_single = (ref.double() - exact).abs().max().item()
        e_batch = (dW.double() - exact).abs().max().item()
        print(f"M={Y0.shape[0]} N={N} K={K}: single {e_single:.3e} batch {e_batch:.3e} (|dW| max {scale:.1f})")
        assert torch.isfinite(dW).all() and torch.isfinite(db).all()
        # fewer, longer M-slices: each slice's fp32 accumulation runs over more rows (C2's 7-job
        # SDF batch: 36 slices of 14,592 rows instead of 256 of 2,048), so the error may grow by
        # about the square root of the length ratio -- still ~1e-6 of |dW|, fp32 class
        assert e_batch <= 4.0 * e_single + 1e-7 * scale and e_batch <= 4e-6 * scale
        torch.testing.assert_close(db, rb, rtol=1e-5, atol=1e-6 * Y0.shape[0] ** 0.5)
        assert torch.equal(dW, dW2) and torch.equal(db, db2)


def test_linear_x6_mul_split_on_the_wide_tile():
    """The skip layer's ∇-pass MUL with a split output (neus_fields.py:276-277: the input adjoint's
    embedding columns go out raw) on the 256x256 tile's direct epilogue: columns < nsplit are
    (A·Bᵀ)/adiv ⊙ σ, [nsplit, 256) of out0 are zero, the split buffer's first N - nsplit columns
    hold the raw product and its tail is untouched; ragged M."""
    from copenerf import _lib, ops
    M, N, K = 1537, 256, 256
    A = _rnd(M, K, seed=31)
    W = _rnd(N, K, seed=32, scale=0.1)
    B = ops.split_bf16x3(W)
    ab = 100.0 * ops.SQRT2
    aux0 = (torch.nn.functional.softplus(_rnd(M, N, seed=33, scale=0.05), beta=100) / ops.SQRT2).contiguous()
    sg = -torch.expm1(-ab * aux0.double())
    out = torch.full((M, 256), float("nan"), device=DEV)
    split = torch.full((M, 64), float("nan"), device=DEV)
    d = _lib.LinearDesc()
    d.M, d.N, d.K, d.K1, d.ldb, d.epilogue, d.tile, d.mfma_dtype = M, N, K, K, B.shape[1], ops.EPI_MUL, 0, 2
    d.out_split, d.nsplit = 16, 204
    assert "linear_kernel<4, 2, 2, 4, 16, 1, 2, 3," in ops.kernel_name(_lib.load().cn_linear_kernel_name, d)
    ops.linear(A, B, N, K, out, ops.EPI_MUL, aux0=aux0, aux_beta=ab, nsplit=204, out_split=split, nzero=256,
               adiv=ops.SQRT2)
    v = A.double() @ W.double().t() / ops.SQRT2
    torch.testing.assert_close(out[:, :204], (v * sg)[:, :204].float(), rtol=2e-5, atol=2e-6)
    assert torch.all(out[:, 204:] == 0)
    torch.testing.assert_close(split[:, :52], v[:, 204:].float(), rtol=2e-5, atol=2e-6)
    assert torch.isnan(split[:, 52:]).all()
