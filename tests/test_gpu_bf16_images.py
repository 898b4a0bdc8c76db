"""bf16 MFMA mode (config C3) on the 256-wide tiles and with bf16 operand images (ABI v10).

* The 256x256 bf16 tile equals the 128x128 one bitwise for every epilogue (same K order of the
  same MFMA, same epilogue code), ragged M and N < 256 included.
* A GEMM operand rounds to bf16 when it is staged, so reading its bf16 image instead gives the
  same bits: A / A2 as images, BWD_RELU's aux0 as an image (its sign), and every out0_b / out1_b
  equal to the RNE bf16 of the fp32 values written beside it.
* The bf16 stage-ring weight gradient: the same dW from fp32 operands and from their images,
  batched == per-call within fp32 summation-order noise, against the bf16-rounded operands in
  double.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _rnd(*s, scale=1.0, seed=0):
    g = torch.Generator(device="cpu").manual_seed(seed)
    return ((torch.rand(*s, generator=g) * 2 - 1) * scale).to(DEV)


def _epi_cases(ops, M, N, seed):
    """(name, epilogue, kwargs, out_split) for every epilogue at width N."""
    aux0 = torch.nn.functional.softplus(_rnd(M, 256, seed=seed, scale=0.05), beta=100).contiguous()
    aux1, aux2 = _rnd(M, 256, seed=seed + 1), _rnd(M, 256, seed=seed + 2)
    bias = _rnd(N, seed=seed + 3, scale=0.3)
    sg = dict(aux0=aux0, aux_beta=100.0)
    cases = [("store", ops.EPI_STORE, dict(bias=bias)), ("softplus", ops.EPI_SOFTPLUS, dict(bias=bias)),
             ("relu", ops.EPI_RELU, dict(bias=bias)), ("mul", ops.EPI_MUL, sg), ("tangent", ops.EPI_TANGENT, dict(sg, odiv=1.5)),
             ("bwd_softplus", ops.EPI_BWD_SOFTPLUS, dict(sg, aux1=aux1, aux2=aux2, aux2_scale=100.0)),
             ("bwd_relu", ops.EPI_BWD_RELU, dict(aux0=aux1))]
    if N == 256:
        cases.append(("mul_split", ops.EPI_MUL, dict(sg, nsplit=204, adiv=ops.SQRT2)))
    return cases


def _run(ops, A, Bb, N, K, epi, kw, tile, *, image=False, a_img=False, aux_img=False):
    M = A.shape[0]
    kw = dict(kw)
    out = torch.full((M, 256), float("nan"), device=DEV)
    ob = torch.full((M, 256), float("nan"), device=DEV).bfloat16() if image else None
    split = None
    if "nsplit" in kw:
        split = torch.full((M, 64), float("nan"), device=DEV)
        kw["out_split"] = split
    if aux_img:
        kw["aux0"] = kw["aux0"].bfloat16()
    Ain = A.bfloat16() if a_img else A
    ops.linear(Ain, Bb, N, K, out, epi, nzero=256, tile=tile, out0_b=ob, **kw)
    return out, ob, split


@pytest.mark.parametrize("N", [256, 204])
def test_bf16_sq_tile_equals_128_tile_bitwise(N):
    from copenerf import _lib, ops
    M, K = 5003, 256
    A = _rnd(M, K, seed=1, scale=0.3)
    Bb = torch.zeros(256, K, device=DEV)
    Bb[:N] = _rnd(N, K, seed=2, scale=0.06)
    Bb = Bb.bfloat16().contiguous()
    for name, epi, kw in _epi_cases(ops, M, N, 10):
        d = _lib.LinearDesc()
        d.M, d.N, d.K, d.K1, d.ldb, d.epilogue, d.tile, d.mfma_dtype = M, N, K, K, K, epi, 0, 1
        # the library's 256-wide bf16 tile: 64x128 wave tiles (TM, TN = 2, 4), 32-deep stages
        assert ", 2, 4, 32, " in ops.kernel_name(_lib.load().cn_linear_kernel_name, d), name
        o_sq, _, s_sq = _run(ops, A, Bb, N, K, epi, kw, 0)
        o_t, _, s_t = _run(ops, A, Bb, N, K, epi, kw, 2)
        assert torch.equal(o_sq, o_t) or torch.equal(torch.nan_to_num(o_sq, 7.0), torch.nan_to_num(o_t, 7.0)), name
        if s_sq is not None:
            assert torch.equal(torch.nan_to_num(s_sq, 7.0), torch.nan_to_num(s_t, 7.0)), name


@pytest.mark.parametrize("tile", [0, 2])
def test_bf16_operand_images_bitwise(tile):
    """A as its bf16 image, out0_b beside out0, BWD_RELU's aux0 as an image: the same bits."""
    from copenerf import ops
    M, N, K = 3001, 256, 256
    A = _rnd(M, K, seed=3, scale=0.3)
    Bb = _rnd(N, K, seed=4, scale=0.06).bfloat16().contiguous()
    for name, epi, kw in _epi_cases(ops, M, N, 20):
        ref, _, s_ref = _run(ops, A, Bb, N, K, epi, kw, tile)
        out, ob, s = _run(ops, A, Bb, N, K, epi, kw, tile, image=True, a_img=True,
                          aux_img=(epi == ops.EPI_BWD_RELU))
        assert torch.equal(out, ref), name
        assert torch.equal(ob, ref.bfloat16()), name  # incl. the zero-filled / split columns
        if s is not None:
            assert torch.equal(torch.nan_to_num(s, 7.0), torch.nan_to_num(s_ref, 7.0)), name
    # out0 NULL: the image alone
    ob = torch.empty(M, 256, device=DEV, dtype=torch.bfloat16)
    ops.linear(A.bfloat16(), Bb, N, K, None, ops.EPI_SOFTPLUS, bias=_rnd(N, seed=5), nzero=256, tile=tile, out0_b=ob)
    ref = torch.empty(M, 256, device=DEV)
    ops.linear(A, Bb, N, K, ref, ops.EPI_SOFTPLUS, bias=_rnd(N, seed=5), nzero=256, tile=tile)
    assert torch.equal(ob, ref.bfloat16())


@pytest.mark.parametrize("N", [256, 204, 228])
@pytest.mark.parametrize("tile", [0, 2])
def test_bf16_image_only_outputs_bitwise(N, tile):
    """out0 NULL, the bf16 image alone, for every epilogue (the image-only epilogues zero-fill through
    their v_perm selectors): equal to the image of the fp32 output, incl. the zero-filled columns
    [N, nzero) and MUL's split columns (out_split written as with out0)."""
    from copenerf import ops
    M, K = 3001, 256
    A = _rnd(M, K, seed=43, scale=0.3)
    Bb = torch.zeros(256, K, device=DEV)
    Bb[:N] = _rnd(N, K, seed=44, scale=0.06)
    Bb = Bb.bfloat16().contiguous()
    for name, epi, kw in _epi_cases(ops, M, N, 40):
        ref, _, s_ref = _run(ops, A, Bb, N, K, epi, kw, tile)
        kw = dict(kw)
        split = None
        if "nsplit" in kw:
            split = torch.full((M, 64), float("nan"), device=DEV)
            kw["out_split"] = split
        ob = torch.full((M, 256), float("nan"), device=DEV).bfloat16()
        ops.linear(A.bfloat16(), Bb, N, K, None, epi, nzero=256, tile=tile, out0_b=ob, **kw)
        assert torch.equal(ob, ref.bfloat16()), name
        if split is not None:
            assert torch.equal(torch.nan_to_num(split, 7.0), torch.nan_to_num(s_ref, 7.0)), name


@pytest.mark.parametrize("tile", [0, 2])
def test_bf16_aux_images_bitwise(tile):
    """MUL / TANGENT / BWD_SOFTPLUS / BWD_RELU with every aux operand as a bf16 image equal the same
    epilogues fed the image's values in fp32 (σ recovered from the same activation value, the
    second-order term from the same s and u̇), with A and the outputs as images too."""
    from copenerf import ops
    M, N, K = 3001, 256, 256
    A = _rnd(M, K, seed=23, scale=0.3)
    Bb = _rnd(N, K, seed=24, scale=0.06).bfloat16().contiguous()
    for name, epi, kw in _epi_cases(ops, M, N, 30):
        if "aux0" not in kw:
            continue
        kr = {k: (v.bfloat16().float() if k in ("aux0", "aux1", "aux2") else v) for k, v in kw.items()}
        ki = {k: (v.bfloat16() if k in ("aux0", "aux1", "aux2") else v) for k, v in kw.items()}
        ref, _, s_ref = _run(ops, A, Bb, N, K, epi, kr, tile)
        out, ob, s = _run(ops, A, Bb, N, K, epi, ki, tile, image=True, a_img=True)
        assert torch.equal(out, ref), name
        assert torch.equal(ob, ref.bfloat16()), name
        if s is not None:
            assert torch.equal(torch.nan_to_num(s, 7.0), torch.nan_to_num(s_ref, 7.0)), name
    # one format for BWD_SOFTPLUS's three aux operands
    kw = dict(_epi_cases(ops, M, N, 30)[5][2])
    assert _epi_cases(ops, M, N, 30)[5][0] == "bwd_softplus"
    kw["aux0"] = kw["aux0"].bfloat16()
    with pytest.raises(RuntimeError):
        _run(ops, A, Bb, N, K, ops.EPI_BWD_SOFTPLUS, kw, tile)


def test_bf16_concat_image_and_head():
    """A virtual concat of two images (A | A2), and SOFTPLUS_HEAD's activation / ∇-pass seed images."""
    from copenerf import ops
    M, K1, K2, N = 2049, 256, 64, 256
    A, A2 = _rnd(M, K1, seed=6, scale=0.3), _rnd(M, K2, seed=7, scale=0.3)
    Bb = _rnd(N, K1 + K2, seed=8, scale=0.05).bfloat16().contiguous()
    bias = _rnd(N, seed=9, scale=0.2)
    o = torch.empty(M, N, device=DEV)
    ops.linear(A, Bb, N, K1 + K2, o, ops.EPI_RELU, A2=A2, K1=K1, bias=bias)
    o2 = torch.empty(M, N, device=DEV)
    ob = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    ops.linear(A.bfloat16(), Bb, N, K1 + K2, o2, ops.EPI_RELU, A2=A2.bfloat16(), K1=K1, bias=bias, out0_b=ob)
    assert torch.equal(o, o2) and torch.equal(ob, o.bfloat16())
    Bh = _rnd(N, N, seed=10, scale=0.06).bfloat16().contiguous()
    hw, hb = _rnd(N, seed=11), _rnd(1, seed=12)
    colv = _rnd(N, seed=13)
    res = []
    for img in (False, True):
        a, s1 = torch.empty(M, N, device=DEV), torch.empty(M, N, device=DEV)
        sdf = torch.empty(M, device=DEV)
        ab = torch.empty(M, N, device=DEV, dtype=torch.bfloat16) if img else None
        sb = torch.empty(M, N, device=DEV, dtype=torch.bfloat16) if img else None
        ops.linear(o.bfloat16() if img else o, Bh, N, N, a, ops.EPI_SOFTPLUS_HEAD, bias=bias, out1=s1, colv=colv,
                   aux_beta=100.0, head_w=hw, head_b=hb, head_out=sdf, out0_b=ab, out1_b=sb)
        res.append((a, s1, sdf, ab, sb))
    (a, s1, sdf, _, _), (a2, s2, sdf2, ab, sb) = res
    assert torch.equal(a, a2) and torch.equal(s1, s2) and torch.equal(sdf, sdf2)
    assert torch.equal(ab, a.bfloat16()) and torch.equal(sb, s1.bfloat16())
    # the ∇-pass seed as an image only (out1 NULL): the same image
    sb2 = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    sdf3 = torch.empty(M, device=DEV)
    ops.linear(o.bfloat16(), Bh, N, N, None, ops.EPI_SOFTPLUS_HEAD, bias=bias, colv=colv, aux_beta=100.0,
               head_w=hw, head_b=hb, head_out=sdf3, out0_b=torch.empty_like(sb2), out1_b=sb2)
    assert torch.equal(sb2, sb) and torch.equal(sdf3, sdf)


def test_bf16_dma_tile_across_tiles_bitwise():
    """The LDS-DMA ring of the 256x256 bf16 tile (image A) with more 256-row tiles than CUs, so every
    workgroup runs several tiles and the ring's stages cross tile boundaries (the next tile's first
    chunks under the previous tile's epilogue, its vmcnt(63) wait): the image-only epilogues with the
    fewest memory operations per wave -- STORE / SOFTPLUS (64 image dwords), MUL with its split
    output, SOFTPLUS_HEAD storing only the ∇-pass seed's image, and with no output at all (the
    sampler's sdf-only launch) -- bitwise equal to the 128x128 register-staged tile."""
    from copenerf import _lib, ops
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    M, N, K = 2 * 256 * cus + 37, 256, 256
    A = _rnd(M, K, seed=51, scale=0.3).bfloat16()
    Bb = _rnd(N, K, seed=52, scale=0.06).bfloat16().contiguous()
    bias = _rnd(N, seed=53, scale=0.3)
    d = _lib.LinearDesc()
    d.M, d.N, d.K, d.K1, d.ldb, d.epilogue, d.tile, d.mfma_dtype, d.a_bf16 = M, N, K, K, K, ops.EPI_STORE, 0, 1, 1
    assert ", 2, 4, 32, " in ops.kernel_name(_lib.load().cn_linear_kernel_name, d)
    aux0 = torch.nn.functional.softplus(_rnd(M, 256, seed=54, scale=0.05), beta=100).bfloat16()
    for name, epi, kw in (("store", ops.EPI_STORE, dict(bias=bias)), ("softplus", ops.EPI_SOFTPLUS, dict(bias=bias)),
                          ("mul_split", ops.EPI_MUL, dict(aux0=aux0, aux_beta=100.0, nsplit=204, adiv=ops.SQRT2))):
        outs = []
        for tile in (0, 2):
            k2 = dict(kw)
            split = None
            if "nsplit" in k2:
                split = torch.full((M, 64), float("nan"), device=DEV)
                k2["out_split"] = split
            ob = torch.full((M, 256), float("nan"), device=DEV).bfloat16()
            ops.linear(A, Bb, N, K, None, epi, nzero=256, tile=tile, out0_b=ob, **k2)
            outs.append((ob, split))
        assert torch.equal(outs[0][0], outs[1][0]), name
        if outs[0][1] is not None:
            assert torch.equal(torch.nan_to_num(outs[0][1], 7.0), torch.nan_to_num(outs[1][1], 7.0)), name
    # SOFTPLUS_HEAD spans whole rows only on the 256-wide tile: the reference is the same kernel over
    # row blocks of at most one tile per workgroup (rows are independent)
    hw, hb, colv = _rnd(N, seed=55), _rnd(1, seed=56), _rnd(N, seed=57)
    step = 256 * (cus // 2)
    for seed_only in (True, False):
        res = []
        for blocks in (False, True):
            sdf = torch.full((M,), float("nan"), device=DEV)
            sb = torch.full((M, 256), float("nan"), device=DEV).bfloat16() if seed_only else None
            for r0 in (range(0, M, step) if blocks else [0]):
                r1 = min(M, r0 + step) if blocks else M
                ops.linear(A[r0:r1], Bb, N, K, None, ops.EPI_SOFTPLUS_HEAD, bias=bias,
                           colv=colv if seed_only else None, aux_beta=100.0, head_w=hw, head_b=hb,
                           head_out=sdf[r0:r1], out1_b=sb[r0:r1] if seed_only else None)
            res.append((sdf, sb))
        assert not torch.isnan(res[0][0]).any()
        assert torch.equal(res[0][0], res[1][0]), seed_only
        if seed_only:
            assert torch.equal(res[0][1], res[1][1])


@pytest.mark.parametrize("M,pairs", [(70001, 2), (4097, 1), (33, 2)])
def test_wgrad_bf16_ring_images(M, pairs):
    """The bf16 stage-ring weight gradient from fp32 operands and from their bf16 images: dW bitwise
    equal (the same rounded products in the same order); db from the images sums their bf16 values;
    both against the rounded operands in double; batched (one launch) against per-call."""
    from copenerf import ops
    N = K = 256
    Y0, X0 = _rnd(M, N, seed=15), _rnd(M, K, seed=16)
    Y1, X1 = (_rnd(M, N, seed=17), _rnd(M, K, seed=18)) if pairs == 2 else (None, None)
    b = lambda t: None if t is None else t.bfloat16()  # noqa: E731
    dW, db = torch.empty(N, K, device=DEV), torch.empty(N, device=DEV)
    ops.wgrad(Y0, X0, N, K, dW, db=db, Y1=Y1, X1=X1, mode="bf16")
    dWi, dbi = torch.empty(N, K, device=DEV), torch.empty(N, device=DEV)
    ops.wgrad(b(Y0), b(X0), N, K, dWi, db=dbi, Y1=b(Y1), X1=b(X1), mode="bf16")
    assert torch.equal(dW, dWi)
    r = lambda t: t.bfloat16().double()  # noqa: E731
    ref = r(Y0).t() @ r(X0)
    if pairs == 2:
        ref = ref + r(Y1).t() @ r(X1)
    tol = 1e-6 * M ** 0.5 + 1e-5
    torch.testing.assert_close(dW, ref.float(), rtol=1e-4, atol=tol)
    torch.testing.assert_close(db, Y0.double().sum(0).float(), rtol=1e-4, atol=tol)
    torch.testing.assert_close(dbi, r(Y0).sum(0).float(), rtol=1e-4, atol=tol)
    # mixed sides: Y an image, X fp32
    dWm = torch.empty(N, K, device=DEV)
    ops.wgrad(b(Y0), X0, N, K, dWm, Y1=b(Y1), X1=X1, mode="bf16")
    assert torch.equal(dW, dWm)
    # batched with a second job (each its share of the workgroups) vs per call
    q = ops.WgradQueue()
    dWq, dbq = torch.empty(N, K, device=DEV), torch.empty(N, device=DEV)
    dW2, dW2r = torch.empty(N, K, device=DEV), torch.empty(N, K, device=DEV)
    q.add(b(Y0), b(X0), N, K, dWq, db=dbq, Y1=b(Y1), X1=b(X1), mode="bf16")
    q.add(b(X0), b(Y0), N, K, dW2, mode="bf16")
    q.flush()
    ops.wgrad(b(X0), b(Y0), N, K, dW2r, mode="bf16")
    torch.testing.assert_close(dWq, dWi, rtol=1e-5, atol=tol)
    torch.testing.assert_close(dbq, dbi, rtol=1e-5, atol=tol)
    torch.testing.assert_close(dW2, dW2r, rtol=1e-5, atol=tol)


def test_sdf_field_bf16_images_match_fp32_operand_path():
    """The SDF field in bf16 mode (every hidden activation / adjoint read as a bf16 image) against the
    same field with the images' fp32 sources as operands (the kernels round those the same way): sdf
    and feature bitwise; ∇ₓsdf and the parameter gradients of a double-backward loss within bf16
    rounding: the mode keeps the hidden activations as images only, so σ is recovered from the bf16
    activation, and it stores the ∇-pass adjoints s and the tangents u̇ in bf16 for the adjoint's
    second-order term (db sums the bf16 adjoint images)."""
    from copenerf import SDFNetwork, fields
    from helpers import SDF_CFG
    torch.manual_seed(3)
    net = SDFNetwork(**SDF_CFG).to(DEV)
    net.mfma_dtype = "bf16"
    x = torch.rand(4099, 4, device=DEV) * 2 - 1
    res = []
    saved = fields._img_mode
    try:
        for img in (True, False):
            fields._img_mode = (lambda pk, lay: saved(pk, lay)) if img else (lambda pk, lay: False)
            sdf, feat, g = net.field(x)
            loss = ((g.norm(dim=-1) - 1) ** 2).mean() + sdf.abs().mean() + 1e-2 * feat.square().mean()
            grads = torch.autograd.grad(loss, list(net.parameters()))
            res.append([sdf.detach(), feat.detach(), g.detach()] + list(grads))
    finally:
        fields._img_mode = saved
    names = ["sdf", "feat", "grad"] + [n for n, _ in net.named_parameters()]
    for n, a, b in zip(names, res[0], res[1]):
        if n in ("sdf", "feat"):
            assert torch.equal(a, b), n
        elif n == "grad":
            rel = ((a - b).norm() / b.norm()).item()
            print(f"grad: relative L2 {rel:.2e}")
            assert rel <= 5e-3, rel
        else:
            rel = ((a - b).norm() / b.norm().clamp_min(1e-30)).item()
            print(f"{n}: relative L2 {rel:.2e}")
            assert rel <= 2e-2, (n, rel)


def test_color_bf16_images_match_fp32_operand_path():
    """The colour network in bf16 mode: hidden activations and adjoints as bf16 images vs their fp32
    sources as operands -- rgb and every gradient (points, normals, directions, feature, weights)
    bitwise; the biases whose adjoint is an image within bf16 rounding."""
    from copenerf import RenderingNetwork, fields
    from copenerf.train_step import COL_CFG
    torch.manual_seed(11)
    net = RenderingNetwork(**COL_CFG).to(DEV)
    net.mfma_dtype = "bf16"
    M = 5003
    pts = torch.rand(M, 4, device=DEV, requires_grad=True)
    nrm = torch.randn(M, 4, device=DEV, requires_grad=True)
    dirs = torch.randn(M, 3, device=DEV, requires_grad=True)
    feat = (0.1 * torch.randn(M, 256, device=DEV)).requires_grad_(True)
    res = []
    saved = fields._img_mode
    try:
        for img in (True, False):
            fields._img_mode = (lambda pk, lay: saved(pk, lay)) if img else (lambda pk, lay: False)
            rgb = net(pts, nrm, dirs, feat)
            loss = (rgb * torch.linspace(0.5, 1.5, 3, device=DEV)).square().sum()
            grads = torch.autograd.grad(loss, [pts, nrm, dirs, feat] + list(net.parameters()))
            res.append([rgb.detach()] + list(grads))
    finally:
        fields._img_mode = saved
    names = ["rgb", "pts", "nrm", "dirs", "feat"] + [n for n, _ in net.named_parameters()]
    for n, a, b in zip(names, res[0], res[1]):
        if n in ("lin1.bias", "lin2.bias", "lin3.bias"):  # (the adjoints that are images: bias sums of bf16 values)
            torch.testing.assert_close(a, b, rtol=1e-2, atol=1e-2 * b.abs().max().item() + 1e-6)
        else:
            assert torch.equal(a, b), n
