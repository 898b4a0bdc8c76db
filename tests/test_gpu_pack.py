"""cn_pack_weights: the weight images of SDFNetwork / RenderingNetwork built in
one launch, against a torch restatement of the same padding / transposition /
column permutation / term split (the packing as plain tensor ops), bit for bit
in every operand mode; and the colour network's column permutation checked
against the reference layer (neus_fields.py:352-356)."""
import pytest
import torch
import torch.nn.functional as F

from helpers import build_modules

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _conv(mode):
    from copenerf import ops
    if mode == "bf16":
        return lambda t: t.to(torch.bfloat16).contiguous()  # noqa: E731
    if mode == "bf16x6":
        return ops.split_bf16x3
    return lambda t: t.contiguous()  # noqa: E731


def _torch_pack_sdf(lay, Ws, mode):
    from copenerf.ops import rup
    kq, cv = (64 if mode == "bf16" else 32), _conv(mode)
    Bf, Bt = [], []
    for l in range(lay.n_lin - 1):
        W = Ws[l].detach()
        o, i = W.shape
        kp = lay.KE if l == 0 else rup(i, kq)
        Bf.append(cv(F.pad(W, (0, kp - i, 0, rup(o, 128) - o))))
        Bt.append(cv(F.pad(W.t(), (0, rup(o, kq) - o, 0, rup(i, 128) - i))))
    Wf = Ws[-1].detach()[1:]
    o, i = Wf.shape
    Bf.append(cv(F.pad(Wf, (0, rup(i, kq) - i, 0, rup(o, 128) - o))))
    Bt.append(cv(F.pad(Wf.t(), (0, rup(o, kq) - o, 0, rup(i, 128) - i))))
    return Bf, Bt


def _torch_pack_color(lay, Ws, mode):
    from copenerf.ops import rup
    kq, cv = (64 if mode == "bf16" else 32), _conv(mode)
    P, V, Gd, Fd = lay.P, lay.V, lay.Gd, lay.F
    W0 = Ws[0].detach()
    o = W0.shape[0]
    pts, emb, g, feat = (W0[:, 0:P], W0[:, P:P + V], W0[:, P + V:P + V + Gd], W0[:, P + V + Gd:])
    ext = torch.cat([g, pts, emb], 1)
    W0k = torch.cat([feat, F.pad(ext, (0, lay.KX - ext.shape[1]))], 1)
    imgs = [cv(F.pad(W0k, (0, 0, 0, rup(o, 128) - o)))]
    for l in range(1, lay.n_lin - 1):
        W = Ws[l].detach()
        oo, ii = W.shape
        imgs.append(cv(F.pad(W, (0, rup(ii, kq) - ii, 0, rup(oo, 128) - oo))))
        imgs.append(cv(F.pad(W.t(), (0, rup(oo, kq) - oo, 0, rup(ii, 128) - ii))))
    imgs.append(cv(F.pad(feat.t(), (0, rup(o, kq) - o, 0, rup(Fd, 128) - Fd))))
    imgs.append(g.t().contiguous())
    imgs.append(cv(F.pad(ext.t(), (0, rup(o, kq) - o, 0, 64 - ext.shape[1]))))
    return imgs


@pytest.mark.parametrize("mode", ["fp32", "bf16", "bf16x6"])
@pytest.mark.parametrize("width", [256, 64])
def test_pack_matches_torch_restatement(mode, width):
    sdf, col, _ = build_modules(5, width, width, device=DEV)
    sdf.mfma_dtype = col.mfma_dtype = mode
    Ws, _, pk = sdf.params_and_pack()
    Bf, Bt = _torch_pack_sdf(sdf.layout(), Ws, mode)
    for a, b in zip(pk.Bf + [pk.Bf8], Bf):
        assert a.shape == b.shape and a.dtype == b.dtype and torch.equal(a, b)
    for a, b in zip(pk.Bt + [pk.Bt8], Bt):
        assert a.shape == b.shape and a.dtype == b.dtype and torch.equal(a, b)
    Wc, _, pc = col.params_and_pack()
    got = [pc.Bf[0]] + [t for l in range(1, len(pc.Bf)) for t in (pc.Bf[l], pc.Bt[l])] + [pc.Btf, pc.Wg, pc.Bxt]
    for a, b in zip(got, _torch_pack_color(col.layout(), Wc, mode)):
        assert a.shape == b.shape and a.dtype == b.dtype and torch.equal(a, b)


def test_pack_sdf_shapes_and_padding():
    sdf, col, dev = build_modules(2, device=DEV)
    Ws, bs, pk = sdf.params_and_pack()
    assert pk.Bf[0].shape == (256, 64) and torch.all(pk.Bf[0][:, 52:] == 0)
    assert pk.Bf[3].shape == (256, 256) and torch.all(pk.Bf[3][204:] == 0)
    assert pk.Bt[3].shape == (256, 224) and torch.all(pk.Bt[3][:, 204:] == 0)
    assert pk.Bt[0].shape == (128, 256) and torch.all(pk.Bt[0][52:] == 0)
    torch.testing.assert_close(pk.w80[0], Ws[8][0].detach())
    torch.testing.assert_close(pk.Bf8, Ws[8][1:].detach())


def test_pack_color_permutation_reproduces_linear():
    """cat([feature, ext]) @ Bf0ᵀ == cat([pts, emb, g, feature]) @ W0ᵀ with ext = [g, pts, emb, 0]."""
    sdf, col, dev = build_modules(3, device=DEV)
    Ws, bs, pk = col.params_and_pack()
    M = 7
    g = torch.Generator().manual_seed(0)
    pts, emb, gr, feat = (torch.randn(M, 4, generator=g), torch.randn(M, 27, generator=g),
                          torch.randn(M, 4, generator=g), torch.randn(M, 256, generator=g))
    pts, emb, gr, feat = (t.to(DEV).double() for t in (pts, emb, gr, feat))
    W0 = Ws[0].detach().double()
    ref = torch.cat([pts, emb, gr, feat], 1) @ W0.t()
    ext = torch.cat([gr, pts, emb, torch.zeros(M, 64 - 35, device=DEV, dtype=torch.float64)], 1)
    got = torch.cat([feat, ext], 1) @ pk.Bf[0][:256].double().t()
    torch.testing.assert_close(got, ref, rtol=1e-10, atol=1e-10)
    # the backward un-permutation used in _ColorFieldFn.backward
    dZ = torch.randn(M, 256, generator=g).to(DEV).double()
    dWf, dWx = dZ.t() @ feat, dZ.t() @ ext
    dW = torch.cat([dWx[:, 4:8], dWx[:, 8:35], dWx[:, 0:4], dWf], 1)
    torch.testing.assert_close(dW, dZ.t() @ torch.cat([pts, emb, gr, feat], 1))
    # dG rows and dfeature columns
    torch.testing.assert_close(dZ @ pk.Wg.double().t(), dZ @ W0[:, 31:35])
    torch.testing.assert_close(dZ @ pk.Btf[:256].double().t(), dZ @ W0[:, 35:])
