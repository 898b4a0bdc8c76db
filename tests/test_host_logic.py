"""Host-side packing logic of the HIP path, checked on the CPU with torch
stand-ins for the kernel contracts (no device needed)."""
import torch

from helpers import build_modules


def test_sdf_layout_default_config():
    sdf, col, dev = build_modules(1)
    lay = sdf.layout()
    assert lay.n_lin == 9 and lay.E == 52 and lay.KE == 64 and lay.HL == 256 and lay.skip == 4
    assert lay.out_dim == [256, 256, 256, 204, 256, 256, 256, 256, 257]
    assert lay.in_dim == [52, 256, 256, 256, 256, 256, 256, 256, 256]
    cl = col.layout()
    assert (cl.F, cl.P, cl.V, cl.Gd, cl.KX) == (256, 4, 27, 4, 64)


def test_pack_sdf_shapes_and_padding():
    sdf, col, dev = build_modules(2)
    Ws, bs, pk = sdf.params_and_pack()
    assert pk.Bf[0].shape == (256, 64) and torch.all(pk.Bf[0][:, 52:] == 0)
    assert pk.Bf[3].shape == (256, 256) and torch.all(pk.Bf[3][204:] == 0)
    assert pk.Bt[3].shape == (256, 224) and torch.all(pk.Bt[3][:, 204:] == 0)
    assert pk.Bt[0].shape == (128, 256) and torch.all(pk.Bt[0][52:] == 0)
    torch.testing.assert_close(pk.w80[0], Ws[8][0].detach())
    torch.testing.assert_close(pk.Bf8, Ws[8][1:].detach())


def test_pack_color_permutation_reproduces_linear():
    """cat([feature, ext]) @ Bf0ᵀ == cat([pts, emb, g, feature]) @ W0ᵀ with ext = [g, pts, emb, 0]."""
    sdf, col, dev = build_modules(3)
    Ws, bs, pk = col.params_and_pack()
    M = 7
    g = torch.Generator().manual_seed(0)
    pts, emb, gr, feat = (torch.randn(M, 4, generator=g), torch.randn(M, 27, generator=g),
                          torch.randn(M, 4, generator=g), torch.randn(M, 256, generator=g))
    ref = torch.cat([pts, emb, gr, feat], 1) @ Ws[0].detach().t()
    ext = torch.cat([gr, pts, emb, torch.zeros(M, 64 - 35)], 1)
    got = torch.cat([feat, ext], 1) @ pk.Bf[0][:256].t()
    torch.testing.assert_close(got, ref, rtol=1e-5, atol=1e-5)
    # the backward un-permutation used in _ColorFieldFn.backward
    dZ = torch.randn(M, 256, generator=g)
    dWf, dWx = dZ.t() @ feat, dZ.t() @ ext
    dW = torch.cat([dWx[:, 4:8], dWx[:, 8:35], dWx[:, 0:4], dWf], 1)
    torch.testing.assert_close(dW, dZ.t() @ torch.cat([pts, emb, gr, feat], 1))
    # dG rows and dfeature columns
    torch.testing.assert_close(dZ @ pk.Wg.t(), dZ @ Ws[0].detach()[:, 31:35])
    torch.testing.assert_close(dZ @ pk.Btf[:256].t(), dZ @ Ws[0].detach()[:, 35:])


def test_state_dict_keys_match_reference_layout():
    sdf, col, dev = build_modules(4)
    keys = list(sdf.state_dict())
    assert keys[:3] == ["lin0.bias", "lin0.weight_g", "lin0.weight_v"] and len(keys) == 27
    assert len(list(col.state_dict())) == 15 and list(dev.state_dict()) == ["variance"]  # 5 Linear layers


def test_inv4x4_matches_lapack_inverse():
    """The capturable cofactor inverse used for ray generation (rays.py) agrees with
    torch.inverse on camera / pose matrices."""
    from copenerf.rays import intrinsics_ndc, inv4x4, make_c2w
    g = torch.Generator().manual_seed(0)
    mats = [intrinsics_ndc(864.0, 864.0, 960, 540), torch.eye(4)]
    for _ in range(8):
        mats.append(make_c2w(torch.randn(3, generator=g), torch.randn(3, generator=g)))
    for m in mats:
        torch.testing.assert_close(inv4x4(m), torch.inverse(m), rtol=1e-5, atol=1e-6)
