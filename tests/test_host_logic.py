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
