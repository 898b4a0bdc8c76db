"""cn_sdf_mlp, the sampler's no-grad SDF query in one launch -- in the bf16 mode (config C3) and, ABI v15, the
fp32-class bf16x6 mode (config C2) -- against the layer-by-layer path it replaces (cn_sdf_embed + nine
cn_linear launches on the same weight images): bitwise equal sdf values -- ragged row counts, more row blocks than CUs (the weight ring and
the persistent loop across blocks), the scattered head (the sampler's merged slots), a perturbed
network (no geometric-init symmetry) -- and the sampler's z-values through NeuSRenderer.sample_z."""
import pytest
import torch

from helpers import REN_CFG, SDF_CFG, build_modules

pytestmark = pytest.mark.gpu
DEV = "cuda"


MODES = ["bf16", "bf16x6"]


def _net(seed, mode="bf16"):
    from copenerf import SDFNetwork
    torch.manual_seed(seed)
    net = SDFNetwork(**SDF_CFG).to(DEV)
    with torch.no_grad():  # off the geometric init: every layer's weights matter
        for p in net.parameters():
            p.add_(0.02 * torch.randn_like(p))
    net.mfma_dtype = mode
    return net


def _query(net, x, fused, sdf_out=None, dst=None):
    from copenerf import fields
    saved = fields.FUSED_SDF_QUERY
    fields.FUSED_SDF_QUERY = fused
    try:
        with torch.no_grad():
            Ws, bs, pk = net.params_and_pack()
            st = fields.sdf_forward(net.layout(), pk, x, want_feat=False, want_grad=False, keep=False,
                                    sdf_out=sdf_out, dst=dst)
        return st["sdf"]
    finally:
        fields.FUSED_SDF_QUERY = saved


@pytest.mark.parametrize("mode", MODES)
@pytest.mark.parametrize("M", [1, 255, 4099, 2 * 256 * 256 + 77])
def test_fused_query_bitwise_equals_layer_by_layer(M, mode):
    from copenerf import fields
    net = _net(3, mode)
    assert fields._fused_query_ok(net.layout(), net.params_and_pack()[2])
    g = torch.Generator(device=DEV).manual_seed(M)
    x = torch.rand(M, 4, device=DEV, generator=g) * 2.4 - 1.2
    a = _query(net, x, True)
    b = _query(net, x, False)
    assert torch.isfinite(a).all()
    assert torch.equal(a, b), (a - b).abs().max().item()


@pytest.mark.parametrize("mode", MODES)
def test_fused_query_scatter_and_fallbacks(mode):
    """The head's scatter into the merged slots (head_idx), and the shapes the kernel does not take
    (the 64-wide network, the exact fp32 MFMA mode) going layer by layer."""
    from copenerf import SDFNetwork, fields
    net = _net(5, mode)
    M = 70001
    x = torch.rand(M, 4, device=DEV) * 2 - 1
    dst = torch.randperm(2 * M, device=DEV)[:M].to(torch.int32)
    a = _query(net, x, True, sdf_out=torch.full((2 * M,), float("nan"), device=DEV), dst=dst)
    b = _query(net, x, False, sdf_out=torch.full((2 * M,), float("nan"), device=DEV), dst=dst)
    assert torch.equal(torch.nan_to_num(a, 9.0), torch.nan_to_num(b, 9.0))
    assert not torch.isnan(a[dst.long()]).any()
    narrow = SDFNetwork(**dict(SDF_CFG, d_hidden=64)).to(DEV)
    narrow.mfma_dtype = mode
    assert not fields._fused_query_ok(narrow.layout(), narrow.params_and_pack()[2])
    net.mfma_dtype = "fp32"
    assert not fields._fused_query_ok(net.layout(), net.params_and_pack()[2])


@pytest.mark.parametrize("mode", MODES)
def test_sampler_z_values_fused_equal_layer_by_layer(mode):
    """NeuSRenderer.sample_z (coarse 64 + 4 rounds of 16, the C2 / C3 sample counts) with the fused query
    and layer by layer: the same z-values bit for bit (the importance samples follow the sdf)."""
    from copenerf import NeuSRenderer, fields
    sdf, col, dev = build_modules(21, device=DEV)
    with torch.no_grad():
        for p in sdf.parameters():
            p.add_(0.01 * torch.randn_like(p))
    r = NeuSRenderer(None, sdf, dev, col, None, **dict(REN_CFG, n_importance=64)).to(DEV).set_mfma_dtype(mode)
    R = 4096
    g = torch.Generator(device=DEV).manual_seed(7)
    o = torch.zeros(R, 3, device=DEV)
    d = torch.cat([(torch.rand(R, 2, device=DEV, generator=g) - 0.5), -torch.ones(R, 1, device=DEV)], -1)
    d = d / d.norm(dim=-1, keepdim=True)
    near, far = torch.full((R, 1), 0.01, device=DEV), torch.full((R, 1), 3.0, device=DEV)
    t = torch.zeros(1, device=DEV)
    t_rand = torch.rand(R, 64, device=DEV, generator=g)
    zs = []
    for fused in (True, False):
        fields.FUSED_SDF_QUERY = fused
        try:
            zs.append(r.sample_z(o, d, t, near, far, 64, 64, t_rand, sdf.params_and_pack()))
        finally:
            fields.FUSED_SDF_QUERY = True
    assert torch.equal(zs[0], zs[1])


@pytest.mark.parametrize("mode", MODES)
def test_fused_query_layer_inputs_match(mode):
    """cn_sdf_mlp's debug dump (every layer's input as its B operand holds it) against the layer-by-layer
    path's operands: layer 0 = the embedding (its image in the bf16 mode), layer l = U_l (its image)."""
    from copenerf import fields, ops
    net = _net(9, mode)
    x6 = mode == "bf16x6"
    dt = torch.float32 if x6 else torch.bfloat16
    lay = net.layout()
    M = 300
    x = torch.rand(M, 4, device=DEV) * 2 - 1
    with torch.no_grad():
        Ws, bs, pk = net.params_and_pack()
        st = fields.sdf_forward(lay, pk, x, want_feat=False, want_grad=False, keep=True)
        u0b = torch.empty(M, 64, device=DEV, dtype=dt)
        tail = torch.empty(M, 64, device=DEV, dtype=dt)
        ops.sdf_embed(x, lay.multires, lay.scale, u0b, tail[:, :lay.E], ops.SQRT2)
        dbg = torch.zeros(8, M, 256, device=DEV, dtype=dt)
        sdf = torch.empty(M, device=DEV)
        ops.sdf_mlp(u0b, tail[:, :lay.E], pk.Bf[:8], pk.b[:8], pk.w80[0], pk.b80, sdf, multires=lay.multires,
                    skip_layer=lay.skip - 1, skip_div=ops.SQRT2, beta=lay.beta, threshold=lay.threshold, debug=dbg)
    refs = [st["U"][l] for l in range(8)] if x6 else [st["U"][0].bfloat16()] + [st["Ub"][l] for l in range(1, 8)]
    report = []
    for l in range(8):
        w = 64 if l == 0 else 256
        a, b = dbg[l, :, :w], refs[l][:, :w]
        bad = (a != b)
        if bad.any():
            cols = bad.any(0).nonzero().flatten()[:24].tolist()
            rows = bad.any(1).nonzero().flatten()[:12].tolist()
            report.append(f"layer {l}: {bad.float().mean().item():.4f} of values differ, cols {cols}, rows {rows}, "
                          f"max |d| {(a.float() - b.float()).abs().max().item():.3g}")
    assert not report, "\n".join(report)
    torch.testing.assert_close(sdf.view(-1, 1), st["sdf"], rtol=0, atol=0)
