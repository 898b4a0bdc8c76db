"""cn_mul_chain (ABI v13, bf16 mode): the SDF network's MUL chains in one launch each -- the ∇ₓSDF pass
of the forward (neus_fields.py:291-303) and the first-order adjoint of the backward (the SDF
consistency re-query with pose gradient, train.py:504) -- against the same layers as cn_linear launches
(fields.MUL_CHAIN False): the same bits, since every step is the layer's MUL epilogue on the same
MFMA k order and its output image is the next step's operand either way."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _net(seed=3):
    from copenerf import SDFNetwork
    from helpers import SDF_CFG
    torch.manual_seed(seed)
    net = SDFNetwork(**SDF_CFG).to(DEV)
    net.mfma_dtype = "bf16"
    return net


def _both(fn):
    from copenerf import fields
    saved = fields.MUL_CHAIN
    try:
        out = []
        for on in (True, False):
            fields.MUL_CHAIN = on
            out.append(fn())
        return out
    finally:
        fields.MUL_CHAIN = saved


@pytest.mark.parametrize("M", [4099, 70001])
def test_grad_pass_chain_bitwise(M):
    """∇ₓsdf and the double-backward parameter gradients (which read the ∇ pass's images s_l) with the
    chained ∇ pass equal the layer-by-layer ones; M = 70001 puts several row blocks on each CU and a
    ragged last block."""
    net = _net()
    x = torch.rand(M, 4, device=DEV) * 2 - 1

    def run():
        sdf, feat, g = net.field(x)
        loss = ((g.norm(dim=-1) - 1) ** 2).mean() + sdf.abs().mean() + 1e-2 * feat.square().mean()
        return [sdf.detach(), feat.detach(), g.detach()] + list(torch.autograd.grad(loss, list(net.parameters())))

    a, b = _both(run)
    names = ["sdf", "feat", "grad"] + [n for n, _ in net.named_parameters()]
    for n, u, v in zip(names, a, b):
        assert torch.equal(u, v), (n, (u - v).abs().max().item())


@pytest.mark.parametrize("want_dx", [True, False])
def test_first_order_adjoint_chain_bitwise(want_dx):
    """An sdf-only loss (the consistency term's shape): the first-order adjoint Z_6 .. Z_0 in one launch;
    with dL/dx wanted the skip layer's embedding columns split off (the input gradient shares the chain),
    without it they are zero."""
    net = _net(5)
    x0 = torch.rand(9001, 4, device=DEV) * 2 - 1

    def run():
        x = x0.clone().requires_grad_(want_dx)
        sdf, _, _ = net.field(x, want_feat=False, want_grad=False)
        loss = (sdf.square() * torch.linspace(0.5, 1.5, sdf.shape[0], device=DEV)[:, None]).mean()
        params = list(net.parameters())
        gr = torch.autograd.grad(loss, ([x] if want_dx else []) + params)
        return [sdf.detach()] + list(gr)

    a, b = _both(run)
    for i, (u, v) in enumerate(zip(a, b)):
        assert torch.equal(u, v), (i, (u - v).abs().max().item())


def test_chain_call_matches_linear_steps_with_fp32_outputs():
    """cn_mul_chain called directly on random images (ops.mul_chain) against the same steps as ops.linear
    MULs: every step's image, the fp32 outputs of two steps and the split columns, bitwise."""
    from copenerf import ops
    g = torch.Generator(device="cpu").manual_seed(7)
    M, n = 3001, 4

    def rnd(*s, scale=1.0):
        return ((torch.rand(*s, generator=g) * 2 - 1) * scale).to(DEV)

    src = rnd(M, 256).bfloat16()
    W = [rnd(256, 256, scale=0.1).bfloat16() for _ in range(n)]
    aux = [torch.nn.functional.softplus(rnd(M, 256, scale=0.05), beta=100).bfloat16() for _ in range(n)]
    nsplit = [256, 204, 256, 200]
    adiv = [1.0, ops.SQRT2, 1.0, 1.0]
    splits = [None, torch.full((M, 64), float("nan"), device=DEV), None, None]
    steps, ref_b, ref_f = [], [], []
    for t in range(n):
        ob = torch.full((M, 256), float("nan"), device=DEV).bfloat16()
        of = torch.full((M, 256), float("nan"), device=DEV) if t in (1, 3) else None
        steps.append(dict(W=W[t], aux=aux[t], aux_beta=100.0 * (1.5 if t == 2 else 1.0), adiv=adiv[t], nsplit=nsplit[t],
                          split=splits[t], out_b=ob, out_f=of))
    ops.mul_chain(src, steps)
    A = src
    for t in range(n):
        st = steps[t]
        ob = torch.full((M, 256), float("nan"), device=DEV).bfloat16()
        of = torch.full((M, 256), float("nan"), device=DEV)
        kw = dict(aux0=st["aux"], aux_beta=st["aux_beta"], adiv=st["adiv"], nzero=256, out0_b=ob)
        N = 256
        sp = None
        if st["split"] is not None:
            sp = torch.full((M, 64), float("nan"), device=DEV)
            kw.update(nsplit=st["nsplit"], out_split=sp)
        elif st["nsplit"] < 256:
            N = st["nsplit"]
        ops.linear(A, st["W"], N, 256, of, ops.EPI_MUL, **kw)
        assert torch.equal(st["out_b"].view(torch.int16), ob.view(torch.int16)), t
        if st["out_f"] is not None:
            assert torch.equal(st["out_f"], of), t
        if sp is not None:
            assert torch.equal(st["split"][:, :256 - st["nsplit"]], sp[:, :256 - st["nsplit"]]), t
        A = ob
