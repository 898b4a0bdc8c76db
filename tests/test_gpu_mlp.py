"""cn_mlp_fwd / cn_mlp_bwd (ABI v14): SDFNetwork.sdf under autograd -- the stage-1 consistency re-query of
train.py:502-505 (neus_fields.py:268-283 forward and its backward) -- as two C calls, against the
layer-by-layer composition they replace (fields.sdf_forward keep / sdf_backward sdf-only first order /
sdf_input_grad: fields.MLP_NATIVE off) with the same packs: sdf, dL/dx and every parameter gradient
(through weight norm) bitwise equal, in each GEMM mode, at both network widths (d_hidden 256: the fused
sdf head and the adjoint's column sums; 64: the row head and cn_colsum), with parameter and input
gradients together and each alone.  The composition itself is pinned to the reference by the stage-1
tests (tests/test_gpu_stage1.py runs this path through train_step)."""
import ctypes

import pytest
import torch

from helpers import build_modules

pytestmark = pytest.mark.gpu
DEV = "cuda"
MODES = ["fp32", "bf16x6", "bf16"]


def _run(sdfn, x, g, native, want_x=True, want_params=True):
    from copenerf import fields
    saved = fields.MLP_NATIVE
    fields.MLP_NATIVE = native
    try:
        for p in sdfn.parameters():
            p.grad = None
            p.requires_grad_(want_params)
        xx = x.clone().requires_grad_(want_x)
        sdf = sdfn.sdf(xx)
        (sdf * g).sum().backward()
        torch.cuda.synchronize()
        grads = {k: p.grad for k, p in sdfn.named_parameters()}
        return sdf.detach(), (xx.grad if want_x else None), grads
    finally:
        fields.MLP_NATIVE = saved
        for p in sdfn.parameters():
            p.requires_grad_(True)


def _inputs(M, seed):
    gen = torch.Generator(device=DEV).manual_seed(seed)
    x = torch.cat([torch.rand(M, 3, device=DEV, generator=gen) * 1.6 - 0.8,
                   torch.full((M, 1), 0.3, device=DEV)], 1).contiguous()
    g = torch.randn(M, 1, device=DEV, generator=gen)
    return x, g


@pytest.mark.parametrize("mode", MODES)
@pytest.mark.parametrize("dh", [256, 64])
def test_mlp_equals_composition(mode, dh, monkeypatch):
    from copenerf import ops
    calls = []
    fwd, bwd = ops.mlp_fwd, ops.mlp_bwd
    monkeypatch.setattr(ops, "mlp_fwd", lambda *a, **k: calls.append("f") or fwd(*a, **k))
    monkeypatch.setattr(ops, "mlp_bwd", lambda *a, **k: calls.append("b") or bwd(*a, **k))
    sdfn = build_modules(21, dh_sdf=dh, device=DEV)[0]
    sdfn.mfma_dtype = mode
    for M in (1, 7, 3000, 70001):
        x, g = _inputs(M, M)
        for want_x, want_params in ((True, True), (False, True), (True, False)):
            calls.clear()
            ref = _run(sdfn, x, g, False, want_x, want_params)
            assert not calls
            out = _run(sdfn, x, g, True, want_x, want_params)
            assert calls == ["f", "b"], calls  # the C calls ran
            assert torch.equal(out[0], ref[0])
            if want_x:
                assert torch.equal(out[1], ref[1]), (out[1] - ref[1]).abs().max().item()
            for k, v in ref[2].items():
                if want_params:
                    assert torch.equal(out[2][k], v), (M, want_x, k, (out[2][k] - v).abs().max().item())
                else:
                    assert out[2][k] is None and v is None


def test_mlp_direct_call():
    """Through ctypes: M = 0 writes nothing; the state and the workspace one byte short are refused; the
    feature rows of the last Linear's gradient are zero."""
    from copenerf import _lib, ops
    lib = _lib.load()
    sdfn = build_modules(4, device=DEV)[0]
    sdfn.mfma_dtype = "bf16"
    lay = sdfn.layout()
    with torch.no_grad():
        pk = sdfn.params_and_pack()[2]
    net, keep = ops.sdf_net(lay, pk)
    M = 5000
    x, g = _inputs(M, 9)
    sdf = torch.full((M,), float("nan"), device=DEV)
    d = ops._mlp_desc(net, 0, x=x, sdf=sdf)
    assert lib.cn_mlp_fwd(ctypes.byref(d), None, 0, None) == 0
    d.M = M
    nb = lib.cn_mlp_state_bytes(ctypes.byref(d))
    state = torch.empty(nb, dtype=torch.uint8, device=DEV)
    assert lib.cn_mlp_fwd(ctypes.byref(d), ctypes.c_void_p(state.data_ptr()), nb - 1, None) == -2
    state = ops.mlp_fwd(net, x, sdf)
    with torch.no_grad():
        ref = torch.empty(M, device=DEV)
        ops.sdf_query(ops.sdf_net(lay, pk, layered=True)[0], x, ref)
    torch.cuda.synchronize()
    assert torch.equal(sdf, ref)  # the kept forward is the layer-by-layer query
    dWs = [torch.full((lay.out_dim[l], lay.in_dim[l]), float("nan"), device=DEV) for l in range(lay.n_lin)]
    dbs = [torch.full((lay.out_dim[l],), float("nan"), device=DEV) for l in range(lay.n_lin)]
    dx = torch.empty(M, 4, device=DEV)
    dsdf = g.reshape(-1).contiguous()
    b = ops._mlp_desc(net, M, dsdf=dsdf, dWs=dWs, dbs=dbs, dx=dx)
    ws = lib.cn_mlp_bwd_workspace_bytes(ctypes.byref(b))
    buf = torch.empty(ws, dtype=torch.uint8, device=DEV)
    assert lib.cn_mlp_bwd(ctypes.byref(b), ctypes.c_void_p(state.data_ptr()), state.numel(),
                          ctypes.c_void_p(buf.data_ptr()), ws - 1, None) == -2
    ops.mlp_bwd(net, M, state, dsdf, dWs, dbs, dx)
    torch.cuda.synchronize()
    assert bool(torch.isfinite(dx).all()) and all(bool(torch.isfinite(t).all()) for t in dWs + dbs)
    assert bool((dWs[-1][1:] == 0).all()) and bool((dbs[-1][1:] == 0).all())
    torch.testing.assert_close(dbs[-1][0], dsdf.sum() / lay.scale, rtol=1e-5, atol=1e-4)
    del keep
