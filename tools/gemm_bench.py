"""Microbenchmark of cn_linear / cn_wgrad at the C2 layer shape against
torch.matmul (hipBLASLt fp32) on the same device: TFLOP/s per variant."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "cope-nerf_amd"), ROOT]
from copenerf import ops  # noqa: E402


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters


ONLY = os.environ.get("ONLY", "")  # substring filter on the variant names


def bench(res, key, fn, div=1):
    if ONLY in key:
        res[key] = timeit(fn) / div


def linear_x6_aimg(As, M, B, N, K, out0, epi, bias=None, aux0=None, aux1=None, aux2=None, aux_beta=0.0,
                   aux2_scale=0.0):
    """cn_linear with A given as a bf16x6 term image (a_bf16 in the bf16x6 mode: a measurement build's switch)."""
    import ctypes  # noqa: F401
    from copenerf import _lib
    d = _lib.LinearDesc()
    d.A, d.B, d.bias = As.data_ptr(), B.data_ptr(), ops._ptr(bias)
    d.aux0, d.aux1, d.aux2 = ops._ptr(aux0), ops._ptr(aux1), ops._ptr(aux2)
    d.ld_aux0, d.ld_aux1, d.ld_aux2 = ops._ld(aux0), ops._ld(aux1), ops._ld(aux2)
    d.aux_beta, d.aux2_scale = aux_beta, aux2_scale
    d.out0, d.ld_out0 = out0.data_ptr(), out0.stride(0)
    d.lda, d.ldb = As.shape[1], B.shape[1]
    d.M, d.N, d.K, d.K1, d.nzero, d.nsplit = M, N, K, K, N, N
    d.epilogue, d.tile, d.adiv, d.odiv, d.beta, d.threshold = epi, 0, 1.0, 1.0, 100.0, 20.0
    d.mfma_dtype, d.a_bf16 = 2, 1
    _lib.check(_lib.load().cn_linear(d, ops._stream()), "cn_linear (x6 A image)")


def main():
    M = int(os.environ.get("M", 524288))
    N = K = 256
    dev = "cuda"
    A = torch.randn(M, K, device=dev) * 0.1
    B = torch.randn(N, K, device=dev) * 0.05
    bias = torch.randn(N, device=dev) * 0.1
    aux0 = torch.rand(M, N, device=dev) * 0.02  # softplus activations: sg = 1 - exp(-100 aux0)
    aux1 = torch.randn(M, N, device=dev)
    aux2 = torch.randn(M, N, device=dev)
    o0 = torch.empty(M, N, device=dev)
    sg = dict(aux0=aux0, aux_beta=100.0)
    so = dict(sg, aux1=aux1, aux2=aux2, aux2_scale=100.0)
    fl = 2.0 * M * N * K
    res = {}
    bench(res, "torch.matmul (hipBLASLt)", lambda: torch.matmul(A, B.t(), out=o0))
    bench(res, "torch addmm+softplus", lambda: torch.nn.functional.softplus(torch.addmm(bias, A, B.t()), beta=100))
    for name, epi, kw in (("store", ops.EPI_STORE, dict(bias=bias)),
                          ("softplus", ops.EPI_SOFTPLUS, dict(bias=bias)),
                          ("mul", ops.EPI_MUL, sg),
                          ("tangent", ops.EPI_TANGENT, sg),
                          ("bwd_softplus", ops.EPI_BWD_SOFTPLUS, so),
                          ("relu", ops.EPI_RELU, dict(bias=bias))):
        bench(res, "cn_linear " + name, lambda: ops.linear(A, B, N, K, o0, epi, **kw))
    Bb = B.bfloat16().contiguous()
    for name, epi, kw in (("store", ops.EPI_STORE, dict(bias=bias)),
                          ("softplus", ops.EPI_SOFTPLUS, dict(bias=bias)),
                          ("tangent", ops.EPI_TANGENT, sg)):
        bench(res, "cn_linear bf16 " + name, lambda: ops.linear(A, Bb, N, K, o0, epi, **kw))
    # bf16 mode with operand images (config C3): A, aux and the output as bf16 images
    Ai, ob = A.bfloat16(), torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    sgi = dict(aux0=aux0.bfloat16(), aux_beta=100.0)
    soi = dict(sgi, aux1=aux1.bfloat16(), aux2=aux2.bfloat16(), aux2_scale=100.0)
    for name, epi, kw in (("store", ops.EPI_STORE, dict(bias=bias)),
                          ("softplus", ops.EPI_SOFTPLUS, dict(bias=bias)),
                          ("relu", ops.EPI_RELU, dict(bias=bias)),
                          ("mul", ops.EPI_MUL, sgi),
                          ("tangent", ops.EPI_TANGENT, sgi),
                          ("bwd_softplus", ops.EPI_BWD_SOFTPLUS, soi),
                          ("bwd_relu", ops.EPI_BWD_RELU, dict(aux0=aux1.bfloat16()))):
        bench(res, "cn_linear img " + name, lambda: ops.linear(Ai, Bb, N, K, None, epi, out0_b=ob, **kw))
    Bs = ops.split_bf16x3(B)
    for name, epi, kw in (("store", ops.EPI_STORE, dict(bias=bias)),
                          ("softplus", ops.EPI_SOFTPLUS, dict(bias=bias)),
                          ("relu", ops.EPI_RELU, dict(bias=bias)),
                          ("mul", ops.EPI_MUL, sg),
                          ("tangent", ops.EPI_TANGENT, sg),
                          ("bwd_softplus", ops.EPI_BWD_SOFTPLUS, so),
                          # (stream-count probes: aux2 = aux1 -- two distinct aux streams; no aux1 / aux2 -- one)
                          ("bwd_softplus_2str", ops.EPI_BWD_SOFTPLUS, dict(so, aux2=aux1)),
                          ("bwd_softplus_1str", ops.EPI_BWD_SOFTPLUS, sg)):
        bench(res, "cn_linear x6 " + name, lambda: ops.linear(A, Bs, N, K, o0, epi, **kw))
    if os.environ.get("X6_AIMG"):  # (a -DCN_AB_X6_AIMG=1 library) A as a bf16x6 term image, no split while staging
        As = ops.split_bf16x3(A)  # [K/16, M, 48]: the layout of B's images
        for name, epi, kw in (("store", ops.EPI_STORE, dict(bias=bias)),
                              ("softplus", ops.EPI_SOFTPLUS, dict(bias=bias)),
                              ("relu", ops.EPI_RELU, dict(bias=bias)),
                              ("mul", ops.EPI_MUL, sg),
                              ("tangent", ops.EPI_TANGENT, sg)):  # (BWD_SOFTPLUS runs on the 128x128 tile)
            bench(res, "cn_linear x6 imgA " + name, lambda: linear_x6_aimg(As, M, Bs, N, K, o0, epi, **kw))
        # the image's products equal the split-while-staging ones bitwise
        o1 = torch.empty_like(o0)
        ops.linear(A, Bs, N, K, o1, ops.EPI_STORE, bias=bias)
        linear_x6_aimg(As, M, Bs, N, K, o0, ops.EPI_STORE, bias=bias)
        torch.cuda.synchronize()
        print("x6 imgA STORE bitwise equal to the fp32-A split:", bool(torch.equal(o0, o1)))
    bench(res, "torch.matmul bf16 (hipBLASLt)", lambda: torch.matmul(A.bfloat16(), Bb.t()))
    dW = torch.empty(N, K, device=dev)
    db = torch.empty(N, device=dev)
    bench(res, "cn_wgrad 1 pair", lambda: ops.wgrad(A, A, N, K, dW, db=db))
    bench(res, "cn_wgrad 2 pairs", lambda: ops.wgrad(A, A, N, K, dW, db=db, Y1=aux1, X1=aux0), 2)
    bench(res, "cn_wgrad x6 1 pair", lambda: ops.wgrad(A, A, N, K, dW, db=db, mode="bf16x6"))
    bench(res, "cn_wgrad x6 2 pairs", lambda: ops.wgrad(A, A, N, K, dW, db=db, Y1=aux1, X1=aux0, mode="bf16x6"), 2)
    bench(res, "cn_wgrad bf16 2 pairs", lambda: ops.wgrad(A, A, N, K, dW, db=db, Y1=aux1, X1=aux0, mode="bf16"), 2)
    bench(res, "torch A^T A", lambda: torch.matmul(A.t(), A, out=dW))
    naux = {"store": 0, "softplus": 0, "relu": 0, "mul": 1, "tangent": 1, "bwd_softplus": 3, "bwd_relu": 1}
    for k, ms in res.items():
        extra = ""
        if k.startswith("cn_linear img "):  # A + aux streams + the output, 2 bytes each
            nb = 2.0 * M * N * (2 + naux[k.split()[-1]])
            extra = f"  {nb / ms / 1e6:7.0f} GB/s"  # (ms in milliseconds)
        print(f"{k:32s} {ms*1e3:9.1f} us  {fl / ms / 1e9:8.1f} TFLOP/s{extra}")


if __name__ == "__main__":
    main()
