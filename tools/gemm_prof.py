"""Launch each cn_linear epilogue a few times at the C2 layer shape (for
rocprofv3 --pmc / --kernel-trace runs; the per-kernel names carry the EPI)."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "cope-nerf_amd"), ROOT]
from copenerf import ops  # noqa: E402


def main():
    M = int(os.environ.get("M", 524288))
    N = K = 256
    dev = "cuda"
    A = torch.randn(M, K, device=dev) * 0.1
    B = torch.randn(N, K, device=dev) * 0.05
    bias = torch.randn(N, device=dev) * 0.1
    aux0 = torch.rand(M, N, device=dev)
    aux1 = torch.randn(M, N, device=dev)
    o0 = torch.empty(M, N, device=dev)
    o1 = torch.empty(M, N, device=dev)
    mode = os.environ.get("GEMM_MODE", "fp32")  # fp32 | bf16 | x6
    if mode == "bf16":
        B = B.bfloat16().contiguous()
    elif mode == "x6":
        B = ops.split_bf16x3(B)
    for epi, kw in ((ops.EPI_STORE, dict(bias=bias)), (ops.EPI_SOFTPLUS, dict(bias=bias)),
                    (ops.EPI_TANGENT, dict(aux0=aux0, aux_beta=100.0)), (7, {})):
        for _ in range(int(os.environ.get("REPS", 5))):
            ops.linear(A, B, N, K, o0, epi, **kw)
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
