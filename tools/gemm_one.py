"""Run one cn_linear variant N times (for rocprofv3 counter passes)."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "cope-nerf_amd"), ROOT]
from copenerf import ops  # noqa: E402

M, N, K = 524288, 256, 256
A = torch.randn(M, K, device="cuda") * 0.1
B = torch.randn(N, K, device="cuda") * 0.05
o0 = torch.empty(M, N, device="cuda")
epi = os.environ.get("EPI", "store")
for _ in range(int(os.environ.get("ITERS", 5))):
    if epi == "store":
        ops.linear(A, B, N, K, o0, ops.EPI_STORE)
    else:
        torch.matmul(A, B.t(), out=o0)
torch.cuda.synchronize()
