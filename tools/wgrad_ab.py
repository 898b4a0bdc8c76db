"""Weight-gradient variant check + timing (COPENERF_WGRAD_KERNEL picks the 256x256 bf16x6
kernel, read once per process): dW/db against float64 at a small M (2 pairs, ragged M),
then the C2-shape timing of a 1-pair and a 2-pair call.  One JSON line."""
import json
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


def main():
    torch.manual_seed(0)
    dev = "cuda"
    res = {"variant": os.environ.get("COPENERF_WGRAD_KERNEL", "0"), "lib": os.environ.get("COPENERF_LIB", "")}
    M = 65536 + 1000
    N = K = 256
    Y0, X0, Y1, X1 = (torch.randn(M, 256, device=dev) * s for s in (0.1, 1.0, 0.05, 0.3))
    dW = torch.zeros(N, K, device=dev)
    db = torch.zeros(N, device=dev)
    ops.wgrad(Y0, X0, N, K, dW, db=db, Y1=Y1, X1=X1, mode="bf16x6")
    ref = Y0.double().t() @ X0.double() + Y1.double().t() @ X1.double()
    refb = Y0.double().sum(0)
    scale = ref.abs().max().item()
    res["dW_err_rel"] = (dW.double() - ref).abs().max().item() / scale
    res["db_err"] = (db.double() - refb).abs().max().item()
    # fp32-class bar: fp32 summation of M terms
    res["ok"] = bool(res["dW_err_rel"] < 2e-6 and res["db_err"] < 1e-3)
    M = 524288
    A, B, C, D = (torch.randn(M, 256, device=dev) * 0.1 for _ in range(4))
    fl = 2.0 * M * N * K
    t1 = timeit(lambda: ops.wgrad(A, B, N, K, dW, db=db, mode="bf16x6"))
    t2 = timeit(lambda: ops.wgrad(A, B, N, K, dW, db=db, Y1=C, X1=D, mode="bf16x6"))
    res.update({"pair1_us": round(t1 * 1e3, 1), "pair2_us": round(t2 * 1e3, 1),
                "pair2_tflops": round(2 * fl / t2 / 1e9, 1), "pair2_frac_416": round(2 * fl / t2 / 1e9 / 416.7, 3)})
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
