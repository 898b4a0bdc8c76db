"""Timing of the 256x256x256 products of the feature-head fold (renderer.py) under a
few torch formulations (GPU box)."""
import torch

a = torch.randn(256, 256, device="cuda")
b = torch.randn(256, 256, device="cuda")


def t(fn, n=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n * 1e3


ref = (a.double() @ b.double())
for name, fn in [("mm", lambda: a @ b), ("mm a.t()", lambda: a.t() @ b), ("mm b.t()", lambda: a @ b.t()),
                 ("bmm 4x64", lambda: (a.view(4, 64, 256) @ b).view(256, 256)),
                 ("bmm 16x16", lambda: (a.view(16, 16, 256) @ b).view(256, 256)),
                 ("f64", lambda: (a.double() @ b.double()).float()),
                 ("einsum", lambda: torch.einsum("ik,kj->ij", a, b))]:
    us = t(fn)
    err = (fn().double() - ref).abs().max().item()
    print(f"{name:12s} {us:8.1f} us  err {err:.2e}")
