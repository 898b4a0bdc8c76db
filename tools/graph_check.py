"""Capture the C2 train step in a HIP graph, replay, compare speed with eager."""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "cope-nerf_amd"), ROOT]
from copenerf.train_step import GraphedTrainer, SyntheticTrainer  # noqa: E402


def timed(fn, n):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        loss = fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / n * 1e3, loss


def main():
    R = int(os.environ.get("RAYS", 4096))
    tr = SyntheticTrainer("cuda:0", rays=R, capturable=True)
    for _ in range(3):
        tr.step()
    ms_e, loss_e = timed(tr.step, 10)
    print(f"eager   {ms_e:.3f} ms/step  loss {loss_e.item():.5f}", flush=True)
    del loss_e  # a live loss keeps its autograd graph (and the leaves' AccumulateGrad nodes) alive
    g = GraphedTrainer(tr)
    ms_g, loss_g = timed(g.step, 10)
    print(f"graphed {ms_g:.3f} ms/step  loss {loss_g.item():.5f}", flush=True)
    l = [g.step().item() for _ in range(3)]
    print("replay losses", l)


if __name__ == "__main__":
    main()
