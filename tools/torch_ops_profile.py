"""Which torch ops (outside the HIP library) run per C2 train step, by CUDA time."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "cope-nerf_amd"), ROOT]
from copenerf.train_step import SyntheticTrainer  # noqa: E402


def main():
    # CONFIG: a bench.py config (default c2)
    from bench import CONFIGS
    rays, kw, _ = CONFIGS[os.environ.get("CONFIG", "c2")]
    kw = {k: v for k, v in kw.items() if k != "graph"}
    tr = SyntheticTrainer("cuda:0", rays=rays, **kw)
    for _ in range(3):
        tr.step()
    torch.cuda.synchronize()
    from torch.profiler import ProfilerActivity, profile
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA],
                 with_stack=bool(os.environ.get("STACKS"))) as prof:
        for _ in range(3):
            tr.step()
        torch.cuda.synchronize()
    print(prof.key_averages().table(sort_by="cuda_time_total", row_limit=45, max_name_column_width=60))
    if os.environ.get("STACKS"):
        print(prof.key_averages(group_by_stack_n=6).table(sort_by="cuda_time_total", row_limit=40,
                                                          max_name_column_width=40, max_src_column_width=120))


if __name__ == "__main__":
    main()
