"""Which torch ops (outside the HIP library) run per C2 train step, by CUDA time."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "cope-nerf_amd"), ROOT]
from copenerf.train_step import SyntheticTrainer  # noqa: E402


def main():
    kw = dict(mfma_dtype=os.environ.get("MODE", "bf16x6"))
    if os.environ.get("C3"):  # the c3fp32 bench config: joint pose + stage 1
        kw.update(joint_pose=True, stage1=True, start_it=30000)
    tr = SyntheticTrainer("cuda:0", rays=4096, **kw)
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
