"""Which autograd graph outlives a training step?  (The "AccumulateGrad node's stream does
not match" warning at graph capture means some tensor of an earlier step's graph is still
referenced.)  Runs eager steps of SyntheticTrainer, drops the loss, then lists every live
tensor that carries a grad_fn, with the attribute path that keeps it (GPU box):
    python tools/graph_alive.py [--stage1] [--joint-pose]"""
import gc
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "cope-nerf_amd"), ROOT]


def owners(obj, depth=3):
    out = []
    for r in gc.get_referrers(obj):
        if r is sys._getframe() or isinstance(r, type(sys._getframe())):
            continue
        desc = type(r).__name__
        if isinstance(r, dict):
            keys = [k for k, v in r.items() if v is obj]
            desc += f"[{keys[:3]}]"
            if depth > 0:
                for rr in gc.get_referrers(r):
                    if hasattr(rr, "__dict__") and rr.__dict__ is r:
                        desc += f" of {type(rr).__name__}"
        out.append(desc)
    return out[:6]


def main():
    from copenerf.train_step import SyntheticTrainer
    tr = SyntheticTrainer("cuda:0", rays=1024, stage1="--stage1" in sys.argv, joint_pose="--joint-pose" in sys.argv,
                          capturable=True, mfma_dtype="bf16x6")
    for _ in range(2):
        tr.step()
    torch.cuda.synchronize()
    gc.collect()
    live = [o for o in gc.get_objects() if torch.is_tensor(o) and o.grad_fn is not None]
    print(f"{len(live)} live tensors with a grad_fn after the steps")
    for t in live[:20]:
        print(tuple(t.shape), type(t.grad_fn).__name__, owners(t))


if __name__ == "__main__":
    main()
