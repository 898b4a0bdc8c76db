"""Where the small torch launches of a train step (CONFIG: a bench.py config) come from: every aten op on a
device tensor during one step, counted by the innermost repo (or torch.optim /
autograd) source line that issued it."""
import collections
import os
import sys
import traceback

import torch
from torch.utils._python_dispatch import TorchDispatchMode

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "cope-nerf_amd"), ROOT]
from copenerf.train_step import SyntheticTrainer  # noqa: E402

SKIP_OPS = {"aten.empty.memory_format", "aten.empty_strided.default", "aten.view.default", "aten.detach.default",
            "aten.t.default", "aten.slice.Tensor", "aten.select.int", "aten._unsafe_view.default",
            "aten.as_strided.default", "aten.expand.default", "aten.unsqueeze.default", "aten.squeeze.dim",
            "aten.permute.default", "aten.alias.default", "aten.transpose.int", "aten.split.Tensor",
            "aten.unbind.int", "aten.reshape.default", "aten.lift_fresh.default"}


class Origins(TorchDispatchMode):
    def __init__(self):
        super().__init__()
        self.count = collections.Counter()

    def __torch_dispatch__(self, func, types, args=(), kwargs=None):
        name = str(func)
        if name not in SKIP_OPS:
            site = "?"
            for fr in reversed(traceback.extract_stack()[:-1]):
                f = fr.filename
                if (ROOT in f and "op_origins" not in f) or "torch/optim" in f or "torch/nn/utils" in f:
                    site = f"{os.path.relpath(f, ROOT) if ROOT in f else f.split('site-packages/')[-1]}:{fr.lineno}"
                    break
            self.count[(name, site)] += 1
        return func(*args, **(kwargs or {}))


def main():
    # CONFIG: a bench.py config (default c2)
    from bench import CONFIGS
    rays, kw, _ = CONFIGS[os.environ.get("CONFIG", "c2")]
    kw = {k: v for k, v in kw.items() if k != "graph"}
    tr = SyntheticTrainer("cuda:0", rays=rays, **kw)
    for _ in range(2):
        tr.step()
    torch.cuda.synchronize()
    m = Origins()
    with m:
        tr.step()
    torch.cuda.synchronize()
    by_site = collections.Counter()
    for (op, site), n in m.count.items():
        by_site[site] += n
    print("total aten ops", sum(m.count.values()))
    for site, n in by_site.most_common(60):
        ops = collections.Counter({op: c for (op, s), c in m.count.items() if s == site})
        top = ", ".join(f"{o.split('.')[1]}x{c}" for o, c in ops.most_common(4))
        print(f"{n:5d} {site:60s} {top}")


if __name__ == "__main__":
    main()
