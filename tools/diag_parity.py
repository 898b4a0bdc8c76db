"""Where do HIP-vs-oracle render differences come from?  Per-ray depth error vs
the largest sample-position shift, and the coarse-SDF forward error."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "cope-nerf_amd"), ROOT, os.path.join(ROOT, "tests")]
from helpers import REN_CFG, build_modules, oracle_params  # noqa: E402
from oracle import neus_oracle as O  # noqa: E402
from copenerf import NeuSRenderer  # noqa: E402

R = int(os.environ.get("R", 1024))
g = torch.Generator().manual_seed(R)
mods_cpu = build_modules(55)
P, Pc, var, leaves = oracle_params(*mods_cpu)
o = torch.tensor([0.05, -0.03, 1.6]).expand(R, 3).contiguous()
d = torch.cat([(torch.rand(R, 2, generator=g) - 0.5) * 0.6, -torch.ones(R, 1)], -1)
nrm = d.norm(dim=-1, keepdim=True)
d = d / nrm
t = torch.tensor([0.25])
near, far = torch.full((R, 1), 0.01), torch.full((R, 1), 3.0)
t_rand = torch.rand(R, 64, generator=g)
torch.set_num_threads(16)
ref = O.render(P, Pc, var, o, d, nrm, t, near, far, car=0.5, t_rand=t_rand)
mods = build_modules(55, device="cuda")
r = NeuSRenderer(None, mods[0], mods[2], mods[1], None, **REN_CFG).cuda()
c = lambda x: x.cuda()  # noqa: E731
out = r(c(o), c(d), c(nrm), c(t), c(near), c(far), cos_anneal_ratio=0.5, it=0, eval=False, t_rand=c(t_rand))
de = (out["depth_pred"].detach().cpu() - ref["depth_pred"]).abs().squeeze(1)
ce = (out["color_fine"].detach().cpu() - ref["color_fine"]).abs().max(1)[0]
zz_h = ((out["sampled_points"].cpu() - o[:, None]) * d[:, None]).sum(-1)
zz_r = ((ref["sampled_points"] - o[:, None]) * d[:, None]).sum(-1)
dz = (zz_h - zz_r).abs().max(1)[0]
print(f"depth err: max {de.max():.3e} p99 {de.quantile(0.99):.3e} median {de.median():.3e}")
print(f"color err: max {ce.max():.3e} p99 {ce.quantile(0.99):.3e} median {ce.median():.3e}")
print(f"sample shift per ray: max {dz.max():.3e}; rays with shift > 1e-4: {(dz > 1e-4).sum().item()}")
top = de.argsort(descending=True)[:8]
for i in top.tolist():
    print(f"  ray {i}: depth err {de[i]:.3e} color err {ce[i]:.3e} max sample shift {dz[i]:.3e}")
# rays without any sample shift: pure arithmetic error
mask = dz < 1e-5
print(f"rays w/o shift ({mask.sum().item()}): depth max {de[mask].max():.3e}, color max {ce[mask].max():.3e}")
# the SDF MLP alone at the same points
x = ref["sampled_points"].reshape(-1, 3)
x = torch.cat([x, t.expand(x.shape[0], 1)], 1)
so = O.sdf_mlp(P, x)[:, :1].detach()
sh, _, _ = mods[0].field(x.cuda(), want_feat=False, want_grad=False)
e = (sh.cpu() - so).abs()
print(f"sdf fwd abs err: max {e.max():.3e} mean {e.mean():.3e}; |sdf| mean {so.abs().mean():.3e}")
