"""__graft_entry__.smoke(): one small train step on cuda:0 checked against the oracle."""
import torch


def run_smoke():
    from helpers import REN_CFG, build_modules, named_params, oracle_params
    from oracle import neus_oracle as O
    from copenerf import NeuSRenderer, _lib
    _lib.load()
    assert torch.cuda.is_available(), "smoke() needs a HIP device"
    R = 32
    g = torch.Generator().manual_seed(0)
    o = torch.tensor([0.05, -0.03, 1.6]).expand(R, 3).contiguous()
    d = torch.cat([(torch.rand(R, 2, generator=g) - 0.5) * 0.5, -torch.ones(R, 1)], -1)
    nrm = d.norm(dim=-1, keepdim=True)
    d = d / nrm
    t, near, far = torch.tensor([0.25]), torch.full((R, 1), 0.01), torch.full((R, 1), 3.0)
    t_rand, gt = torch.rand(R, 64, generator=g), torch.rand(R, 3, generator=g)
    P, Pc, var, leaves = oracle_params(*build_modules(5, 64, 64))
    ref = O.render(P, Pc, var, o, d, nrm, t, near, far, car=0.5, t_rand=t_rand)
    ref_loss = O.train_loss(ref, gt)
    mods = build_modules(5, 64, 64, device="cuda")
    r = NeuSRenderer(None, mods[0], mods[2], mods[1], None, **REN_CFG).cuda()
    c = lambda x: x.cuda()  # noqa: E731
    out = r(c(o), c(d), c(nrm), c(t), c(near), c(far), cos_anneal_ratio=0.5, it=0, eval=False, t_rand=c(t_rand))
    loss = O.train_loss(out, c(gt))
    loss.backward()
    err = max((out[k].detach().cpu() - ref[k].detach()).abs().max().item() for k in ("color_fine", "depth_pred"))
    assert err <= 1e-4, f"smoke: rgb/depth differ from the oracle by {err}"
    assert abs(loss.item() - ref_loss.item()) <= 1e-4 * abs(ref_loss.item()) + 1e-5
    assert all(p.grad is not None and torch.isfinite(p.grad).all() for _, p in named_params(*mods))
    print(f"smoke ok: max |Δ rgb/depth| = {err:.2e}, loss {loss.item():.6f} vs oracle {ref_loss.item():.6f}")
