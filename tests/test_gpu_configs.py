"""The BASELINE.json configs as they are run (bench.py): C2 at full size in the
timed GEMM mode (bf16x6) against the oracle, C4's 8192-ray batch, and C5's
HIP-graph-captured step replayed against eager steps under the reference's
schedule."""
import pytest
import torch

from helpers import REN_CFG, build_modules, named_params, oracle_params
from oracle import neus_oracle as O

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _rays(R, seed, device="cpu"):
    g = torch.Generator().manual_seed(seed)
    o = torch.tensor([0.05, -0.03, 1.6]).expand(R, 3).contiguous()
    d = torch.cat([(torch.rand(R, 2, generator=g) - 0.5) * 0.6, -torch.ones(R, 1)], -1)
    nrm = d.norm(dim=-1, keepdim=True)
    return o.to(device), (d / nrm).to(device), nrm.to(device)


def test_c2_full_size_bf16x6_against_oracle():
    """4096 rays x 128 samples (M = 524,288 sample rows in every GEMM) in the bench's
    GEMM mode.  Rays 0..511 carry the oracle's sample positions, repeated 8 times to
    fill the batch: rgb / depth of every copy within 1e-4 of the oracle, parameter
    gradients within 2e-3 of the oracle's (the loss is a per-ray mean, so the 8-fold
    batch has the 512-ray gradient), plus the invariants of the sampler path."""
    from copenerf import NeuSRenderer
    R0, R = 512, 4096
    seed = 57
    o, d, nrm = _rays(R0, 3)
    t = torch.tensor([0.25])
    near, far = torch.full((R0, 1), 0.01), torch.full((R0, 1), 3.0)
    g = torch.Generator().manual_seed(4)
    t_rand, gt = torch.rand(R0, 64, generator=g), torch.rand(R0, 3, generator=g)
    P, Pc, var, leaves = oracle_params(*build_modules(seed))
    torch.set_num_threads(16)
    z = O.hierarchical_z(P, o, d, t, near, far, 64, 64, 4, t_rand)
    ref = O.render_core(P, Pc, var, o, d, nrm, t, z, (far[0, 0] - near[0, 0]) / 64, 0.5)
    loss_ref = O.train_loss(ref, gt)
    gref = torch.autograd.grad(loss_ref, list(leaves.values()))
    mods = build_modules(seed, device=DEV)
    r = NeuSRenderer(None, mods[0], mods[2], mods[1], None, **REN_CFG).to(DEV).set_mfma_dtype("bf16x6")
    rep = lambda x: x.repeat(R // R0, *([1] * (x.dim() - 1))).to(DEV)  # noqa: E731
    out = r(rep(o), rep(d), rep(nrm), t.to(DEV), rep(near), rep(far), cos_anneal_ratio=0.5, it=0, eval=False,
            z_vals=rep(z))
    for k in ("color_fine", "depth_pred"):
        err = (out[k].detach().cpu() - ref[k].detach().repeat(R // R0, 1)).abs().max().item()
        assert err <= 1e-4, (k, err)
    loss = O.train_loss(out, rep(gt))
    assert abs(loss.item() - loss_ref.item()) <= 1e-4 * abs(loss_ref.item())
    loss.backward()
    keys = list(leaves)
    for name, p in named_params(*mods):
        ref_g = gref[keys.index(name)]
        err = (p.grad.detach().cpu() - ref_g).abs().max().item()
        assert err <= 2e-3 * (ref_g.abs().max().item() + 1e-12), (name, err)
    # the sampler path at full size: deterministic, sorted samples, weights in [0, 1]
    oo, dd, nn = _rays(R, 5, DEV)
    args = (oo, dd, nn, torch.tensor([0.0], device=DEV), torch.full((R, 1), 0.01, device=DEV),
            torch.full((R, 1), 3.0, device=DEV))
    tr = torch.rand(R, 64, device=DEV, generator=torch.Generator(device=DEV).manual_seed(6))
    with torch.no_grad():
        a = r(*args, cos_anneal_ratio=0.5, it=0, eval=False, t_rand=tr)
        b = r(*args, cos_anneal_ratio=0.5, it=0, eval=False, t_rand=tr)
    for k in ("color_fine", "depth_pred", "weights", "normals"):
        assert torch.isfinite(a[k]).all() and torch.equal(a[k], b[k]), k
    w = a["weights"]
    assert w.shape == (R, 128) and (w >= 0).all() and (w.sum(-1) <= 1 + 1e-5).all()
    zz = ((a["sampled_points"] - oo[:, None, :]) * dd[:, None, :]).sum(-1)
    assert (zz[:, 1:] >= zz[:, :-1] - 1e-5).all()


def test_c4_8192_rays_step_and_ray_independence():
    """C4's per-GPU workload (bench.py --config c4: Co3D/skateboard's stage 1 at 8192 rays x 128
    samples): the training step runs with finite parameters, and a ray's render does not depend on
    the batch it is in (8192 = two 4096 halves, bitwise)."""
    from copenerf.train_step import SyntheticTrainer
    skateboard = dict(sdf_consistency_enable_pose_grad=True, rgb_weight=0.33333, end_sdf_weight_increase_iteration=-1)
    tr = SyntheticTrainer(DEV, rays=8192, mfma_dtype="bf16x6", stage1=True, start_it=30000, train_cfg=skateboard)
    for _ in range(2):
        loss = tr.step()
    assert torch.isfinite(loss).item()
    tr.check_finite()
    r = tr.renderer
    o, d, n = _rays(8192, 8, DEV)
    near, far = torch.full((8192, 1), 0.01, device=DEV), torch.full((8192, 1), 3.0, device=DEV)
    trand = torch.rand(8192, 64, device=DEV, generator=torch.Generator(device=DEV).manual_seed(9))
    t = torch.tensor([0.0], device=DEV)
    with torch.no_grad():
        full = r(o, d, n, t, near, far, cos_anneal_ratio=0.5, it=0, t_rand=trand)
        halves = [r(o[s], d[s], n[s], t, near[s], far[s], cos_anneal_ratio=0.5, it=0, t_rand=trand[s])
                  for s in (slice(0, 4096), slice(4096, 8192))]
    for k in ("color_fine", "depth_pred", "weights"):
        assert torch.equal(full[k], torch.cat([h[k] for h in halves])), k


C5_REN = dict(REN_CFG, n_importance=128)  # coarse 64 + 4 rounds of 32 = 192 samples


@pytest.mark.parametrize("start_it", [0, 1000, 5000])
@pytest.mark.filterwarnings("error:The AccumulateGrad node's stream")  # no earlier step's graph alive at capture
def test_c5_graph_replays_equal_eager_steps(start_it):
    """The HIP-graph-captured step (GraphedTrainer) at C5's sample counts under the
    reference's schedule (cos_anneal_ratio ramp, learning-rate warm-up, annealed loss
    weights, the frame cycling) from iteration start_it: three replays equal three
    eager steps of an identical trainer bitwise -- loss, parameters, Adam state."""
    from copenerf.train_step import GraphedTrainer, SyntheticTrainer
    kw = dict(rays=512, H=96, W=128, ren_cfg=C5_REN, capturable=True, schedule="reference", start_it=start_it,
              mfma_dtype="bf16x6", n_images=4)
    a = SyntheticTrainer(DEV, **kw)
    b = SyntheticTrainer(DEV, **kw)
    g = GraphedTrainer(b, warmup=2)  # 2 eager warm-up steps + the captured step, run once
    for _ in range(3):
        a.step()
    assert a.it == b.it == start_it + 3
    for _ in range(3):
        la = a.step().detach().clone()
        lb = g.step().detach().clone()
        torch.cuda.synchronize()
        assert torch.equal(la, lb), (la.item(), lb.item())
    assert b.sched.car.item() == a.sched.car.item()
    assert abs(a.sched.car.item() - min(1.0, (start_it + 6) / 50000)) <= 1e-7
    for (n, pa), pb in zip(a.sdf.named_parameters(), b.sdf.parameters()):
        assert torch.equal(pa, pb), n
    for pa, pb in zip(a.all_params, b.all_params):
        assert torch.equal(pa, pb)
        sa, sb = a.opt.state[pa], b.opt.state[pb]
        for k in ("exp_avg", "exp_avg_sq", "step"):
            assert torch.equal(sa[k], sb[k]), k
    for ga, gb in zip(a.opt.param_groups, b.opt.param_groups):
        assert torch.equal(ga["lr"], gb["lr"])


@pytest.mark.filterwarnings("error:The AccumulateGrad node's stream")
def test_c5_graph_stage1_joint_pose_replays():
    """The captured step with joint pose and the stage-1 losses (device image index,
    masked reference frames) also replays equal to eager, across frames."""
    from copenerf.train_step import GraphedTrainer, SyntheticTrainer
    kw = dict(rays=256, H=48, W=64, capturable=True, schedule="reference", start_it=30000, mfma_dtype="bf16x6",
              n_images=6, joint_pose=True, stage1=True)
    a = SyntheticTrainer(DEV, **kw)
    b = SyntheticTrainer(DEV, **kw)
    g = GraphedTrainer(b, warmup=1)
    for _ in range(2):
        a.step()
    frames = set()
    for _ in range(6):  # every frame, incl. the world camera and the last one
        frames.add(a.image_index(a.it + 1))
        la = a.step().detach().clone()
        lb = g.step().detach().clone()
        torch.cuda.synchronize()
        assert torch.equal(la, lb), (la.item(), lb.item())
    assert frames == set(range(6))
    for pa, pb in zip(a.all_params, b.all_params):
        assert torch.equal(pa, pb)
