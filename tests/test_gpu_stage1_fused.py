"""cn_stage1_fwd / cn_stage1_bwd (copenerf.motion._Stage1Terms) against the same terms as
torch fp32 expressions of the reference's lines (train.py:467-477 scene-flow residual
sums, the per-ray weighted point sums of train.py:484-495, the world points of
train.py:502-504), values and every input gradient, on inputs laid out as the renderer
hands them over (column slices of [M, 4] buffers).  The trainer-level parity of the
fused path against the oracle is tests/test_gpu_stage1.py."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _inputs(R, S, seed):
    g = torch.Generator(device="cpu").manual_seed(seed)
    M = R * S
    P = torch.randn(M, 4, generator=g).to(DEV)           # pts_time: xyz + t
    G = torch.randn(M, 4, generator=g).to(DEV)           # ∇sdf: normals xyz + ∂/∂t
    w = torch.rand(R, S, generator=g).to(DEV)
    mv = (0.3 * torch.randn(6, generator=g)).to(DEV)
    cw2 = torch.eye(4) + 0.2 * torch.randn(4, 4, generator=g)
    cw2[3] = torch.tensor([0.0, 0.0, 0.0, 1.0])
    return [t.requires_grad_(True) for t in (P, G, w, mv, cw2.to(DEV))]


def _torch_terms(pts, normals, flows, w, mv, cw2, t_world):
    p, n, f = pts.reshape(-1, 3), normals.reshape(-1, 3), flows.reshape(-1)
    om = mv[:3].reshape(1, 3).expand_as(p)
    lhs = torch.sum((torch.cross(om, p, dim=-1) + mv[3:].reshape(1, 3)) * n, dim=-1)
    wd = w.reshape(-1).detach()
    num = torch.sum(torch.abs(lhs + f) * wd)
    R = w.shape[0]
    pbar = torch.sum(w.reshape(R, -1, 1) * pts.reshape(R, -1, 3), dim=1)
    wbar = torch.sum(w, dim=1, keepdim=True)
    x = (cw2[:3, :3] @ p.T + cw2[:3, [-1]]).T
    return num, torch.sum(wd), torch.cat([pbar, wbar], 1), torch.cat([x, torch.full_like(x[:, :1], t_world)], 1)


@pytest.mark.parametrize("R,S,x_grad", [(64, 128, True), (37, 96, False), (5, 200, True), (1, 1, True)])
def test_stage1_terms_match_torch(R, S, x_grad):
    from copenerf.motion import _Stage1Terms
    P, G, w, mv, cw2 = _inputs(R, S, 40 + R)
    gy = torch.Generator(device="cpu").manual_seed(7)
    c_num = 0.7
    c_ray = torch.randn(R, 4, generator=gy).to(DEV)
    c_x = torch.randn(R * S, 4, generator=gy).to(DEV)
    views = lambda P, G: (P[:, :3].reshape(R, S, 3), G[:, :3].reshape(R, S, 3), G[:, 3:].reshape(R, S, 1))

    def run(fn):
        for t in (P, G, w, mv, cw2):
            t.grad = None
        num, sumw, ray, x = fn(*views(P, G), w, mv, cw2 if x_grad else cw2.detach(), 0.25)
        loss = c_num * num.sum() + (ray * c_ray).sum() + ((x * c_x).sum() if x_grad else 0.0)
        loss.backward()
        return [num.detach().reshape(()), sumw.detach().reshape(()), ray.detach(), x.detach()], \
               [t.grad.clone() if t.grad is not None else torch.zeros_like(t) for t in (P, G, w, mv, cw2)]

    ours_v, ours_g = run(lambda *a: _Stage1Terms.apply(*a, x_grad))
    ref_v, ref_g = run(_torch_terms)
    for name, a, b in zip(("num", "sumw", "ray_acc", "x"), ours_v, ref_v):
        torch.testing.assert_close(a, b, rtol=2e-5, atol=2e-5 * max(1.0, b.abs().max().item()), msg=name)
    for name, a, b in zip(("pts", "G", "weights", "mv", "cw2"), ours_g, ref_g):
        scale = max(1e-6, b.abs().max().item())
        assert (a - b).abs().max().item() <= 1e-5 * scale + 1e-6 * (R * S) ** 0.5 * scale, name
    assert ours_g[0][:, 3].abs().max().item() == 0.0  # the time column of the points gets nothing


def test_stage1_terms_bitwise_reproducible_and_empty():
    from copenerf.motion import _Stage1Terms
    R, S = 300, 128
    P, G, w, mv, cw2 = _inputs(R, S, 3)
    outs = []
    for _ in range(2):
        for t in (P, G, w, mv, cw2):
            t.grad = None
        num, sumw, ray, x = _Stage1Terms.apply(P[:, :3].reshape(R, S, 3), G[:, :3].reshape(R, S, 3),
                                               G[:, 3:].reshape(R, S, 1), w, mv, cw2, 0.0, True)
        (num.sum() + ray.sum() + x.sum()).backward()
        outs.append([num.detach().clone(), sumw.clone(), mv.grad.clone(), cw2.grad.clone(), G.grad.clone()])
    for a, b in zip(*outs):
        assert torch.equal(a, b)
    # no rays: zero sums, no launch on empty buffers
    P0 = torch.zeros(0, 4, device=DEV)
    w0 = torch.zeros(0, 8, device=DEV)
    num, sumw, ray, x = _Stage1Terms.apply(P0[:, :3].reshape(0, 8, 3), P0[:, :3].reshape(0, 8, 3),
                                           P0[:, 3:].reshape(0, 8, 1), w0, torch.zeros(6, device=DEV),
                                           torch.eye(4, device=DEV), 0.0, False)
    assert num.item() == 0.0 and sumw.item() == 0.0 and ray.shape == (0, 4)


def test_trainer_stage1_fused_matches_torch_expressions():
    """The trainer's stage-1 terms through the fused pass and through the torch
    expressions (stage1_fused=False) on the same step: losses and gradients."""
    from copenerf.train_step import SyntheticTrainer
    res = []
    for fused in (True, False):
        tr = SyntheticTrainer(DEV, rays=256, seed=5, stage1=True, joint_pose=True, n_images=8, start_it=3000,
                              mfma_dtype="fp32", train_cfg={"sdf_consistency_enable_pose_grad": True},
                              stage1_fused=fused)
        tr.begin_iteration()
        batch = tr.make_batch()
        torch.manual_seed(0)
        out = tr.renderer(batch["rays_o"], batch["rays_d"], batch["norm"], tr.query_time(),
                          torch.full((256, 1), 0.01, device=DEV), torch.full((256, 1), 3.0, device=DEV),
                          cos_anneal_ratio=tr.sched.car, it=3000, eval=False, t_rand=batch.get("t_rand"))
        terms = tr.stage1_terms(out, batch)
        total = sum(terms)
        params = [p for p in tr.params + list(tr.motion.parameters()) + list(tr.poses.parameters()) if p.requires_grad]
        grads = torch.autograd.grad(total, params, allow_unused=True)
        res.append(([t.detach() for t in terms], [g if g is not None else torch.zeros_like(p)
                                                  for g, p in zip(grads, params)]))
    (tf, gf), (tt, gt) = res
    for a, b in zip(tf, tt):
        torch.testing.assert_close(a, b, rtol=1e-5, atol=1e-6)
    for a, b in zip(gf, gt):
        scale = max(1e-8, b.abs().max().item())
        assert (a - b).abs().max().item() <= 1e-4 * scale


@pytest.mark.parametrize("n", [1, 3, 10, 21])
def test_mat4_chain_matches_torch_products(n):
    """cn_mat4_chain_fwd / _bwd: the running products of the stage-1 pose chains and their
    gradient (every product may carry one) against torch matmuls in fp32."""
    from copenerf.motion import _Mat4Chain
    g = torch.Generator(device="cpu").manual_seed(n)
    A = (torch.eye(4) + 0.2 * torch.randn(n, 4, 4, generator=g)).to(DEV).requires_grad_(True)
    dC = torch.randn(n, 4, 4, generator=g).to(DEV)
    C = _Mat4Chain.apply(A)
    (gk,) = torch.autograd.grad(C, A, dC)
    out, cur = [], None
    for a in A.unbind(0):
        cur = a if cur is None else a @ cur
        out.append(cur)
    Ct = torch.stack(out)
    (gt,) = torch.autograd.grad(Ct, A, dC)
    torch.testing.assert_close(C, Ct, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(gk, gt, rtol=1e-4, atol=1e-4 * gt.abs().max().item())
