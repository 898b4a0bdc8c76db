"""Joint pose training and the stage-1 motion losses through the HIP path,
against the CPU oracle with identical sample positions: learnable SE(3) poses
(PoseRetriever) -> rays -> render -> L1/eikonal/smoothness + scene-flow SDF
loss + SDF consistency at motion-mapped world points (train.py:425-505) ->
gradients of the poses, the motion network and the fields."""
import pytest
import torch

from helpers import REN_CFG, build_modules, named_params, oracle_params
from oracle import neus_oracle as O

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _setup(device):
    from copenerf.motion import MotionNetwork
    from copenerf.rays import PoseRetriever
    from copenerf.train_step import MOTION_CFG
    torch.manual_seed(5)
    motion = MotionNetwork(**MOTION_CFG)
    poses = PoseRetriever(4)
    with torch.no_grad():
        poses.r.copy_(torch.tensor([[0.01, -0.02, 0.015]] * 4))
        poses.t.copy_(torch.tensor([[0.02, 0.01, -0.03]] * 4))
    return motion.to(device), poses.to(device)


def _rays(poses, R, device):
    from copenerf.rays import intrinsics_ndc, world_rays
    g = torch.Generator().manual_seed(9)
    pixn = ((torch.rand(R, 2, generator=g) - 0.5) * 0.5).to(device)
    K = intrinsics_ndc(0.9 * 64, 0.9 * 64, 64, 64, device=device)
    o, d, n = world_rays(pixn, K, poses(2), torch.eye(4, device=device))
    o = o + torch.tensor([0.05, -0.03, 1.6], device=device)
    return o, d, n


def _stage1(motion, sdf_fn, out, t_img):
    from copenerf.motion import scene_flow_loss, world_points
    omega, vel = motion(torch.tensor([[t_img]], device=out["sdf"].device))
    l_sf = scene_flow_loss(out["sampled_points"], out["normals"], out["sdf_flows"], out["weights"], omega, vel)
    _, rel = motion.compute_relative_camera_pose(0, 2, 4, 10)
    c2c = motion.compute_w2c_mappings(rel)[-1]
    pw = world_points(out["sampled_points"], torch.inverse(c2c))
    sdf_w = sdf_fn(torch.cat([pw, torch.full((pw.shape[0], 1), -1.0, device=pw.device)], 1))
    return 0.1 * l_sf + torch.mean(torch.abs(sdf_w - out["sdf"].reshape(-1, 1)))


def test_joint_pose_stage1_gradients_match_oracle():
    R, t_img = 128, 2 / 3 * 2 - 1
    # oracle (CPU)
    mods_cpu = build_modules(55, 256, 256)
    P, Pc, var, leaves = oracle_params(*mods_cpu)
    motion_c, poses_c = _setup("cpu")
    o, d, n = _rays(poses_c, R, "cpu")
    t = torch.tensor([t_img])
    near, far = torch.full((R, 1), 0.01), torch.full((R, 1), 3.0)
    g = torch.Generator().manual_seed(4)
    t_rand, gt = torch.rand(R, 64, generator=g), torch.rand(R, 3, generator=g)
    torch.set_num_threads(8)
    z = O.hierarchical_z(P, o.detach(), d.detach(), t, near, far, 64, 64, 4, t_rand)
    ref = O.render_core(P, Pc, var, o, d, n, t, z, (far[0, 0] - near[0, 0]) / 64, 0.5)
    loss_ref = O.train_loss(ref, gt) + _stage1(motion_c, lambda x: O.sdf_mlp(P, x)[:, :1], ref, t_img)
    ref_leaves = [poses_c.r, poses_c.t] + list(motion_c.parameters()) + list(leaves.values())
    gref = torch.autograd.grad(loss_ref, ref_leaves, allow_unused=True)

    # HIP path
    from copenerf import NeuSRenderer
    mods = build_modules(55, 256, 256, device=DEV)
    sdf, col, dev = mods
    r = NeuSRenderer(None, sdf, dev, col, None, **REN_CFG).to(DEV)
    motion_h, poses_h = _setup(DEV)
    oh, dh, nh = _rays(poses_h, R, DEV)
    out = r(oh, dh, nh, t.to(DEV), near.to(DEV), far.to(DEV), cos_anneal_ratio=0.5, it=0, eval=False,
            z_vals=z.to(DEV))
    loss = O.train_loss(out, gt.to(DEV)) + _stage1(motion_h, sdf.sdf, out, t_img)
    assert abs(loss.item() - loss_ref.item()) <= 1e-4 * abs(loss_ref.item()) + 1e-6
    loss.backward()

    def close(got, ref, name, rtol=5e-3):
        assert got is not None, name
        got = got.detach().cpu()
        scale = ref.abs().max().item() + 1e-12
        err = (got - ref).abs().max().item()
        assert err <= rtol * scale, (name, err, scale)

    close(poses_h.r.grad[2], gref[0][2], "pose r")
    close(poses_h.t.grad[2], gref[1][2], "pose t")
    nm = len(list(motion_c.parameters()))
    for (name, p), gr in zip(motion_h.named_parameters(), gref[2:2 + nm]):
        close(p.grad, gr, "motion." + name)
    keys = list(leaves)
    for name, p in named_params(*mods):
        close(p.grad, gref[2 + nm + keys.index(name)], name, rtol=2e-2)


@pytest.mark.parametrize("joint_pose,stage1", [(True, False), (True, True)])
def test_synthetic_trainer_modes_step(joint_pose, stage1):
    """The C3-style training step (joint pose, optionally stage 1) runs and updates
    the poses / motion network with finite values."""
    from copenerf.train_step import SyntheticTrainer
    tr = SyntheticTrainer(DEV, rays=1024, joint_pose=joint_pose, stage1=stage1)
    r0 = tr.poses.r.detach().clone()
    for _ in range(2):
        loss = tr.step()
    assert torch.isfinite(loss).item()
    assert not torch.equal(tr.poses.r.detach(), r0)
    for p in tr.all_params:
        assert torch.isfinite(p).all()
