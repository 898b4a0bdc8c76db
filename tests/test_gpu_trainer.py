"""train.py's per-iteration call sequence (train.py:433-438, 441-444, 526-532)
through `from model import Trainer` with the HIP NeuSRenderer: process_data ->
near_far_from_sphere -> get_cos_anneal_ratio -> renderer -> the reference's
loss expressions -> compute_loss -> backpropagation; the first iteration's
loss against the CPU oracle on the same rays and sample positions."""
import os
import sys

import pytest
import torch

from helpers import REN_CFG, build_modules, oracle_params
from oracle import neus_oracle as O

pytestmark = pytest.mark.gpu
DEV = "cuda"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_train_py_sequence_on_hip():
    sys.path.insert(0, os.path.join(ROOT, "cope-nerf_amd"))
    from model import NeuSRenderer, Trainer
    sdf, col, var = build_modules(13, device=DEV)
    renderer = NeuSRenderer(None, sdf, var, col, None, **REN_CFG).set_mfma_dtype("bf16x6")
    P, Pc, varc, leaves = oracle_params(*build_modules(13))
    opt = torch.optim.Adam(list(renderer.parameters()), lr=1e-3)
    cfg = dict(n_training_points=1024, rgb_weight=[1.0, 1.0], eikonal_weight=[0.1, 0.1], sdf_weight=[0.1, 0.1],
               flow_rgb_weight=[7.5, 7.5], sdf_consistency_weight=[0.0, 1.0],
               edge_aware_smoothness_weight=[1.0, 0.0], smoothness_weight=[1e-4, 0.0])
    tr = Trainer(renderer, opt, None, cfg, device=torch.device(DEV), total_nb_images=5,
                 cfg_all={"rendering": {"depth_range": [0.01, 3.0]}}, logger=None, gt_depths=None, world_cam_idx=2)
    g = torch.Generator().manual_seed(2)
    h, w = 60, 80
    f = 0.9 * w
    K = torch.tensor([[[2 * f / w, 0, 0, 0], [0, -2 * f / h, 0, 0], [0, 0, -1, 0], [0, 0, 0, 1]]])
    data = {"img": torch.rand(1, 3, h, w, generator=g), "img.camera_mat": K, "img.scale_mat": torch.eye(4)[None],
            "img.idx": torch.tensor([1]), "img.ref_imgs": torch.rand(1, 3, h, w, generator=g),
            "img.ref_idxs": [torch.tensor([2])]}
    world_mat = torch.eye(4, device=DEV)
    world_mat[2, 3] = 1.6
    before = [p.detach().clone() for p in renderer.parameters()]
    for it in (1, 2, 3):
        torch.manual_seed(100 + it)
        (img, ref_img, p, pn, rays_o, rays_d, rays_d_norm, rgb_gt, camera_mat, scale_mat) = tr.process_data(
            data, world_mat, it=it, epoch=0, patch_size=4)
        near, far = tr.near_far_from_sphere(rays_o, rays_d)
        car = tr.get_cos_anneal_ratio(it, 50000)
        z = None
        if it == 1:  # oracle on the same rays and sample positions
            t_rand = torch.rand(rays_o.shape[0], 64, generator=g)
            args = [x.detach().cpu() for x in (rays_o, rays_d, rays_d_norm)]
            zc = O.hierarchical_z(P, args[0], args[1], torch.tensor([0.0]), near.cpu(), far.cpu(), 64, 64, 4, t_rand)
            ref = O.render_core(P, Pc, varc, *args, torch.tensor([0.0]), zc, (far[0, 0] - near[0, 0]).cpu() / 64,
                                float(car))
            loss_ref = O.train_loss(ref, rgb_gt.cpu(), w_edge=0.5, w_smooth=0.5e-4)
            z = zc.to(DEV)
        out = renderer(rays_o, rays_d, rays_d_norm, torch.tensor([0.0], device=DEV), near, far,
                       cos_anneal_ratio=car, it=it, eval=False, z_vals=z)
        normals = out["normals"].view(-1, 3)
        gradient_loss = torch.mean((torch.linalg.norm(normals, ord=2, dim=-1) - 1.0) ** 2)
        d = out["depth_pred"].view(-1, 4, 4, 1)
        gt = rgb_gt.view(-1, 4, 4, 3)
        edge = 1 / 2 * O.edge_smoothness(d, gt)  # 1 / 2**s, s = 1 (train.py:317, 519-525)
        smooth = 1 / 2 * O.smoothness(d)
        zero = torch.zeros((), device=DEV)
        loss_dict = tr.compute_loss(data, out["color_fine"], rgb_gt, gradient_loss, zero, zero, zero, edge, smooth,
                                    it=it)
        if it == 1:
            assert abs(loss_dict["loss"].item() - loss_ref.item()) <= 1e-4 * abs(loss_ref.item())
        tr.backpropagation(loss_dict, train_motion_network=False)
        assert torch.isfinite(loss_dict["loss"]).item()
    assert all(not torch.equal(a, b.detach()) for a, b in zip(before, renderer.parameters()))


def test_dataparallel_wrapped_renderer():
    """train.py:54 wraps the renderer in torch.nn.DataParallel(renderer, device_ids=gpu_ids)
    and calls it as train.py:441-444 does (query time repeated per GPU, background_rgb=None):
    the wrapped HIP renderer returns the bare one's outputs and gradients bit for bit, and
    its state dict carries the `module.` prefix the reference's checkpoints hold."""
    sys.path.insert(0, os.path.join(ROOT, "cope-nerf_amd"))
    from model import MotionNetwork, NeuSRenderer
    from copenerf.train_step import MOTION_CFG
    sdf, col, var = build_modules(21, device=DEV)
    motion = MotionNetwork(**MOTION_CFG).to(DEV)
    renderer = NeuSRenderer(None, sdf, var, col, motion, **REN_CFG).set_mfma_dtype("bf16x6")
    dp = torch.nn.DataParallel(renderer, device_ids=[0])
    assert all(k.startswith("module.") for k in dp.state_dict())
    assert any(k.startswith("module.motion_network.") for k in dp.state_dict())
    g = torch.Generator().manual_seed(22)
    R = 512
    d = torch.cat([(torch.rand(R, 2, generator=g) - 0.5) * 0.5, -torch.ones(R, 1)], -1)
    norm = d.norm(dim=-1, keepdim=True)
    rays_o = torch.tensor([[0.05, -0.03, 1.6]]).expand(R, 3).contiguous().to(DEV)
    rays_d, norm = (d / norm).to(DEV), norm.to(DEV)
    near, far = torch.full((R, 1), 0.01, device=DEV), torch.full((R, 1), 3.0, device=DEV)
    t_rand = torch.rand(R, 64, generator=g).to(DEV)
    q = torch.tensor([0.25], device=DEV).repeat(1)  # query_time_step.repeat(len(gpu_ids))
    res = []
    for mod in (renderer, dp):
        for p in renderer.parameters():
            p.grad = None
        out = mod(rays_o, rays_d, norm, q, near, far, background_rgb=None, cos_anneal_ratio=0.5, it=10, eval=False,
                  t_rand=t_rand)
        loss = out["color_fine"].abs().sum() + out["depth_pred"].sum() + out["normals"].square().sum()
        loss.backward()
        res.append(({k: v.detach().clone() for k, v in out.items() if torch.is_tensor(v)},
                    [p.grad.clone() if p.grad is not None else None for p in renderer.parameters()]))
    (o1, g1), (o2, g2) = res
    assert o1.keys() == o2.keys()
    for k in o1:
        assert torch.equal(o1[k], o2[k]), k
    for a, b in zip(g1, g2):
        assert (a is None and b is None) or torch.equal(a, b)
