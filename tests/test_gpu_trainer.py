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
