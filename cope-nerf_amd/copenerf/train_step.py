"""One cope-nerf training iteration on synthetic data (the per-iteration
sequence of train.py:407-532 restricted to the rendering hot path):

  patch sampling + ray generation   training.py:413-487      (rays.py, device)
  NeuSRenderer forward               train.py:441-444         (HIP)
  losses: L1 rgb, eikonal, edge-aware + plain depth smoothness on 4x4 patches
                                     training.py:506-533, train.py:519-526
  backward + Adam                    training.py:552-558      (HIP backward, torch Adam)

Options beyond the C2 headline step:
  joint_pose  learnable SE(3) camera poses (PoseRetriever, poses_retriever.py:6-32)
              produce the rays, so the HIP backward returns ray gradients into r, t
              (train.py:425-431, stage 2 "query in canonical space");
  stage1      MotionNetwork scene-flow loss and SDF-consistency re-query at the
              world points of the motion-integrated relative pose (train.py:467-505).

Data-parallel over ranks: each rank renders its own R rays;
gradients of SDF + colour + variance are summed with ONE all-reduce of a flat
fp32 bucket (RCCL over xGMI when the process group is nccl) and divided by the
world size, which equals the gradient of the mean loss over all ranks' rays.
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from .fields import RenderingNetwork, SDFNetwork, SingleVarianceNetwork
from .losses import EdgePreservingSmoothnessLoss, SmoothnessLoss, eikonal_loss, rgb_l1, train_losses
from .motion import MotionNetwork, scene_flow_loss, world_points
from .rays import (PoseRetriever, get_patch_indices, inv4x4, intrinsics_ndc, near_far_from_sphere, pixels_from_indices,
                   world_rays)
from .renderer import NeuSRenderer

SDF_CFG = dict(d_in=4, d_out=257, d_hidden=256, n_layers=8, skip_in=[4], multires=6, bias=0.5, scale=1.0,
               geometric_init=True, weight_norm=True)
COL_CFG = dict(d_feature=256, mode="idr", d_in=11, d_out=3, d_hidden=256, n_layers=4, weight_norm=True,
               multires_view=4, squeeze_out=True, use_negative_ray_vector=False)
REN_CFG = dict(n_samples=64, n_importance=64, n_outside=0, up_sample_steps=4, perturb=1.0,
               n_max_network_queries=64000, importance_sampling_start=0, naive_render=False)
MOTION_CFG = dict(d_out=6, d_in=1, d_hidden=256, n_layers=4, skip_in=[2], multires=6, bias=0.5, scale=1.0,
                  geometric_init=False, weight_norm=True)  # default.yaml:113-123


def flat_allreduce_mean(params, group=None):
    """Sum every gradient across ranks in one flat bucket, then divide by world size."""
    grads = [p.grad for p in params if p.grad is not None]
    if not grads:
        return
    world = dist.get_world_size(group)
    flat = torch.cat([g.reshape(-1) for g in grads])
    dist.all_reduce(flat, op=dist.ReduceOp.SUM, group=group)
    flat.div_(world)
    views = [v.view_as(g) for v, g in zip(flat.split([g.numel() for g in grads]), grads)]
    torch._foreach_copy_(grads, views)  # one multi-tensor launch instead of a copy per parameter


class SyntheticTrainer:
    def __init__(self, device, rays=4096, H=540, W=960, patch=4, seed=678, depth_range=(0.01, 5.0),
                 cos_anneal_ratio=0.5, lr=1e-3, weights=dict(rgb=1.0, eikonal=0.1, edge=1.0, smooth=1e-4),
                 distributed=False, sdf_cfg=None, col_cfg=None, ren_cfg=None, joint_pose=False, stage1=False,
                 n_images=10, nb_sample_timestep=10, sdf_weight=0.1, sdf_consistency_weight=1.0,
                 capturable=False, mfma_dtype="fp32"):
        self.device = torch.device(device)
        self.R, self.H, self.W, self.patch = rays, H, W, patch
        self.depth_range = depth_range
        self.car = cos_anneal_ratio
        self.w = weights
        self.distributed = distributed
        torch.manual_seed(seed)
        self.sdf = SDFNetwork(**(sdf_cfg or SDF_CFG)).to(self.device)
        self.col = RenderingNetwork(**(col_cfg or COL_CFG)).to(self.device)
        self.var = SingleVarianceNetwork(0.3).to(self.device)
        self.renderer = NeuSRenderer(None, self.sdf, self.var, self.col, None, **(ren_cfg or REN_CFG)).to(self.device)
        self.renderer.set_mfma_dtype(mfma_dtype)
        self.params = list(self.sdf.parameters()) + list(self.var.parameters()) + list(self.col.parameters())
        self.joint_pose, self.stage1 = joint_pose, stage1
        self.n_images, self.nb_sample_timestep = n_images, nb_sample_timestep
        self.sdf_weight, self.cons_weight = sdf_weight, sdf_consistency_weight
        groups = [{"params": self.params, "lr": lr}]
        if joint_pose:
            self.poses = PoseRetriever(n_images).to(self.device)
            with torch.no_grad():  # a non-trivial starting pose per camera
                g = torch.Generator().manual_seed(seed + 1)
                self.poses.r.copy_(0.02 * torch.randn(n_images, 3, generator=g))
                self.poses.t.copy_(0.02 * torch.randn(n_images, 3, generator=g))
            groups.append({"params": [self.poses.r, self.poses.t], "lr": lr})
        if stage1:
            self.motion = MotionNetwork(**MOTION_CFG).to(self.device)
            groups.append({"params": list(self.motion.parameters()), "lr": 5e-4})
        self.all_params = [p for g in groups for p in g["params"]]
        self.opt = torch.optim.Adam(groups, lr=lr, capturable=capturable)
        gen = torch.Generator(device=self.device).manual_seed(seed + (dist.get_rank() if distributed else 0))
        self.gen = gen
        self.image = torch.rand(3, H, W, device=self.device, generator=gen)
        f = 0.9 * W
        self.K = intrinsics_ndc(f, f, W, H, device=self.device)
        self.I = torch.eye(4, device=self.device)
        self.time_step = torch.zeros(1, device=self.device)
        self.edge = EdgePreservingSmoothnessLoss(patch)
        self.smooth = SmoothnessLoss(patch)
        self.it = 0

    def image_index(self):
        return 1 + self.it % (self.n_images - 1)

    def make_batch(self):
        idx = get_patch_indices(self.H, self.W, self.patch, self.R, generator=self.gen, device=self.device)
        pix, pixn = pixels_from_indices(idx, self.H, self.W)
        world_mat = self.poses(self.image_index()) if self.joint_pose else self.I
        rays_o, rays_d, norm = world_rays(pixn, self.K, world_mat, self.I)
        rgb_gt = self.image[:, pix[:, 1], pix[:, 0]].t().contiguous()
        return rays_o, rays_d, norm, rgb_gt

    def loss(self, out, rgb_gt):
        """L1 rgb + eikonal + edge-aware / plain depth smoothness (training.py:506-533,
        train.py:519-526) in one HIP call; `loss_torch` is the same sum as torch
        expressions of the reference's loss classes."""
        w = self.w
        return train_losses(out["color_fine"], rgb_gt, out["depth_pred"], out["normals"], w_rgb=w["rgb"],
                            w_eik=w["eikonal"], w_edge=w["edge"], w_smooth=w["smooth"], patch=self.patch)

    def loss_torch(self, out, rgb_gt):
        w = self.w
        loss = w["rgb"] * rgb_l1(out["color_fine"], rgb_gt) + w["eikonal"] * eikonal_loss(out["normals"])
        if self.patch > 1:
            d = out["depth_pred"].view(-1, self.patch, self.patch, 1)
            g = rgb_gt.view(-1, self.patch, self.patch, 3)
            loss = loss + w["edge"] * self.edge(d, g) + w["smooth"] * self.smooth(d)
        return loss

    def stage1_losses(self, out):
        """Scene-flow SDF loss and SDF consistency at the world points (train.py:467-505)."""
        img = self.image_index()
        t = torch.tensor([[img / (self.n_images - 1) * 2 - 1]], device=self.device)
        omega, vel = self.motion(t)
        pts, normals = out["sampled_points"], out["normals"]
        l_sf = scene_flow_loss(pts, normals, out["sdf_flows"], out["weights"], omega, vel)
        _, rel = self.motion.compute_relative_camera_pose(0, img, self.n_images, self.nb_sample_timestep)
        c2c = self.motion.compute_w2c_mappings(rel)[-1]
        pw = world_points(pts, inv4x4(c2c))
        t_world = torch.full((pw.shape[0], 1), -1.0, device=self.device)
        sdf_w = self.sdf.sdf(torch.cat([pw, t_world], 1))
        l_cons = torch.mean(torch.abs(sdf_w - out["sdf"]))
        return self.sdf_weight * l_sf + self.cons_weight * l_cons

    def step(self):
        rays_o, rays_d, norm, rgb_gt = self.make_batch()
        near, far = near_far_from_sphere(rays_o, self.depth_range)
        t = self.time_step
        if self.stage1:  # stage 1 queries the SDF at the frame's own time step (train.py:440)
            t = torch.full((1,), self.image_index() / (self.n_images - 1) * 2 - 1, device=self.device)
        out = self.renderer(rays_o, rays_d, norm, t, near, far, cos_anneal_ratio=self.car, it=self.it,
                            eval=False)
        loss = self.loss(out, rgb_gt)
        if self.stage1:
            loss = loss + self.stage1_losses(out)
        self.opt.zero_grad(set_to_none=True)
        loss.backward()
        if self.distributed:
            flat_allreduce_mean(self.all_params)
        self.opt.step()
        self.it += 1
        return loss


class GraphedTrainer:
    """The whole training step -- patch sampling and ray generation, the HIP
    sampler / renderer forward, losses, the HIP backward and Adam -- captured
    once into a HIP graph and replayed (config C5).

    Everything on the step is stream-ordered device work on torch's current
    stream with no host synchronisation: the library launches on the stream it
    is given and allocates nothing, the RNG (patch corners, stratified jitter)
    draws from generators registered with the graph so every replay advances
    their Philox offsets, and Adam runs with capturable=True.  Buffers come from
    the graph's private pool, so the replayed addresses are the captured ones.
    Not supported with distributed=True (the all-reduce is left eager).  The
    caller must not hold a loss (or any output) of an earlier eager step: a live
    autograd graph keeps the leaves' AccumulateGrad nodes bound to the stream
    they were created on, and capture then records work on two streams."""

    def __init__(self, trainer: SyntheticTrainer, warmup: int = 3):
        if trainer.distributed:
            raise NotImplementedError("GraphedTrainer: capture the single-GPU step; DP all-reduce stays eager")
        self.tr = trainer
        s = torch.cuda.Stream(device=trainer.device)
        s.wait_stream(torch.cuda.current_stream(trainer.device))
        with torch.cuda.stream(s):
            for _ in range(warmup):
                trainer.step()  # result dropped: no autograd graph outlives its step
        torch.cuda.current_stream(trainer.device).wait_stream(s)
        torch.cuda.synchronize(trainer.device)
        self.graph = torch.cuda.CUDAGraph()
        reg = getattr(self.graph, "register_generator_state", None)
        if reg is not None:
            reg(trainer.gen)
        trainer.opt.zero_grad(set_to_none=True)
        with torch.cuda.graph(self.graph):
            self.loss = trainer.step()

    def step(self):
        self.graph.replay()
        self.tr.it += 1
        return self.loss
