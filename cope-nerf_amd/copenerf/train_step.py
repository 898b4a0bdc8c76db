"""One cope-nerf training iteration on synthetic data (the per-iteration
sequence of train.py:407-532 restricted to the rendering hot path):

  schedule                           train.py:409-413, 246-268; training.py:120-124
  patch sampling + ray generation    training.py:413-487      (rays.py, device)
  NeuSRenderer forward               train.py:441-444         (HIP)
  losses: L1 rgb, eikonal, edge-aware + plain depth smoothness on 4x4 patches
                                     training.py:506-533, train.py:519-526   (cn_train_loss)
  stage 1 (optional): scene-flow SDF loss, flow-RGB warp to the next frames and
  SDF consistency at the world frame  train.py:467-517        (motion.py, device)
  backward + Adam                    training.py:552-558      (HIP backward, torch Adam)

Everything per iteration is stream-ordered device work: the iteration's
schedule values (cos_anneal_ratio, learning-rate warm-up, annealed loss
weights, the training image and its time step) live in device tensors
(`Schedule`) that the host updates between steps, and every index-dependent
choice (which pose, which reference frames, whether the SDF-consistency term
applies) is a device-side gather or mask with fixed shapes.  So the whole step
can be captured once into a HIP graph and replayed for any iteration
(`GraphedTrainer`), following the reference's schedule.

Options beyond the C2 headline step:
  joint_pose  learnable SE(3) camera poses (PoseRetriever, poses_retriever.py:6-32)
              produce the rays (train.py:425-431, "query in canonical space"), so
              the HIP backward returns ray gradients into r, t;
  stage1      the MotionNetwork losses of stage 1 (train.py:467-517).

Data-parallel over ranks: every rank trains on the same image
and time step (rank-independent data generator) with its own patches (per-rank
sampling generator); the two global normalisers (Σw of the scene-flow loss,
Σvalid of flow-RGB) are all-reduced before the divide, and the gradients of all
parameters are summed with ONE all-reduce of a flat fp32 bucket (RCCL over xGMI
when the process group is nccl) and divided by the world size -- exactly the
single-GPU gradient of the loss over all ranks' rays.
"""
from __future__ import annotations


import numpy as np
import torch
import torch.distributed as dist

from .fields import RenderingNetwork, SDFNetwork, SingleVarianceNetwork
from .losses import EdgePreservingSmoothnessLoss, SmoothnessLoss, eikonal_loss, rgb_l1, train_losses
from .motion import (MotionNetwork, affine_points, flow_rgb_loss, masked_chain, mat4_chain, project_flow,
                     project_flow_sums,
                     scene_flow_loss, stage1_terms_fused)
from .rays import PoseRetriever, get_patch_indices, intrinsics_ndc, inv4x4, pixels_from_indices, world_rays
from .renderer import NeuSRenderer

SDF_CFG = dict(d_in=4, d_out=257, d_hidden=256, n_layers=8, skip_in=[4], multires=6, bias=0.5, scale=1.0,
               geometric_init=True, weight_norm=True)
COL_CFG = dict(d_feature=256, mode="idr", d_in=11, d_out=3, d_hidden=256, n_layers=4, weight_norm=True,
               multires_view=4, squeeze_out=True, use_negative_ray_vector=False)
REN_CFG = dict(n_samples=64, n_importance=64, n_outside=0, up_sample_steps=4, perturb=1.0,
               n_max_network_queries=64000, importance_sampling_start=0, naive_render=False)
MOTION_CFG = dict(d_out=6, d_in=1, d_hidden=256, n_layers=4, skip_in=[2], multires=6, bias=0.5, scale=1.0,
                  geometric_init=False, weight_norm=True)  # default.yaml:113-123
# default.yaml:31-57 (training) and 158 (neus_anneal_end)
TRAIN_CFG = dict(learning_rate=1e-3, pose_learning_rate=5e-4, rgb_weight=1.0, eikonal_weight=0.1,
                 sdf_weight=(0.1, 0.1), flow_rgb_weight=(7.5, 7.5), sdf_consistency_weight=(0.0, 1.0),
                 edge_aware_smoothness_weight=(1.0, 0.0), smoothness_weight=(1e-4, 0.0), nb_warm_up_it=5000,
                 nb_sample_timestep=10, end_sdf_weight_increase_iteration=100000,
                 end_consistency_weight_increase_iteration=100000, patch_size=4, world_idx="mid",
                 random_ref_interval=(1, 2, 3), neus_anneal_end=50000, s=1,
                 sdf_consistency_enable_pose_grad=False)
PAIR_WEIGHTS = ("sdf_weight", "flow_rgb_weight", "sdf_consistency_weight", "edge_aware_smoothness_weight",
                "smoothness_weight")


class small_gemm_blas:
    """torch's fp32 GEMMs of a step (the MotionNetwork's layers and their gradients, ray and pose matrices: tens
    to a few hundred rows) through rocBLAS instead of hipBLASLt for the duration of a `with` block, the caller's
    preferred library restored on exit: hipBLASLt's tiles for these shapes run ~30 us each, rocBLAS's in a few
    (C3 +1.9 %, profiles/r5_ab.txt r5q; both fp32).  torch's setting is process-wide, so the trainers scope it
    to their own steps (SyntheticTrainer(small_gemm_blas=True), the default; the reference-API Trainer only on
    request) instead of leaving it switched for the rest of the process.  Re-entrant."""

    def __init__(self, enabled=True):
        self.enabled = enabled and torch.cuda.is_available()
        self.prev = None

    def __enter__(self):
        if self.enabled:
            self.prev = torch.backends.cuda.preferred_blas_library()
            torch.backends.cuda.preferred_blas_library("cublas")  # (rocBLAS on ROCm)
        return self

    def __exit__(self, *exc):
        if self.enabled:
            torch.backends.cuda.preferred_blas_library(self.prev)
        return False


def normalise_train_cfg(cfg):
    """Accept the reference's cfg['training'] as it is (default.yaml:40-46 stores every loss
    weight as a [start, end] pair): rgb / eikonal weights use their first entry
    (training.py:37-38 reads cfg[...][0]); the annealed weights are pairs (a scalar w
    becomes (w, w))."""
    out = dict(cfg)
    for k in ("rgb_weight", "eikonal_weight"):
        if isinstance(out[k], (list, tuple)):
            out[k] = out[k][0]
    for k in PAIR_WEIGHTS:
        if not isinstance(out[k], (list, tuple)):
            out[k] = (out[k], out[k])
    out["random_ref_interval"] = tuple(int(j) for j in out["random_ref_interval"])
    if not out["random_ref_interval"] or min(out["random_ref_interval"]) < 1:
        raise ValueError(f"random_ref_interval must be positive frame offsets (got {out['random_ref_interval']})")
    return out


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


def scalar_annealing(it, start_anneal, end_anneal, start_weight, end_weight):
    """train.py:246-249."""
    it = np.clip(it, start_anneal, end_anneal)
    return start_weight + (end_weight - start_weight) * np.clip(
        (it - start_anneal) / (end_anneal - start_anneal + 1e-10), 0, 1)


class Schedule:
    """The per-iteration values of the reference's loop in device memory:
      car        cos_anneal_ratio = min(1, it / anneal_end)          training.py:120-124
      lr_factor  clip(it / nb_warm_up_it, 0, 1) while it <= warm-up   train.py:265-268, 411-413
      loss_w     (rgb, eikonal, edge / 2^s, smooth / 2^s)              training.py:37-44, train.py:519-525
      stage1_w   (sdf, flow_rgb, sdf_consistency) with the linear ramps of train.py:251-263
      img        the training image index, t its time step           train.py:415-419
    `fixed=True` keeps car / weights / lr constant (the bench workloads)."""

    def __init__(self, device, cfg, n_images, fixed_car=None):
        self.cfg = cfg
        self.n_images = n_images
        self.fixed_car = fixed_car
        self.car = torch.zeros(1, device=device)
        self.loss_w = torch.zeros(4, device=device)
        self.stage1_w = torch.zeros(3, device=device)
        self.img = torch.zeros(1, dtype=torch.long, device=device)
        self.t = torch.zeros(1, device=device)
        self.lr_factor = 1.0
        self._last = {}  # host copies of what the device tensors hold: write only what changes

    def values(self, it, image_idx):
        c = self.cfg
        car = self.fixed_car if self.fixed_car is not None else (
            1.0 if c["neus_anneal_end"] == 0 else float(min(1.0, it / c["neus_anneal_end"])))
        sc = 1.0 / (2 ** c["s"])
        loss_w = [c["rgb_weight"], c["eikonal_weight"], c["edge_aware_smoothness_weight"][0] * sc,
                  c["smoothness_weight"][0] * sc]
        sdf_w = c["sdf_weight"][0]
        if c["end_sdf_weight_increase_iteration"] != -1:
            sdf_w = scalar_annealing(it, 0.0, c["end_sdf_weight_increase_iteration"], *c["sdf_weight"])
        cons_w = c["sdf_consistency_weight"][0]
        if c["end_consistency_weight_increase_iteration"] != -1:
            cons_w = scalar_annealing(it, 0.0, c["end_consistency_weight_increase_iteration"],
                                      *c["sdf_consistency_weight"])
        t = image_idx / (self.n_images - 1) * 2 - 1
        return dict(car=car, loss_w=loss_w, stage1_w=[float(sdf_w), c["flow_rgb_weight"][0], float(cons_w)],
                    img=image_idx, t=t)

    def set(self, it, image_idx):
        """Write iteration `it`'s values into the device tensors (host -> device fills,
        outside any captured graph); returns the warm-up learning-rate factor."""
        v = self.values(it, image_idx)
        # fill kernels with the value as an argument: asynchronous, no pageable copy (which
        # would stall the host behind the queue every step); unchanged values are skipped
        items = [(("car", 0), self.car, 0, v["car"]), (("img", 0), self.img, 0, int(image_idx)),
                 (("t", 0), self.t, 0, float(v["t"]))]
        items += [(("loss_w", k), self.loss_w, k, float(x)) for k, x in enumerate(v["loss_w"])]
        items += [(("stage1_w", k), self.stage1_w, k, float(x)) for k, x in enumerate(v["stage1_w"])]
        for key, ten, k, x in items:
            if self._last.get(key) != x:
                ten[k].fill_(x)
                self._last[key] = x
        if self.fixed_car is None and it <= self.cfg["nb_warm_up_it"]:
            self.lr_factor = float(np.clip(it / self.cfg["nb_warm_up_it"], 0, 1))
        return self.lr_factor


class SyntheticTrainer:
    """The training loop of train.py on a synthetic multi-frame scene: n_images
    random 540x960 frames with identical intrinsics (fx = fy = 0.9 W), one
    frame per iteration (cycling), 4x4 patches.  `schedule="fixed"` (the bench
    workloads: cos_anneal_ratio 0.5, constant learning rate) or "reference"
    (the reference's warm-up and annealing from iteration `start_it`)."""

    def __init__(self, device, rays=4096, H=540, W=960, patch=4, seed=678, depth_range=(0.01, 5.0),
                 cos_anneal_ratio=0.5, schedule="fixed", start_it=0, distributed=False, group=None,
                 sdf_cfg=None, col_cfg=None, ren_cfg=None, joint_pose=False, stage1=False, n_images=10,
                 capturable=False, mfma_dtype="fp32", train_cfg=None, stage1_fused=True, small_gemm_blas=True):
        if schedule not in ("fixed", "reference"):
            raise ValueError(f"schedule must be 'fixed' or 'reference' (got {schedule!r})")
        self.small_gemm_blas = small_gemm_blas  # rocBLAS for torch's small GEMMs inside the steps only
        self.device = torch.device(device)
        self.R, self.H, self.W, self.patch = rays, H, W, patch
        self.depth_range = depth_range
        self.cfg = normalise_train_cfg(dict(TRAIN_CFG, **(train_cfg or {})))
        self.distributed = distributed
        self.group = (group if group is not None else dist.group.WORLD) if distributed else None
        self.rank = dist.get_rank(self.group) if distributed else 0
        torch.manual_seed(seed)
        self.sdf = SDFNetwork(**(sdf_cfg or SDF_CFG)).to(self.device)
        self.col = RenderingNetwork(**(col_cfg or COL_CFG)).to(self.device)
        self.var = SingleVarianceNetwork(0.3).to(self.device)
        self.renderer = NeuSRenderer(None, self.sdf, self.var, self.col, None, **(ren_cfg or REN_CFG)).to(self.device)
        self.renderer.set_mfma_dtype(mfma_dtype)
        self.renderer.expose_sdf_pack = stage1  # the stage-1 SDF re-query reuses the step's weight images
        self.params = list(self.sdf.parameters()) + list(self.var.parameters()) + list(self.col.parameters())
        self.joint_pose, self.stage1 = joint_pose, stage1
        # stage-1 per-sample terms in the fused HIP pass; stage1_fused=False keeps the torch
        # expressions (device ops too: the parity test's reference, tests/test_gpu_stage1_fused.py)
        self.stage1_fused = stage1_fused
        self.n_images = n_images
        self.nst = self.cfg["nb_sample_timestep"]
        wi = self.cfg["world_idx"]
        self.world_cam_idx = n_images // 2 if wi == "mid" else int(wi)  # train.py:85-86
        self.world_time_step = self.world_cam_idx / (n_images - 1) * 2 - 1  # train.py:91
        self.capturable = capturable
        lr = self.cfg["learning_rate"]
        lr0 = torch.tensor(lr, device=self.device) if capturable else lr
        groups = [{"params": self.params, "lr": lr0}]
        self.base_lr = [lr]
        if joint_pose:
            self.poses = PoseRetriever(n_images).to(self.device)
            with torch.no_grad():  # a non-trivial starting pose per camera
                g = torch.Generator().manual_seed(seed + 1)
                self.poses.r.copy_(0.02 * torch.randn(n_images, 3, generator=g))
                self.poses.t.copy_(0.02 * torch.randn(n_images, 3, generator=g))
            groups.append({"params": [self.poses.r, self.poses.t],
                           "lr": torch.tensor(lr, device=self.device) if capturable else lr})
            self.base_lr.append(lr)
        if stage1:
            self.motion = MotionNetwork(**MOTION_CFG).to(self.device)
            mlr = self.cfg["pose_learning_rate"]  # train.py:57-60: the motion optimizer's lr
            groups.append({"params": list(self.motion.parameters()),
                           "lr": torch.tensor(mlr, device=self.device) if capturable else mlr})
            self.base_lr.append(None)  # the warm-up does not touch the motion optimizer (train.py:268-270)
            self.steps_grid, self.dts = self.motion.interval_time_grid(n_images, self.nst)
            self.ref_intervals = torch.tensor(self.cfg["random_ref_interval"], device=self.device)
            self.chain_steps = torch.arange(max(self.cfg["random_ref_interval"]), device=self.device)
        self.all_params = [p for g in groups for p in g["params"]]
        # torch's fused multi-tensor Adam: one kernel chain per step instead of the foreach
        # implementation's ~8 launches (same update rule, training.py:552-558 / train.py:57-60)
        self.opt = torch.optim.Adam(groups, lr=lr, capturable=capturable, fused=True)
        # data: rank-independent (every rank sees the same frames); sampling: per rank
        gdata = torch.Generator(device=self.device).manual_seed(seed)
        self.images = torch.rand(n_images, 3, H, W, device=self.device, generator=gdata)
        self.gen = torch.Generator(device=self.device).manual_seed(seed + 7919 * (self.rank + 1))
        f = 0.9 * W
        self.K = intrinsics_ndc(f, f, W, H, device=self.device)
        self.camera_mats = self.K.expand(n_images, 4, 4).contiguous()
        self.I = torch.eye(4, device=self.device)
        self.sched = Schedule(self.device, self.cfg, n_images,
                              fixed_car=cos_anneal_ratio if schedule == "fixed" else None)
        self.nonfinite = torch.zeros(1, dtype=torch.int32, device=self.device)
        self.edge = EdgePreservingSmoothnessLoss(patch)
        self.smooth = SmoothnessLoss(patch)
        self.it = start_it
        self.it_captured = None

    # -- host side: the iteration's schedule -------------------------------
    def image_index(self, it):
        """The frame of iteration it (the reference's shuffled loader; here cycling)."""
        return (it - 1) % self.n_images

    def begin_iteration(self):
        """train.py:409-413: it += 1, loss-weight annealing, learning-rate warm-up --
        written into device memory (Schedule) and the optimizer's lr."""
        self.it += 1
        f = self.sched.set(self.it, self.image_index(self.it))
        for g, base in zip(self.opt.param_groups, self.base_lr):
            if base is None:
                continue
            if torch.is_tensor(g["lr"]):
                if g.get("_lr_host") != base * f:
                    g["lr"].fill_(base * f)
                    g["_lr_host"] = base * f
            else:
                g["lr"] = base * f

    # -- device side: one iteration ------------------------------------------
    def make_batch(self):
        idx = get_patch_indices(self.H, self.W, self.patch, self.R, generator=self.gen, device=self.device)
        pix, pixn = pixels_from_indices(idx, self.H, self.W)
        # the stratified jitter from the trainer's own generator (neus_renderer.py:482 draws it
        # with the global RNG): per rank in data parallel, and replayed graphs advance it
        t_rand = torch.rand(self.R, self.renderer.n_samples, generator=self.gen, device=self.device)
        return self.batch_from_pixels(pix, pixn, t_rand)

    def batch_from_pixels(self, pix, pixn, t_rand=None):
        """Rays of the current frame's camera through the pixels pix [R,2] (x, y; normalised
        pixn) and their ground-truth colours (training.py:439-471)."""
        img = self.sched.img
        pix = pix.long()
        if self.joint_pose:  # identity for the world camera (train.py:425-429)
            world_mat = torch.where(img.view(1, 1) == self.world_cam_idx, self.I, self.poses.pose_at(img))
        else:
            world_mat = self.I
        rays_o, rays_d, norm = world_rays(pixn, self.K, world_mat, self.I)
        frame = self.images.index_select(0, img)[0]
        rgb_gt = frame[:, pix[:, 1], pix[:, 0]].t().contiguous()
        return dict(rays_o=rays_o, rays_d=rays_d, norm=norm, rgb_gt=rgb_gt, pix=pix.float(), pixn=pixn, t_rand=t_rand)

    def query_time(self):
        """train.py:440: the frame's time step in stage 1, the world time step when
        querying in canonical space (joint pose), else 0 (the single-frame C2 scene)."""
        if self.stage1:
            return self.sched.t
        if self.joint_pose:
            return torch.full((1,), self.world_time_step, device=self.device)
        return torch.zeros(1, device=self.device)

    def loss(self, out, rgb_gt):
        """L1 rgb + eikonal + edge-aware / plain depth smoothness (training.py:506-533,
        train.py:519-526) in one HIP call with the schedule's device weights."""
        return train_losses(out["color_fine"], rgb_gt, out["depth_pred"], out["normals"], patch=self.patch,
                            weights=self.sched.loss_w, nonfinite=self.nonfinite)

    def loss_torch(self, out, rgb_gt):
        """The same sum as torch expressions of the reference's loss classes (host weights)."""
        w = self.sched.values(max(self.it, 1), 0)["loss_w"]
        loss = w[0] * rgb_l1(out["color_fine"], rgb_gt) + w[1] * eikonal_loss(out["normals"])
        if self.patch > 1:
            d = out["depth_pred"].view(-1, self.patch, self.patch, 1)
            g = rgb_gt.view(-1, self.patch, self.patch, 3)
            loss = loss + w[2] * self.edge(d, g) + w[3] * self.smooth(d)
        return loss

    def stage1_terms(self, out, batch):
        """(sdf_loss, flow_rgb_loss, sdf_consistency_loss) of train.py:467-517 with the
        image index on the device: all K = n_images - 1 consecutive relative poses
        come from one batched motion-network evaluation; the reference frames i+1..i+3
        (dataset.py:231-250) are gathered and masked by validity; the consistency
        chain between the world camera and frame i is a masked product."""
        grp = self.group  # None without data parallel
        n = self.n_images
        img = self.sched.img
        R = batch["rgb_gt"].shape[0]
        # one motion-network evaluation: the K*n Euler time steps and the frame's own time
        P, (omega, vel) = self.motion.batched_relative_poses(self.steps_grid, self.dts, extra_t=self.sched.t)
        K = P.shape[0]
        # flow-RGB: reference frame i + j maps through w2c_j = P[i+j-1] @ ... @ P[i]
        # (compute_w2c_mappings(c2c)[ref - i], train.py:483): the running product up to the
        # largest interval, taken at each interval (any random_ref_interval, e.g. [1, 5, 10])
        js = self.ref_intervals
        ref = img + js                                    # [T]
        valid = (ref <= n - 1)                            # next_time_step <= 1 (train.py:421)
        # (one launch each way: motion.mat4_chain over the gathered poses)
        k = torch.clamp(img + self.chain_steps, max=K - 1)  # past the last frame: masked by `valid`
        w2c = mat4_chain(P.index_select(0, k)).index_select(0, self.ref_intervals - 1)
        refc = torch.clamp(ref, max=n - 1)
        # SDF consistency at the world frame (train.py:495-505): with
        # sdf_consistency_enable_pose_grad (most dataset configs, e.g. Co3D/skateboard.yaml:27)
        # the loss reaches the motion network through c2c, i.e. through the SDF's input
        # gradient at the world points; default.yaml:62 detaches the chain
        w = self.world_cam_idx
        pose_grad = bool(self.cfg["sdf_consistency_enable_pose_grad"]) and torch.is_grad_enabled()
        with torch.set_grad_enabled(pose_grad):
            lo, hi = torch.clamp(img, max=w), torch.clamp(img, min=w)
            c2c = masked_chain(P, lo, hi)
            cw2 = torch.where(img.view(1, 1) >= w, inv4x4(c2c), c2c)
        pts = out["sampled_points"]
        if self.stage1_fused:
            # one HIP pass each way over the samples (cn_stage1_fwd / cn_stage1_bwd)
            sdf_loss, pbar, wbar, x = stage1_terms_fused(pts, out["normals"], out["sdf_flows"], out["weights"], omega,
                                                         vel, cw2, self.world_time_step, pose_grad, group=grp)
            flows = project_flow_sums(pbar, wbar, w2c, self.camera_mats.index_select(0, refc), self.I, batch["pixn"],
                                      (self.H, self.W))
        else:  # the same terms as torch expressions (the parity test's reference: stage1_fused=False)
            sdf_loss = scene_flow_loss(pts, out["normals"], out["sdf_flows"], out["weights"], omega, vel, group=grp)
            flows = project_flow(pts, out["weights"], w2c, self.camera_mats.index_select(0, refc), self.I,
                                 batch["pixn"], (self.H, self.W))
            with torch.set_grad_enabled(pose_grad):
                pw = affine_points(pts.reshape(-1, 3), cw2)
                x = torch.cat([pw, torch.full_like(pw[:, :1], self.world_time_step)], 1)
        per = flow_rgb_loss(flows, batch["pix"], self.images.index_select(0, refc), batch["rgb_gt"], group=grp)
        flow_rgb = torch.where(valid, per, torch.zeros_like(per)).sum() / 3.0
        # SDFNetwork.sdf (train.py:504) on the weights the renderer packed for this step
        pack, self.renderer.last_sdf_pack = self.renderer.last_sdf_pack, None
        sdf_w = self.sdf.field(x, want_feat=False, want_grad=False, packed=pack)[0]
        cons = torch.mean(torch.abs(sdf_w - out["sdf"].reshape(-1, 1))) * (img != w).float().view(())
        return sdf_loss, flow_rgb, cons

    def iteration(self, batch, t_rand=None, z_vals=None, return_out=False):
        """Forward, losses, backward, gradient all-reduce and Adam for one batch
        (t_rand / z_vals: the renderer's test hooks, e.g. to pin sample positions)."""
        with small_gemm_blas(self.small_gemm_blas):
            return self._iteration(batch, t_rand, z_vals, return_out)

    def _iteration(self, batch, t_rand, z_vals, return_out):
        near_far = (torch.full((batch["rays_o"].shape[0], 1), float(self.depth_range[0]), device=self.device),
                    torch.full((batch["rays_o"].shape[0], 1), float(self.depth_range[1]), device=self.device))
        if t_rand is None:
            t_rand = batch.get("t_rand")
        out = self.renderer(batch["rays_o"], batch["rays_d"], batch["norm"], self.query_time(), *near_far,
                            cos_anneal_ratio=self.sched.car, it=max(self.it, 0), eval=False, t_rand=t_rand,
                            z_vals=z_vals)
        loss = self.loss(out, batch["rgb_gt"])
        if self.stage1:
            l_sdf, l_flow, l_cons = self.stage1_terms(out, batch)
            w = self.sched.stage1_w
            loss = loss + w[0] * l_sdf + w[1] * l_flow + w[2] * l_cons
            # cn_train_loss flags its own terms; the stage-1 terms are added here (device op,
            # no host sync, capturable; training.py:532 asserts on the total)
            self.nonfinite.bitwise_or_((~torch.isfinite(loss)).to(torch.int32).view(1))
        self.opt.zero_grad(set_to_none=True)
        loss.backward()
        if self.distributed:
            flat_allreduce_mean(self.all_params, self.group)
        self.opt.step()
        return (loss, out) if return_out else loss

    def device_step(self):
        """The capturable part of an iteration (no host work)."""
        with small_gemm_blas(self.small_gemm_blas):
            return self.iteration(self.make_batch())

    def step(self):
        self.begin_iteration()
        return self.device_step()

    def check_finite(self):
        """Raise if any loss since the last check was not finite (the device form of
        training.py:532-533's assert; one host sync)."""
        if int(self.nonfinite.item()):
            self.nonfinite.zero_()
            raise FloatingPointError("Nan loss found")


class GraphedTrainer:
    """The whole training step -- patch sampling and ray generation, the HIP
    sampler / renderer forward, losses (and the stage-1 terms), the HIP backward,
    the data-parallel gradient all-reduce and Adam -- captured once into a HIP
    graph and replayed (config C5).

    Every replay follows the reference's schedule: before each replay the host
    writes the iteration's values into the trainer's device tensors (Schedule:
    cos_anneal_ratio, annealed loss weights, image index / time step; the Adam
    learning-rate tensors), which the captured kernels read.  The RNG (patch
    corners, stratified jitter) draws from generators registered with the graph,
    so every replay advances their Philox offsets; Adam runs with capturable=True
    and tensor learning rates.  With distributed=True the flat all-reduce of the
    gradients is captured too (RCCL collectives are graph-capturable on the nccl
    backend), as are the scalar all-reduces of the stage-1 normalisers.  The
    renderer's `it >= importance_sampling_start` branch is fixed at capture.

    The caller must not hold a loss (or any output) of an earlier eager step: a
    live autograd graph keeps the leaves' AccumulateGrad nodes bound to the stream
    they were created on, and capture then records work on two streams."""

    def __init__(self, trainer: SyntheticTrainer, warmup: int = 3):
        if not trainer.capturable:
            raise ValueError("GraphedTrainer needs SyntheticTrainer(capturable=True) (tensor learning rates)")
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
        trainer.begin_iteration()  # the captured step is this iteration's
        with torch.cuda.graph(self.graph):
            loss = trainer.device_step()
        # the replays write the loss into this static storage; a detached view keeps it without the
        # captured step's autograd graph, whose AccumulateGrad nodes would stay bound to the capture
        # stream (an eager step afterwards -- bench.py's instrumented pass -- would then warn and sync)
        self.loss = loss.detach()
        del loss
        torch.cuda.synchronize(trainer.device)
        self.graph.replay()  # capture records without executing: run the captured iteration once

    def step(self):
        self.tr.begin_iteration()
        self.graph.replay()
        return self.loss
