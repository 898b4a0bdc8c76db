"""Trainer: drop-in for the reference's model.training.Trainer (model/training.py:15-558).

train.py constructs it as `mdl.Trainer(renderer, optimizer, motion_optimizer,
cfg['training'], device=..., total_nb_images=..., cfg_all=cfg, logger=...,
gt_depths=..., world_cam_idx=..., train_dataset=...)` (train.py:102) and, per
iteration, calls process_data (train.py:433-435), near_far_from_sphere and
get_cos_anneal_ratio (train.py:437-438), compute_loss (train.py:528) and
backpropagation (train.py:532).  Those methods keep the reference's
signatures, argument meaning and return values; underneath, rays come from the
device-side ray generation of copenerf/rays.py (no full-image pixel grid, no
torch.inverse) and the renderer they feed is the HIP NeuSRenderer.

Differences, by design:
  * get_patch_indices draws the patch corners with torch.randperm on the CPU
    exactly as training.py:422 (so a seeded run samples the reference's patches)
    unless `patch_rng="device"` (cn_patch_indices: the first corners of a keyed
    pseudo-random permutation, one launch, no host sync).
  * compute_loss checks for NaN like training.py:532-533 (`nan_check="sync"`,
    the default: AssertionError at once) or sets a device flag without a host
    sync (`nan_check="deferred"`, for captured steps; `check_finite()` raises).
  * render_visdata / the visualisation helpers (training.py:157-374: cv2,
    imageio, matplotlib output) are outside the hot path; copenerf.inference
    renders full images on the device.
"""
from __future__ import annotations

import numpy as np
import torch
import torch.nn.functional as F

from .rays import get_patch_indices as _device_patch_indices
from .rays import near_far_from_sphere as _near_far
from .rays import world_rays

_WEIGHT_NAMES = ("rgb_weight", "eikonal_weight", "sdf_weight", "flow_rgb_weight", "sdf_consistency_weight",
                 "edge_aware_smoothness_weight", "smoothness_weight")  # training.py:493-497


class Trainer(object):
    def __init__(self, renderer, optimizer, motion_optimizer, cfg, device=None, patch_rng="cpu", nan_check="sync",
                 small_gemm_blas=False, **kwargs):
        """Reference: model/training.py:16-50.  small_gemm_blas=True switches torch's preferred BLAS to rocBLAS
        for the process (train.py's motion-network GEMMs run outside this class, so the switch cannot be scoped
        to its methods); the default leaves the caller's setting alone."""
        if small_gemm_blas and torch.cuda.is_available():
            torch.backends.cuda.preferred_blas_library("cublas")  # (rocBLAS on ROCm; train_step.small_gemm_blas)
        self.total_nb_images = kwargs["total_nb_images"]
        self.renderer = renderer
        self.optimizer = optimizer
        self.motion_optimizer = motion_optimizer
        self.cfg = cfg
        self.cfg_all = kwargs["cfg_all"]
        self.depth_range = kwargs["cfg_all"]["rendering"]["depth_range"]
        self.logger = kwargs.get("logger")
        self.gt_depths = kwargs.get("gt_depths")
        self.device = device
        self.n_training_points = cfg["n_training_points"]
        for name in _WEIGHT_NAMES:
            setattr(self, name, cfg[name][0])
        if "world_cam_idx" in kwargs:
            self.world_cam_idx = kwargs["world_cam_idx"]
        if "train_dataset" in kwargs:
            self.train_dataset = kwargs["train_dataset"]
        if patch_rng not in ("cpu", "device"):
            raise ValueError("patch_rng must be 'cpu' or 'device'")
        if nan_check not in ("sync", "deferred"):
            raise ValueError("nan_check must be 'sync' or 'deferred'")
        self.patch_rng = patch_rng
        self.nan_check = nan_check
        self._nonfinite = None

    # -- schedule helpers (training.py:101-124, 403-411) ---------------------
    def near_far_from_sphere(self, rays_o, rays_d):
        """training.py:101-118: the sphere mid-point is computed and then overwritten by
        the configured depth range; the result is the constant fill."""
        return _near_far(rays_o, self.depth_range)

    def get_cos_anneal_ratio(self, iter_step, anneal_end):
        if anneal_end == 0.0:
            return 1.0
        return np.min([1.0, iter_step / anneal_end])

    def anneal(self, start_weight, end_weight, anneal_start_epoch, anneal_epoches, current):
        if current <= anneal_start_epoch:
            return start_weight
        if current >= anneal_start_epoch + anneal_epoches:
            return end_weight
        return start_weight + (end_weight - start_weight) * (current - anneal_start_epoch) / anneal_epoches

    # -- data ------------------------------------------------------------------
    def get_patch_indices(self, h, w, patch_size, n_points):
        """training.py:413-436: flat ids of n_points // patch_size**2 random patches."""
        if self.patch_rng == "device":
            return _device_patch_indices(h, w, patch_size, n_points, device=self.device)
        n_patches = n_points // (patch_size ** 2)
        h_adj, w_adj = h - patch_size + 1, w - patch_size + 1
        n_patches = min(n_patches, h_adj * w_adj)
        corners = torch.randperm(h_adj * w_adj)[:n_patches]  # the reference's CPU RNG stream
        rows, cols = corners // w_adj, corners % w_adj
        offs = torch.arange(patch_size).repeat(patch_size, 1)
        offs = (offs + offs.t() * w).flatten()
        return ((rows * w + cols).unsqueeze(1) + offs.view(-1)).flatten()

    def process_data_dict(self, data):
        """training.py:377-391."""
        img = data.get("img").to(self.device)
        return img, data.get("img.camera_mat").to(self.device), data.get("img.scale_mat").to(self.device), \
            data.get("img.idx")

    def process_data_reference(self, data):
        """training.py:392-402."""
        return data.get("img.ref_imgs").to(self.device), None, data.get("img.ref_idxs")

    def process_data(self, data, world_mat, eval_mode=False, it=None, epoch=None, scheduling_start=None,
                     out_render_path=None, patch_size=1):
        """training.py:439-471 -> (img, ref_img, pixels [R,2] float, normalised pixels [R,2],
        rays_o [R,3], rays_d [R,3] (unit), |rays_d| [R,1], rgb_gt [R,3], camera_mat, scale_mat).
        Only the sampled pixels are generated (not the full arange_pixels grid)."""
        img, camera_mat, scale_mat, _ = self.process_data_dict(data)
        ref_img, _, _ = self.process_data_reference(data)
        batch_size, _, h, w = img.shape
        ray_idx = self.get_patch_indices(h, w, patch_size, self.n_training_points).to(img.device)
        rgb_gt = img.view(batch_size, 3, h * w).permute(0, 2, 1)[:, ray_idx]
        y, x = ray_idx // w, ray_idx % w
        p = torch.stack([x, y], -1).float()  # arange_pixels' (x, y) order (common.py:28-31)
        pn = torch.stack([2.0 * p[:, 0] / (w - 1) - 1.0, 2.0 * p[:, 1] / (h - 1) - 1.0], -1)
        ray_o, ray_d, rays_d_norm = self.get_world_cameraOrigin_cameraRay(pn[None], camera_mat, world_mat, scale_mat)
        return img, ref_img, p, pn, ray_o, ray_d, rays_d_norm, rgb_gt[0], camera_mat, scale_mat

    def get_world_cameraOrigin_cameraRay(self, pixels, camera_mat, world_mat, scale_mat):
        """training.py:474-487 (origin_to_world / image_points_to_world, common.py:175-215):
        o = S⁻¹W⁻¹K⁻¹[0,0,0,1], p = S⁻¹W⁻¹K⁻¹[u,v,1,1], d = (p - o) / |p - o|;
        pixels [1, R, 2], matrices [1, 4, 4] or [4, 4]."""
        # the one ray generator of this build (rays.world_rays: also SyntheticTrainer's and the
        # bench's), pinned here by trainer.npz
        s, w, c = (m.reshape(-1, 4, 4)[0] for m in (scale_mat, world_mat, camera_mat))
        return world_rays(pixels.reshape(-1, 2).to(c.dtype), c, w, s)

    # -- losses and the update ---------------------------------------------------
    def compute_loss(self, data, rendered_rgb, rgb_gt, gradient_loss, sdf_loss, flow_rgb_loss, sdf_consistency_loss,
                     edge_aware_smoothness_loss, smoothness_loss, it=None, epoch=None, scheduling_start=None,
                     out_render_path=None):
        """training.py:490-549: the weighted sum of the loss terms and the loss dict."""
        dev = rendered_rgb.device
        weights = {n: getattr(self, n) for n in _WEIGHT_NAMES}
        zero = lambda: torch.zeros((), device=dev)  # noqa: E731
        rgb_l2_mean = None
        if weights["rgb_weight"] == 0.0:
            rgb_full_loss = zero()
        else:
            rgb_full_loss = torch.sum(torch.abs(rendered_rgb - rgb_gt)) / float(rendered_rgb.shape[0])
            rgb_l2_mean = F.mse_loss(rendered_rgb, rgb_gt)
        if weights["eikonal_weight"] == 0.0:
            gradient_loss = zero()
        if weights["sdf_weight"] == 0.0:
            sdf_loss = zero()
        if weights["flow_rgb_weight"] == 0.0:
            flow_rgb_loss = zero()
        if weights["edge_aware_smoothness_weight"] == 0.0:
            edge_aware_smoothness_loss = zero()
        if weights["smoothness_weight"] == 0.0:
            smoothness_loss = zero()
        loss = weights["rgb_weight"] * rgb_full_loss + \
            weights["eikonal_weight"] * gradient_loss + \
            weights["sdf_weight"] * sdf_loss + \
            weights["flow_rgb_weight"] * flow_rgb_loss + \
            weights["sdf_consistency_weight"] * sdf_consistency_loss + \
            weights["edge_aware_smoothness_weight"] * edge_aware_smoothness_loss + \
            weights["smoothness_weight"] * smoothness_loss
        if self.nan_check == "sync":
            if torch.isnan(loss):
                assert False, "Nan loss found"
        else:
            if self._nonfinite is None or self._nonfinite.device != loss.device:
                self._nonfinite = torch.zeros((), dtype=torch.bool, device=loss.device)
            self._nonfinite |= torch.isnan(loss.detach())
        return {"loss": loss, "loss_rgb": rgb_full_loss, "loss_eikonal": gradient_loss, "l2_mean": rgb_l2_mean,
                "loss_sdf": sdf_loss, "loss_flow_rgb": flow_rgb_loss, "sdf_consistency_loss": sdf_consistency_loss,
                "edge_aware_smoothness_loss": edge_aware_smoothness_loss, "smoothness_loss": smoothness_loss}

    def check_finite(self):
        """Raise if a deferred NaN check saw a NaN loss since the last call."""
        if self._nonfinite is not None and bool(self._nonfinite.item()):
            self._nonfinite.zero_()
            raise AssertionError("Nan loss found")

    def backpropagation(self, loss_dict, train_motion_network):
        """training.py:552-558."""
        self.optimizer.zero_grad()
        if train_motion_network:
            self.motion_optimizer.zero_grad()
        loss_dict["loss"].backward()
        self.optimizer.step()
        if train_motion_network:
            self.motion_optimizer.step()
