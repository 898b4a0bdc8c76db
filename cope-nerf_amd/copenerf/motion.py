"""Stage-1 motion model and losses.

  MotionNetwork                   model/neus_fields.py:79-190
  euler_angles_to_matrix (XYZ)    utils_poses/pose_pytorch3d.py (pytorch3d convention)
  scene_flow_loss                 train.py:467-477 (sdf_loss)
  project_flow / warp_pixel       train.py:478-496, 235-244 (flow-RGB warp)
  sdf_consistency_points          train.py:497-505

The motion network maps a time step to an angular and a linear velocity.  It is
evaluated on a handful of time steps per training step (one query time, plus
nb_sample_timestep per frame interval for relative poses).  That is a few
hundred rows through a 256-wide MLP, so it stays a torch module: a HIP launch
would cost more than the math.  Everything it feeds runs on the renderer's
device outputs: sampled_points, normals, sdf_flows and weights.  The scene-flow
loss and the SDF re-query at world points (sdf_network.sdf, the HIP SDF
forward and backward) then take the renderer's gradients back into the HIP
path.  Unlike the reference, nothing here calls .cuda(): tensors follow the
parameters' device.
"""
from __future__ import annotations

import numpy as np
import torch
import torch.nn as nn

from .embedder import get_embedder


def _axis_rotation(axis: str, angle: torch.Tensor) -> torch.Tensor:
    """Right-handed rotation about one axis by `angle` (broadcast over the batch)."""
    c, s = torch.cos(angle), torch.sin(angle)
    one, zero = torch.ones_like(angle), torch.zeros_like(angle)
    if axis == "X":
        rows = (one, zero, zero, zero, c, -s, zero, s, c)
    elif axis == "Y":
        rows = (c, zero, s, zero, one, zero, -s, zero, c)
    elif axis == "Z":
        rows = (c, -s, zero, s, c, zero, zero, zero, one)
    else:
        raise ValueError(f"axis {axis}")
    return torch.stack(rows, -1).reshape(angle.shape + (3, 3))


def euler_angles_to_matrix(euler_angles: torch.Tensor, convention: str = "XYZ") -> torch.Tensor:
    """[..., 3] Euler angles -> [..., 3, 3]: R = R_a(e0) R_b(e1) R_c(e2) for convention 'abc'
    (the pytorch3d definition the reference uses, utils_poses/pose_pytorch3d.py)."""
    if len(convention) != 3:
        raise ValueError("convention must have 3 letters")
    mats = [_axis_rotation(a, e) for a, e in zip(convention, torch.unbind(euler_angles, -1))]
    return (mats[0] @ mats[1]) @ mats[2]


class MotionNetwork(nn.Module):
    """Reference: model/neus_fields.py:79-190 (same constructor, parameter names,
    initialisation order and forward).  forward(t [N,1]) -> (angular velocity
    [N,3], velocity [N,3])."""

    def __init__(self, d_in, d_out, d_hidden, n_layers, skip_in=(4,), multires=0, bias=0.5, scale=1,
                 geometric_init=True, weight_norm=True, inside_outside=False):
        super().__init__()
        dims = [d_in] + [d_hidden] * n_layers + [d_out]
        self.embed_fn_fine = None
        self.scale = scale
        if multires > 0:
            self.embed_fn_fine, dims[0] = get_embedder(multires, input_dims=d_in)
        self.num_layers = len(dims)
        self.skip_in = skip_in
        for l in range(self.num_layers - 1):
            out_dim = dims[l + 1] - dims[0] if (l + 1) in skip_in else dims[l + 1]
            lin = nn.Linear(dims[l], out_dim)
            if geometric_init:
                if l == self.num_layers - 2:
                    m = np.sqrt(np.pi) / np.sqrt(dims[l])
                    torch.nn.init.normal_(lin.weight, mean=-m if inside_outside else m, std=0.0001)
                    torch.nn.init.constant_(lin.bias, bias if inside_outside else -bias)
                elif multires > 0 and l == 0:
                    torch.nn.init.constant_(lin.bias, 0.0)
                    torch.nn.init.constant_(lin.weight[:, 3:], 0.0)
                    torch.nn.init.normal_(lin.weight[:, :3], 0.0, np.sqrt(2) / np.sqrt(out_dim))
                elif multires > 0 and l in skip_in:
                    torch.nn.init.constant_(lin.bias, 0.0)
                    torch.nn.init.normal_(lin.weight, 0.0, np.sqrt(2) / np.sqrt(out_dim))
                    torch.nn.init.constant_(lin.weight[:, -(dims[0] - 3):], 0.0)
                else:
                    torch.nn.init.constant_(lin.bias, 0.0)
                    torch.nn.init.normal_(lin.weight, 0.0, np.sqrt(2) / np.sqrt(out_dim))
            if weight_norm:
                lin = nn.utils.weight_norm(lin)
            setattr(self, f"lin{l}", lin)
        self.activation = nn.LeakyReLU(0.2)

    def _device(self):
        return self.lin0.bias.device

    def forward(self, inputs):
        if self.embed_fn_fine is not None:
            inputs = self.embed_fn_fine(inputs)
        x = inputs
        for l in range(self.num_layers - 1):
            if l in self.skip_in:
                x = torch.cat([x, inputs], 1) / np.sqrt(2)
            x = getattr(self, f"lin{l}")(x)
            if l < self.num_layers - 2:
                x = self.activation(x)
        x = x * self.scale
        return x[:, :3], x[:, 3:]

    def compute_consecutive_relative_pose(self, target_cam_idx, total_nb_images, nb_sample_timestep):
        """Integrate the velocities over [t_i, t_{i+1}) in nb_sample_timestep steps:
        T <- R_k T + V_k, R <- R R_k with R_k = Euler_XYZ(ω_k Δt), V_k = v_k Δt
        (neus_fields.py:146-165).  Returns (Δt, 4x4 relative pose)."""
        dev = self._device()
        ref_cam_idx = target_cam_idx + 1.0
        t0 = target_cam_idx / (total_nb_images - 1) * 2 - 1
        t1 = ref_cam_idx / (total_nb_images - 1) * 2 - 1
        n = int(nb_sample_timestep * (ref_cam_idx - target_cam_idx))
        steps = torch.linspace(float(t0), float(t1), n + 1)[:-1]
        dt = steps[1] - steps[0]
        omega, vel = self.forward(steps.view(-1, 1).to(dev))
        dt_d = dt.to(dev)
        R_list = euler_angles_to_matrix(omega * dt_d, "XYZ")
        V_list = vel * dt_d
        R = torch.eye(3, device=dev)
        T = torch.zeros(3, device=dev)
        for k in range(len(steps)):
            T = R_list[k] @ T.view(3, 1) + V_list[k].view(3, 1)
            R = R @ R_list[k]
        pose = torch.eye(4, device=dev)
        pose[:3, :3] = R
        pose[:3, -1] = T.view(1, 3)
        return dt, pose

    def compute_relative_camera_pose(self, target_cam_idx, final_ref_cam_idx, total_nb_images, nb_sample_timestep):
        poses = []
        dt = None
        for cam in range(int(target_cam_idx), int(final_ref_cam_idx)):
            dt, p = self.compute_consecutive_relative_pose(cam, total_nb_images, nb_sample_timestep)
            poses.append(p)
        return dt, poses

    def compute_w2c_mappings(self, relative_camera_pose):
        """w2c[0] = I, w2c[i+1] = rel[i] @ w2c[i] (neus_fields.py:174-186)."""
        w2c = [torch.eye(4, device=self._device())]
        for rel in relative_camera_pose:
            w2c.append(rel @ w2c[-1])
        return torch.stack(w2c)


def scene_flow_loss(pts, normals, sdf_flows, weights, angular_velocity, velocity):
    """SDF scene-flow consistency (train.py:467-477): the scene flow ω × p + v of
    every sample must satisfy the level-set equation ∇sdf · flow + ∂sdf/∂t = 0;
    L1, weighted by the detached render weights over their global sum."""
    pts = pts.reshape(-1, 3)
    normals = normals.reshape(-1, 3)
    sdf_flows = sdf_flows.reshape(-1)
    w = weights.reshape(-1).detach()
    omega = angular_velocity.reshape(1, 3).expand(pts.shape[0], 3)
    vel = velocity.reshape(1, 3).expand(pts.shape[0], 3)
    flow = torch.cross(omega, pts, dim=-1) + vel
    lhs = torch.sum(flow * normals, dim=-1)
    return torch.sum(torch.abs(lhs + sdf_flows) * w) / (torch.sum(w) + 1e-10)


def project_flow(pts, weights, w2c, ref_camera_mat, scale_mat, normalized_pixels, img_hw):
    """Forward optical flow to a reference frame (train.py:478-496): the
    weight-averaged sample point of each ray, mapped by the relative pose w2c
    [4,4] and projected with the reference camera; returns pixel offsets [R,2]."""
    R = normalized_pixels.shape[0]
    pts_map = (w2c[:3, :3] @ pts.reshape(-1, 3).T + w2c[:3, [-1]]).T
    wp = torch.sum(weights.reshape(R, -1, 1) * pts_map.reshape(R, -1, 3), dim=1)
    pix = (scale_mat[0, :3, :3] @ ref_camera_mat[0, :3, :3] @ wp.T).T
    pix = pix[:, :2] / pix[:, [-1]]
    flow = pix - normalized_pixels
    h, w = img_hw
    return torch.stack([flow[:, 0] * (w / 2), flow[:, 1] * (h / 2)], -1)


def warp_pixel(src_frame, uv, normalize_pix=True):
    """Bilinear warp with border padding, align_corners=True (train.py:235-244)."""
    _, _, height, width = src_frame.shape
    wx, wy = uv[:, 0], uv[:, 1]
    if normalize_pix:
        wx = wx / ((width - 1) / 2) - 1
        wy = wy / ((height - 1) / 2) - 1
    coord = torch.stack([wx, wy], dim=-1)
    return torch.nn.functional.grid_sample(src_frame, coord, mode="bilinear", padding_mode="border",
                                           align_corners=True)


def flow_rgb_loss(flow_fw, sampled_pixel, ref_img, rgb_gt):
    """Photometric loss of the reference frame warped by the predicted flow
    (train.py:506-515), masked to correspondences inside the image."""
    corr = sampled_pixel + flow_fw
    with torch.no_grad():
        lim = torch.tensor([ref_img.shape[3], ref_img.shape[2]], dtype=torch.float32, device=corr.device)
        valid = ((corr >= 0) & (corr < lim)).all(dim=1, keepdim=True)
    warped = warp_pixel(ref_img, corr.T.unsqueeze(0).unsqueeze(-1)).squeeze().T
    return torch.sum(torch.abs(warped - rgb_gt) * valid) / (torch.sum(valid) + 1e-10)


def world_points(pts, cw2):
    """Sample points mapped into the world (canonical) frame for the SDF
    consistency re-query (train.py:497-505)."""
    return (cw2[:3, :3] @ pts.reshape(-1, 3).T + cw2[:3, [-1]]).T
