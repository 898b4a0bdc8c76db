"""Full-image inference rendering.

Mirrors the per-chunk loop of Trainer.render_visdata / render_eval
(model/training.py:157-300):
* arange_pixels (common.py:12-39);
* rays per chunk, under the given world matrix;
* NeuSRenderer(eval=True) with no autograd;
* rgb, depth (/‖d‖), weighted z, the weight-averaged normal, the depth of the
  highest-weight sample, and (given a motion network) the forward flow of the
  weight-averaged scene-flow-advected point (training.py:262-280).

The reference renders 1024 rays per chunk and copies each result to the host.
Here a chunk is a free parameter (default 65,536 rays, 8.4 M samples), every
output stays on the device, and the whole image comes back as [h, w, ·]
tensors.  The renderer runs forward-only: no buffers are kept for a backward,
and the ∇ₓSDF pass runs only because normals and α need it.
"""
from __future__ import annotations

import torch

from .rays import inv4x4, near_far_from_sphere, world_rays


def arange_pixels(h, w, device="cpu"):
    """(pixel [h*w, 2] long (x, y), normalised [h*w, 2] in [-1, 1]), row-major over
    (y, x) like common.py:12-39."""
    yy, xx = torch.meshgrid(torch.arange(h, device=device), torch.arange(w, device=device), indexing="ij")
    loc = torch.stack([xx, yy], -1).reshape(-1, 2)
    sc = loc.float()
    sc = torch.stack([2.0 * sc[:, 0] / (w - 1) - 1.0, 2.0 * sc[:, 1] / (h - 1) - 1.0], -1)
    return loc, sc


@torch.no_grad()
def render_image(renderer, camera_mat, world_mat, scale_mat, resolution, time_step, *, depth_range=(0.01, 5.0),
                 cos_anneal_ratio=1.0, it=0, chunk=65536, motion=None, next_time_step=None, nb_sample_timestep=10):
    """Render a full image; returns a dict of device tensors shaped [h, w, ·]."""
    h, w = resolution
    dev = camera_mat.device
    _, pixels = arange_pixels(h, w, device=dev)
    t = time_step.reshape(1).to(dev).float()
    identity = torch.equal(world_mat, torch.eye(4, device=dev))
    flows = motion is not None and next_time_step is not None
    if flows:  # velocities along [t, t_next) (training.py:197-201)
        steps = torch.linspace(float(t), float(next_time_step), nb_sample_timestep + 1, device=dev)[:-1]
        omegas, vels = motion(steps.view(-1, 1))
        dt = (float(next_time_step) - float(t)) / nb_sample_timestep
    acc = {k: [] for k in ("rgb", "depth", "weighted_z", "normal", "depth_max_w", "flow")}
    for i in range(0, pixels.shape[0], chunk):
        pix = pixels[i:i + chunk]
        rays_o, rays_d, norm = world_rays(pix, camera_mat, world_mat, scale_mat)
        near, far = near_far_from_sphere(rays_o, depth_range)
        out = renderer(rays_o, rays_d, norm, t, near, far, cos_anneal_ratio=cos_anneal_ratio, it=it, eval=True)
        wts = out["weights"]
        pts = out["sampled_points"]
        acc["rgb"].append(out["color_fine"])
        acc["depth"].append(out["depth_pred"])
        acc["weighted_z"].append(out["weighted_z_vals"])
        normal = (out["normals"] * wts[:, :, None]).sum(1)
        amax = wts.argmax(1)
        p_max = pts[torch.arange(pts.shape[0], device=dev), amax]
        if identity:
            depth_max = -p_max[:, 2]
        else:
            depth_max = -(p_max @ world_mat[:3, :3].T + world_mat[:3, 3])[:, 2]
            normal = normal @ world_mat[:3, :3].T
        acc["normal"].append(normal)
        acc["depth_max_w"].append(depth_max)
        if flows:
            p = pts.reshape(-1, 3).clone()
            for k in range(nb_sample_timestep):
                p = p + dt * (torch.cross(omegas[k].expand_as(p), p, dim=-1) + vels[k])
            p = (wts[:, :, None] * p.view(wts.shape[0], -1, 3)).sum(1)
            proj = (scale_mat[:3, :3] @ camera_mat[:3, :3] @ p.T).T
            acc["flow"].append(proj[:, :2] / proj[:, 2:] - pix)
    res = {
        "rgb": torch.cat(acc["rgb"]).view(h, w, 3),
        "depth": torch.cat(acc["depth"]).view(h, w),
        "weighted_z": torch.cat(acc["weighted_z"]).view(h, w),
        "normal": torch.cat(acc["normal"]).view(h, w, 3),
        "depth_highest_weight": torch.cat(acc["depth_max_w"]).view(h, w),
    }
    if flows:
        f = torch.cat(acc["flow"]).view(h, w, 2).clone()
        f[..., 0] *= w / 2
        f[..., 1] *= h / 2
        res["flow"] = f
    return res


def relative_world_mat(motion, query_cam_idx, image_idx, total_nb_images, nb_sample_timestep):
    """world_mat for rendering image `image_idx` in the frame of `query_cam_idx` from
    the motion network's integrated relative pose (training.py:171-179)."""
    lo, hi = min(query_cam_idx, image_idx), max(query_cam_idx, image_idx)
    _, rel = motion.compute_relative_camera_pose(lo, hi, total_nb_images, nb_sample_timestep)
    c2c = motion.compute_w2c_mappings(rel)[-1]
    return c2c if query_cam_idx <= image_idx else inv4x4(c2c)
