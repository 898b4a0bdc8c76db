"""CPU oracle for cope-nerf's NeuS rendering hot path.

TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg may import this module, and only as the checker (or as the
timed CPU baseline).  The product path (cope-nerf_amd/copenerf) never imports
it and has no CPU fallback.

A functional restatement, in plain PyTorch on the CPU, of the reference
algorithm (HoangChuongNguyen/cope-nerf):
  encode            model/neus_embedder.py:6-51
  sdf_mlp           model/neus_fields.py:268-286 (SDFNetwork.forward / .sdf)
  sdf_gradient      model/neus_fields.py:291-303 (autograd, create_graph=True)
  color_mlp         model/neus_fields.py:346-374 (RenderingNetwork, mode 'idr')
  sample_pdf        model/neus_renderer.py:39-70 (det=True)
  up_sample         model/neus_renderer.py:178-224
  cat_z_vals        model/neus_renderer.py:282-298
  render_core       model/neus_renderer.py:307-450
  render            model/neus_renderer.py:453-584 (n_outside = 0, naive_render False)
  losses            model/losses.py:7-38, model/training.py:506-509, train.py:519-526
Parity pinning: tests/test_oracle_golden.py checks every function here against
fixtures produced by running the reference modules themselves
(tests/golden/make_golden.py, run in the build container only).
"""
from __future__ import annotations

import math
from dataclasses import dataclass
from typing import List, Optional

import numpy as np
import torch
import torch.nn.functional as F


# ---------------------------------------------------------------------------
# parameters
@dataclass
class SDFParams:
    W: List[torch.Tensor]   # effective weights [out, in]
    b: List[torch.Tensor]
    skip: int = 4
    multires: int = 6
    scale: float = 1.0


@dataclass
class ColorParams:
    W: List[torch.Tensor]
    b: List[torch.Tensor]
    multires_view: int = 4


def weight_norm_effective(g: torch.Tensor, v: torch.Tensor) -> torch.Tensor:
    """torch.nn.utils.weight_norm(dim=0): w = g * v / ||v|| per output row."""
    return g * (v / v.norm(dim=1, keepdim=True))


def params_from_state_dict(sd, n_layers, prefix="", requires_grad=False, **kw):
    W, b = [], []
    for l in range(n_layers):
        p = f"{prefix}lin{l}."
        if p + "weight_g" in sd:
            w = torch._weight_norm(sd[p + "weight_v"], sd[p + "weight_g"], 0)
        else:
            w = sd[p + "weight"]
        W.append(w.detach().clone().float().requires_grad_(requires_grad))
        b.append(sd[p + "bias"].detach().clone().float().requires_grad_(requires_grad))
    return W, b


def params_from_module(mod, requires_grad=False):
    n = mod.num_layers - 1
    W, b = [], []
    for l in range(n):
        lin = getattr(mod, f"lin{l}")
        w = torch._weight_norm(lin.weight_v, lin.weight_g, 0) if hasattr(lin, "weight_v") else lin.weight
        W.append(w.detach().cpu().clone().float().requires_grad_(requires_grad))
        b.append(lin.bias.detach().cpu().clone().float().requires_grad_(requires_grad))
    return W, b


# ---------------------------------------------------------------------------
# fields
def encode(x: torch.Tensor, multires: int) -> torch.Tensor:
    if multires <= 0:
        return x
    bands = 2.0 ** torch.linspace(0.0, multires - 1, multires)
    parts = [x]
    for f in bands:
        parts += [torch.sin(x * f), torch.cos(x * f)]
    return torch.cat(parts, -1)


def sdf_mlp(P: SDFParams, x: torch.Tensor) -> torch.Tensor:
    """[M, 1 + H]: sdf / scale and the feature vector."""
    e = encode(x * P.scale, P.multires)
    h = e
    last = len(P.W) - 1
    for l, (W, b) in enumerate(zip(P.W, P.b)):
        if l == P.skip:
            h = torch.cat([h, e], 1) / np.sqrt(2)
        h = F.linear(h, W, b)
        if l < last:
            h = F.softplus(h, beta=100)
    return torch.cat([h[:, :1] / P.scale, h[:, 1:]], -1)


def sdf_gradient(P: SDFParams, x: torch.Tensor) -> torch.Tensor:
    """∂sdf/∂x [M, 4] with create_graph=True (the input is detached, as in the reference)."""
    with torch.enable_grad():
        x = x.detach().requires_grad_(True)
        y = sdf_mlp(P, x)[:, :1]
        (g,) = torch.autograd.grad(y, x, torch.ones_like(y), create_graph=True, retain_graph=True)
    return g


def color_mlp(Pc: ColorParams, pts_time, gradients, dirs, feature):
    h = torch.cat([pts_time, encode(dirs, Pc.multires_view), gradients, feature], -1)
    last = len(Pc.W) - 1
    for l, (W, b) in enumerate(zip(Pc.W, Pc.b)):
        h = F.linear(h, W, b)
        if l < last:
            h = F.relu(h)
    return torch.sigmoid(h)


# ---------------------------------------------------------------------------
# sampling
def exclusive_cumprod(a: torch.Tensor) -> torch.Tensor:
    """T_i = prod_{j<i} (1 - a_j + 1e-7)."""
    ones = torch.ones_like(a[:, :1])
    return torch.cumprod(torch.cat([ones, 1.0 - a + 1e-7], -1), -1)[:, :-1]


def sample_pdf(bins, weights, n_samples):
    w = weights + 1e-5
    pdf = w / torch.sum(w, -1, keepdim=True)
    cdf = torch.cat([torch.zeros_like(pdf[..., :1]), torch.cumsum(pdf, -1)], -1)
    u = torch.linspace(0.5 / n_samples, 1.0 - 0.5 / n_samples, steps=n_samples)
    u = u.expand(list(cdf.shape[:-1]) + [n_samples]).contiguous()
    idx = torch.searchsorted(cdf, u, right=True)
    lo = (idx - 1).clamp(min=0)
    hi = idx.clamp(max=cdf.shape[-1] - 1)
    c_lo, c_hi = torch.gather(cdf, 1, lo), torch.gather(cdf, 1, hi)
    b_lo, b_hi = torch.gather(bins, 1, lo), torch.gather(bins, 1, hi)
    den = c_hi - c_lo
    den = torch.where(den < 1e-5, torch.ones_like(den), den)
    return b_lo + (u - c_lo) / den * (b_hi - b_lo)


def up_sample(z, sdf, n_importance, inv_s):
    """NeuS up-sampling with a fixed inv_s (the reference's inside_sphere mask is all ones)."""
    R = z.shape[0]
    s0, s1 = sdf[:, :-1], sdf[:, 1:]
    z0, z1 = z[:, :-1], z[:, 1:]
    mid = (s0 + s1) * 0.5
    cosv = (s1 - s0) / (z1 - z0 + 1e-5)
    prev = torch.cat([torch.zeros(R, 1), cosv[:, :-1]], -1)
    cosv = torch.min(torch.stack([prev, cosv], -1), -1)[0].clip(-1e3, 0.0)
    dist = z1 - z0
    pe = mid - cosv * dist * 0.5
    ne = mid + cosv * dist * 0.5
    pc, nc = torch.sigmoid(pe * inv_s), torch.sigmoid(ne * inv_s)
    alpha = (pc - nc + 1e-5) / (pc + 1e-5)
    w = alpha * exclusive_cumprod(alpha)
    return sample_pdf(z, w, n_importance).detach()


def cat_z_vals(z, new_z, sdf, new_sdf=None):
    zc, idx = torch.sort(torch.cat([z, new_z], -1), -1)
    if new_sdf is None:
        return zc, None
    return zc, torch.gather(torch.cat([sdf, new_sdf], -1), 1, idx)


def points(rays_o, rays_d, z, t):
    p = (rays_o[:, None, :] + rays_d[:, None, :] * z[..., None]).reshape(-1, 3)
    return torch.cat([p, t.reshape(1, 1).expand(p.shape[0], 1)], -1)


def coarse_z(near, far, n, t_rand=None):
    lin = torch.linspace(0.0, 1.0, n)
    z = near * (1.0 - lin[None, :]) + far * lin[None, :]
    if t_rand is not None:
        mids = 0.5 * (z[..., 1:] + z[..., :-1])
        upper = torch.cat([mids, z[..., -1:]], -1)
        lower = torch.cat([z[..., :1], mids], -1)
        z = lower + (upper - lower) * t_rand
    return z


def hierarchical_z(P, rays_o, rays_d, t, near, far, n_samples, n_importance, up_steps, t_rand):
    with torch.no_grad():
        R = rays_o.shape[0]
        z = coarse_z(near, far, n_samples, t_rand)
        if n_importance <= 0:
            return z
        sdf = sdf_mlp(P, points(rays_o, rays_d, z, t))[:, :1].reshape(R, n_samples)
        k = n_importance // up_steps
        for i in range(up_steps):
            nz = up_sample(z, sdf, k, 64 * 2 ** i)
            last = (i + 1) == up_steps
            nsdf = None if last else sdf_mlp(P, points(rays_o, rays_d, nz, t))[:, :1].reshape(R, k)
            z, sdf = cat_z_vals(z, nz, sdf, nsdf)
        return z


# ---------------------------------------------------------------------------
# compositing
def render_core(P, Pc, variance, rays_o, rays_d, rays_d_norm, t, z, sample_dist, car, eval_mode=False):
    R, S = z.shape
    dists = torch.cat([z[..., 1:] - z[..., :-1], sample_dist.reshape(1, 1).expand(R, 1)], -1)
    mid = z + dists * 0.5
    pts_time = points(rays_o, rays_d, mid, t)
    dirs = rays_d[:, None, :].expand(R, S, 3).reshape(-1, 3)
    out = sdf_mlp(P, pts_time)
    sdf, feat = out[:, :1], out[:, 1:]
    g = sdf_gradient(P, pts_time)
    normals, flows = g[:, :3], g[:, 3:]
    rgb = color_mlp(Pc, pts_time, g, dirs, feat).reshape(R, S, 3)
    inv_s = (torch.ones(1, 1) * torch.exp(variance * 10.0)).clip(1e-3, 1e3)
    color, depth, w, pc = composite(z, dists, sdf, normals, rgb, dirs, inv_s, car)
    weighted_z = depth.detach().clone()
    if eval_mode:
        depth = depth / rays_d_norm
    return {"color_fine": color, "depth_pred": depth, "weighted_z_vals": weighted_z, "sdf": sdf,
            "normals": normals.reshape(R, S, 3), "sdf_flows": flows.reshape(R, S, 1), "weights": w,
            "cdf_fine": pc.reshape(R, S), "sampled_points": pts_time[:, :3].reshape(R, S, 3),
            "s_val": (1.0 / inv_s).expand(R * S, 1).reshape(R, S).mean(-1, keepdim=True), "z_vals": z,
            "rgb": rgb}


def composite(z, dists, sdf, normals, rgb, dirs, inv_s, car):
    """SDF -> alpha (NeuS eq. 13) -> exclusive-cumprod weights -> colour / depth
    (neus_renderer.py:365-417).  rgb [R,S,3]; sdf, normals, dirs per sample [M,*]."""
    R, S = z.shape
    tc = (dirs * normals).sum(-1, keepdim=True)
    ic = -(F.relu(-tc * 0.5 + 0.5) * (1.0 - car) + F.relu(-tc) * car)
    en = sdf + ic * dists.reshape(-1, 1) * 0.5
    ep = sdf - ic * dists.reshape(-1, 1) * 0.5
    pc, nc = torch.sigmoid(ep * inv_s), torch.sigmoid(en * inv_s)
    alpha = ((pc - nc + 1e-5) / (pc + 1e-5)).reshape(R, S).clip(0.0, 1.0)
    w = alpha * exclusive_cumprod(alpha)
    color = (rgb * w[:, :, None]).sum(1)
    depth = (z * w).sum(1).unsqueeze(-1)
    return color, depth, w, pc


def render(P, Pc, variance, rays_o, rays_d, rays_d_norm, t, near, far, *, n_samples=64, n_importance=64,
           up_steps=4, car=0.0, t_rand=None, eval_mode=False):
    z = hierarchical_z(P, rays_o, rays_d, t, near, far, n_samples, n_importance, up_steps,
                       None if eval_mode else t_rand)
    sample_dist = (far[0, 0] - near[0, 0]) / n_samples
    return render_core(P, Pc, variance, rays_o, rays_d, rays_d_norm, t, z, sample_dist, car, eval_mode)


# ---------------------------------------------------------------------------
# losses
def smoothness(d):
    l1 = lambda x: torch.mean(torch.abs(x))  # noqa: E731
    return (l1(d[:, :, :-1] - d[:, :, 1:]) + l1(d[:, :-1, :] - d[:, 1:, :]) +
            l1(d[:, :-1, :-1] - d[:, 1:, 1:]) + l1(d[:, 1:, :-1] - d[:, :-1, 1:])) / 4


def edge_smoothness(d, img, gamma=0.1):
    l1 = lambda x: torch.mean(torch.abs(x))  # noqa: E731
    bw = lambda x: torch.exp(-torch.abs(x).sum(-1) / gamma).unsqueeze(-1)  # noqa: E731
    return (l1(bw(img[:, :, :-1] - img[:, :, 1:]) * (d[:, :, :-1] - d[:, :, 1:])) +
            l1(bw(img[:, :-1, :] - img[:, 1:, :]) * (d[:, :-1, :] - d[:, 1:, :])) +
            l1(bw(img[:, :-1, :-1] - img[:, 1:, 1:]) * (d[:, :-1, :-1] - d[:, 1:, 1:])) +
            l1(bw(img[:, 1:, :-1] - img[:, :-1, 1:]) * (d[:, 1:, :-1] - d[:, :-1, 1:]))) / 4


def train_loss(out, rgb_gt, *, patch=4, w_rgb=1.0, w_eik=0.1, w_edge=1.0, w_smooth=1e-4, s=0):
    """L1 rgb + eikonal + edge-aware / plain depth smoothness on 4x4 patches
    (training.py:506-533, train.py:519-526); the stage-1 motion terms are zero here."""
    rgb = out["color_fine"]
    loss = w_rgb * torch.sum(torch.abs(rgb - rgb_gt)) / float(rgb.shape[0])
    loss = loss + w_eik * torch.mean((torch.linalg.norm(out["normals"].reshape(-1, 3), ord=2, dim=-1) - 1.0) ** 2)
    if patch > 1 and (w_edge or w_smooth):
        d = out["depth_pred"].view(-1, patch, patch, 1)
        g = rgb_gt.view(-1, patch, patch, 3)
        loss = loss + w_edge * (1 / (2 ** s)) * edge_smoothness(d, g) + w_smooth * (1 / (2 ** s)) * smoothness(d)
    return loss


# ---------------------------------------------------------------------------
# stage-1 scene-flow loss (train.py:467-477)
def scene_flow_loss(pts, normals, sdf_flows, weights, omega, vel):
    """sum |(ω × p + v) · n + ∂sdf/∂t| · w.detach() / (sum w + 1e-10) over all samples."""
    pts = pts.reshape(-1, 3)
    n = normals.reshape(-1, 3)
    w = weights.reshape(-1).detach()
    sf = torch.cross(omega.reshape(1, 3).repeat(pts.shape[0], 1), pts, dim=-1) + vel.reshape(1, 3).repeat(pts.shape[0], 1)
    lhs = torch.sum(sf * n, dim=-1)
    return torch.sum(torch.abs(lhs + sdf_flows.reshape(-1)) * w) / (torch.sum(w) + 1e-10)


# ---------------------------------------------------------------------------
# stage 1: motion network poses, flow-RGB and SDF consistency (train.py:467-517)
def euler_xyz(angles):
    """pytorch3d euler_angles_to_matrix(..., 'XYZ') (utils_poses/pose_pytorch3d.py)."""
    def axis(a, ang):
        c, s = torch.cos(ang), torch.sin(ang)
        o, z = torch.ones_like(ang), torch.zeros_like(ang)
        rows = {"X": (o, z, z, z, c, -s, z, s, c), "Y": (c, z, s, z, o, z, -s, z, c),
                "Z": (c, -s, z, s, c, z, z, z, o)}[a]
        return torch.stack(rows, -1).reshape(ang.shape + (3, 3))
    x, y, zz = torch.unbind(angles, -1)
    return (axis("X", x) @ axis("Y", y)) @ axis("Z", zz)


def consecutive_relative_pose(motion, cam, n_images, nb_sample_timestep):
    """neus_fields.py:142-161, one interval cam -> cam + 1 (sequential Euler steps)."""
    ref = cam + 1.0
    t0 = cam / (n_images - 1) * 2 - 1
    t1 = ref / (n_images - 1) * 2 - 1
    n = int(nb_sample_timestep * (ref - cam))
    steps = torch.linspace(t0, t1, n + 1)[:-1]
    dt = steps[1] - steps[0]
    R = torch.eye(3)
    T = torch.zeros(3)
    omega, vel = motion(steps.view(-1, 1))
    R_list = euler_xyz(omega * dt)
    V_list = vel * dt
    for k in range(len(steps)):
        T = R_list[k] @ T.view(3, 1) + V_list[k].view(3, 1)
        R = R @ R_list[k]
    pose = torch.eye(4)
    pose[:3, :3] = R
    pose[:3, -1] = T.view(1, 3)
    return dt, pose


def relative_camera_pose(motion, lo, hi, n_images, nb_sample_timestep):
    """neus_fields.py:163-168 + compute_w2c_mappings 174-186: the w2c chain lo -> hi."""
    w2c = [torch.eye(4)]
    for cam in range(int(lo), int(hi)):
        _, p = consecutive_relative_pose(motion, cam, n_images, nb_sample_timestep)
        w2c.append(p @ w2c[-1])
    return torch.stack(w2c)


def stage1_losses(out, motion, sdf_fn, *, image_idx, n_images, world_cam_idx, nb_sample_timestep, rgb_gt,
                  sampled_pixel, normalized_pixel, camera_mats, ref_images, scale_mat, img_hw,
                  ref_intervals=(1, 2, 3), consistency_pose_grad=False):
    """(sdf_loss, flow_rgb_loss, sdf_consistency_loss) of one stage-1 iteration,
    train.py:467-517 (query_in_canonical_space False).  motion(t [N,1]) -> (ω, v);
    sdf_fn(x [M,4]) -> sdf [M,1]; camera_mats [n_images, 4, 4]; ref_images
    [n_images, 3, H, W]; ref frames image_idx + ref_intervals (dataset.py:231-250);
    consistency_pose_grad: cfg['training']['sdf_consistency_enable_pose_grad'] (train.py:498)."""
    R = rgb_gt.shape[0]
    pts = out["sampled_points"].reshape(-1, 3)
    normals = out["normals"].reshape(-1, 3)
    sdf_flows = out["sdf_flows"].reshape(-1)
    weights = out["weights"].reshape(-1)
    time_step = image_idx / (n_images - 1) * 2 - 1
    world_time_step = world_cam_idx / (n_images - 1) * 2 - 1
    omega, vel = motion(torch.tensor([time_step]).float().view(-1, 1))
    omega = omega.repeat(pts.shape[0], 1)
    vel = vel.repeat(pts.shape[0], 1)
    scene_flow = torch.cross(omega, pts, dim=-1) + vel
    lhs = torch.sum(scene_flow * normals, dim=-1)
    sdf_loss = torch.sum(torch.abs(lhs + sdf_flows) * weights.detach()) / (torch.sum(weights.detach()) + 1e-10)

    ref_idx = [image_idx + k for k in ref_intervals]
    next_t = [(r / (n_images - 1) * 2 - 1) for r in ref_idx]
    nb_valid = len([t for t in next_t if t <= 1.0])
    flow_rgb = torch.tensor(0.0)
    consistency = torch.tensor(0.0)
    w2c = relative_camera_pose(motion, image_idx, ref_idx[nb_valid - 1], n_images, nb_sample_timestep)
    w2c = w2c[[r - image_idx for r in ref_idx][:nb_valid]]
    flows = []
    for t in range(len(w2c)):
        ref_K = camera_mats[ref_idx[t]][None]
        pts_map = (w2c[t, :3, :3] @ pts.T + w2c[t, :3, [-1]]).T
        wp = torch.sum(weights.view(R, -1, 1) * pts_map.view(R, -1, 3), dim=1)
        pix = (scale_mat[0, :3, :3] @ ref_K[0, :3, :3] @ wp.T).T
        pix = pix[:, :2] / pix[:, [-1]]
        f = pix - normalized_pixel
        f = torch.stack([f[:, 0] * (img_hw[1] / 2), f[:, 1] * (img_hw[0] / 2)], -1)
        flows.append(f)
    if image_idx != world_cam_idx:
        with torch.set_grad_enabled(consistency_pose_grad):  # train.py:498 (default.yaml:62: False)
            lo, hi = min(world_cam_idx, image_idx), max(world_cam_idx, image_idx)
            c2c = relative_camera_pose(motion, lo, hi, n_images, nb_sample_timestep)[-1]
            cw2 = torch.inverse(c2c) if world_cam_idx <= image_idx else c2c
            pts_world = (cw2[:3, :3] @ pts.T + cw2[:3, [-1]]).T
        sdf_w = sdf_fn(torch.cat([pts_world, torch.ones_like(pts_world[:, [0]]) * world_time_step], dim=1))
        consistency = torch.mean(torch.abs(sdf_w - out["sdf"].reshape(-1, 1)))
    for t in range(nb_valid):
        ref_img = ref_images[ref_idx[t]][None]
        corr = sampled_pixel + flows[t]
        with torch.no_grad():
            valid = ((corr >= 0) & (corr < torch.tensor([ref_img.shape[3], ref_img.shape[2]]).float())).all(
                dim=1, keepdim=True)
        H, W = ref_img.shape[2], ref_img.shape[3]
        gx = corr[:, 0] / ((W - 1) / 2) - 1
        gy = corr[:, 1] / ((H - 1) / 2) - 1
        grid = torch.stack([gx, gy], -1).view(1, R, 1, 2)
        warped = F.grid_sample(ref_img, grid, mode="bilinear", padding_mode="border", align_corners=True)
        warped = warped.squeeze().T
        flow_rgb = flow_rgb + torch.sum(torch.abs(warped - rgb_gt) * valid) / (torch.sum(valid) + 1e-10)
    flow_rgb = flow_rgb / 3.0
    return sdf_loss, flow_rgb, consistency
