"""Ray generation under SE(3) poses.

Restates, on the device and without host syncs:
  get_patch_indices                 model/training.py:413-436
  arange_pixels (only the R needed) model/common.py:12-39
  get_world_cameraOrigin_cameraRay  model/training.py:474-487 with
  origin_to_world / image_points_to_world / transform_to_world  model/common.py:175-215
  near_far_from_sphere, get_cos_anneal_ratio  model/training.py:101-124
  vec2skew / Exp / make_c2w / convert3x4_4x4  model/common.py:255-308
  PoseRetriever                     model/poses_retriever.py:6-32
This is 4x4 matrix algebra plus O(R) elementwise work (microseconds), kept in
torch device ops; the per-sample work starts at the sampler (cn_coarse_z).
"""
from __future__ import annotations

import numpy as np
import torch
import torch.nn as nn


def get_patch_indices(h, w, patch_size, n_points, generator=None, device="cpu"):
    """Flat pixel ids of n_points // patch_size**2 random patch_size x patch_size patches."""
    n_patches = n_points // (patch_size ** 2)
    h_adj, w_adj = h - patch_size + 1, w - patch_size + 1
    n_patches = min(n_patches, h_adj * w_adj)
    if torch.device(device).type == "cuda":
        # the first n_patches of a keyed pseudo-random permutation of the corners, as
        # randperm(...)[:n_patches] (training.py:422), in one launch (cn_patch_indices)
        from . import ops
        key = torch.randint(-2 ** 31, 2 ** 31 - 1, (4,), generator=generator, device=device, dtype=torch.int32)
        return ops.patch_indices(h, w, patch_size, n_patches, key)
    # CPU tensors: a uniformly random n_patches-subset by the top-k of random keys
    keys = torch.rand(h_adj * w_adj, generator=generator, device=device)
    corners = torch.topk(keys, n_patches, sorted=False).indices
    rows, cols = corners // w_adj, corners % w_adj
    offs = torch.arange(patch_size, device=device).repeat(patch_size, 1)
    offs = (offs + offs.t() * w).flatten()
    return ((rows * w + cols).unsqueeze(1) + offs.view(-1)).flatten()


def pixels_from_indices(idx, h, w):
    """(pixel [R,2] long (x, y), normalised [R,2] float in [-1, 1]) of flat ids -- the
    rows of arange_pixels((h, w)) the reference gathers, without building the grid."""
    y, x = idx // w, idx % w
    p = torch.stack([x, y], -1)
    pn = p.float()
    pn = torch.stack([2.0 * pn[:, 0] / (w - 1) - 1.0, 2.0 * pn[:, 1] / (h - 1) - 1.0], -1)
    return p, pn


def intrinsics_ndc(fx, fy, w, h, device="cpu"):
    """K of the reference loaders (dataloading/dataset.py:108-111)."""
    return torch.tensor([[2 * fx / w, 0, 0, 0], [0, -2 * fy / h, 0, 0], [0, 0, -1, 0], [0, 0, 0, 1]],
                        dtype=torch.float32, device=device)


def _cofactor_tables():
    """Flat indices [16, 6, 3] and signs [16, 6] of the six permutation terms of
    every 3x3 minor's determinant, (-1)^(i+j) folded in: cofactor C_ij =
    sum_p sign[ij, p] * prod_k a[idx[ij, p, k]]."""
    perms = (((0, 1, 2), 1), ((0, 2, 1), -1), ((1, 0, 2), -1), ((1, 2, 0), 1), ((2, 0, 1), 1), ((2, 1, 0), -1))
    idx = np.zeros((16, 6, 3), np.int64)
    sgn = np.zeros((16, 6), np.float32)
    for i in range(4):
        for j in range(4):
            rows = [r for r in range(4) if r != i]
            cols = [c for c in range(4) if c != j]
            for p, (perm, s) in enumerate(perms):
                idx[4 * i + j, p] = [rows[k] * 4 + cols[perm[k]] for k in range(3)]
                sgn[4 * i + j, p] = s * (-1) ** (i + j)
    return idx, sgn


_COF = _cofactor_tables()
_COF_DEV = {}


def inv4x4(m):
    """Inverse of 4x4 matrices [..., 4, 4] by cofactors (adjugate / determinant):
    the 96 minor-term triples of the 16 entries are gathered by a one-hot matrix
    product (exact: each output is 1.0 x one entry; and its backward is a matrix
    product, where an index gather's backward is an accumulating index_put that
    cannot be captured in a HIP graph), then their products (explicit multiplies:
    prod()'s backward syncs) and signed sums, a
    determinant and a division -- a handful of device ops, differentiable and
    graph-capturable (the LAPACK path behind torch.inverse is neither); agrees with
    torch.inverse to fp32 rounding on the well-conditioned camera / pose matrices
    of this path."""
    key = (m.device, m.dtype)
    if key not in _COF_DEV:  # first use is outside any graph capture (warmup steps)
        onehot = torch.zeros(16, _COF[0].size, dtype=m.dtype)
        onehot[torch.as_tensor(_COF[0]).reshape(-1), torch.arange(_COF[0].size)] = 1.0
        _COF_DEV[key] = (onehot.to(m.device), torch.as_tensor(_COF[1], device=m.device, dtype=m.dtype))
    onehot, sgn = _COF_DEV[key]
    a = m.reshape(-1, 16)
    terms = (a @ onehot).reshape(*m.shape[:-2], 16, 6, 3)
    # the triple products written out: prod()'s backward looks for zeros with nonzero(), a host sync
    trip = terms[..., 0] * terms[..., 1] * terms[..., 2]
    cof = (trip * sgn).sum(-1).reshape(*m.shape[:-2], 4, 4)  # C_ij
    det = (m[..., 0, :] * cof[..., 0, :]).sum(-1)
    return cof.transpose(-1, -2) / det[..., None, None]


def world_rays(pixels_norm, camera_mat, world_mat, scale_mat):
    """rays_o [R,3], unit rays_d [R,3], |p - o| [R,1] (training.py:474-487)."""
    inv_s, inv_w, inv_c = inv4x4(torch.stack([scale_mat, world_mat, camera_mat])).unbind(0)
    inv = inv_s @ inv_w @ inv_c  # [4,4]
    o = inv[:3, 3]
    R = pixels_norm.shape[0]
    ph = torch.cat([pixels_norm, torch.ones(R, 2, device=pixels_norm.device)], -1)  # [x, y, 1, 1]
    pw = (ph @ inv.t())[:, :3]
    v = pw - o
    n = v.norm(2, -1)
    return o.expand(R, 3).contiguous(), (v / n.unsqueeze(-1)).contiguous(), n.view(-1, 1)


def near_far_from_sphere(rays_o, depth_range):
    """The reference computes the sphere mid-point and then overwrites near/far
    with the configured depth range (training.py:101-118)."""
    R = rays_o.shape[0]
    near = torch.full((R, 1), float(depth_range[0]), device=rays_o.device)
    far = torch.full((R, 1), float(depth_range[1]), device=rays_o.device)
    return near, far


def get_cos_anneal_ratio(iter_step, anneal_end):
    return 1.0 if anneal_end == 0.0 else float(np.min([1.0, iter_step / anneal_end]))


def vec2skew(v):
    z = torch.zeros(1, dtype=v.dtype, device=v.device)
    return torch.stack([torch.cat([z, -v[2:3], v[1:2]]), torch.cat([v[2:3], z, -v[0:1]]),
                        torch.cat([-v[1:2], v[0:1], z])], 0)


def Exp(r):
    """so(3) -> SO(3), Rodrigues with the reference's +1e-15 on |r|."""
    K = vec2skew(r)
    th = r.norm() + 1e-15
    I = torch.eye(3, dtype=r.dtype, device=r.device)
    return I + (torch.sin(th) / th) * K + ((1 - torch.cos(th)) / th ** 2) * (K @ K)


def convert3x4_4x4(m):
    if torch.is_tensor(m):  # the [0, 0, 0, 1] row from torch.eye: no host scalar copy (graph-capturable)
        row = torch.eye(4, dtype=m.dtype, device=m.device)[3:4]
        if m.dim() == 3:
            return torch.cat([m, row.expand(m.shape[0], 1, 4)], 1)
        return torch.cat([m, row], 0)
    if m.ndim == 3:
        out = np.concatenate([m, np.zeros_like(m[:, 0:1])], 1)
        out[:, 3, 3] = 1.0
        return out
    out = np.concatenate([m, np.array([[0, 0, 0, 1]], dtype=m.dtype)], 0)
    out[3, 3] = 1.0
    return out


def make_c2w(r, t):
    return convert3x4_4x4(torch.cat([Exp(r), t.unsqueeze(1)], 1))


class PoseRetriever(nn.Module):
    """Reference: model/poses_retriever.py:6-32 (learnable axis-angle + translation per camera)."""

    def __init__(self, num_cams, learn_R=True, learn_t=True, init_c2w=None):
        super().__init__()
        self.num_cams = num_cams
        if init_c2w is not None:
            self.init_c2w = nn.Parameter(init_c2w, requires_grad=False)
        else:
            self.init_c2w = nn.Parameter(torch.eye(4).float().unsqueeze(0).repeat(num_cams, 1, 1),
                                         requires_grad=False)
        self.r = nn.Parameter(torch.zeros(num_cams, 3), requires_grad=learn_R)
        self.t = nn.Parameter(torch.zeros(num_cams, 3), requires_grad=learn_t)

    def forward(self, cam_id):
        cam_id = int(cam_id)
        c2w = make_c2w(self.r[cam_id], self.t[cam_id])
        if self.init_c2w is not None:
            c2w = c2w @ self.init_c2w[cam_id]
        return c2w

    def pose_at(self, idx):
        """forward() for a device index tensor [1]: gathers instead of int(cam_id), so
        no host sync (graph-capturable); same arithmetic."""
        c2w = make_c2w(self.r.index_select(0, idx)[0], self.t.index_select(0, idx)[0])
        if self.init_c2w is not None:
            c2w = c2w @ self.init_c2w.index_select(0, idx)[0]
        return c2w
