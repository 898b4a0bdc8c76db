"""Stage-1 motion model and losses.

  MotionNetwork                   model/neus_fields.py:79-190
  euler_angles_to_matrix (XYZ)    utils_poses/pose_pytorch3d.py (pytorch3d convention)
  scene_flow_loss                 train.py:467-477 (sdf_loss)
  project_flow / warp_pixel       train.py:478-496, 235-244 (flow-RGB warp)
  stage1_terms_fused              train.py:467-504 per-sample work in one HIP pass each way
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
import torch.nn.functional as F

from .embedder import get_embedder
from .fields import effective_weight, release_weight_norm_graphs


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
        release_weight_norm_graphs(self)

    def _device(self):
        return self.lin0.bias.device

    def forward(self, inputs):
        if self.embed_fn_fine is not None:
            inputs = self.embed_fn_fine(inputs)
        x = inputs
        for l in range(self.num_layers - 1):
            if l in self.skip_in:
                x = torch.cat([x, inputs], 1) / np.sqrt(2)
            lin = getattr(self, f"lin{l}")
            # the weight-norm weight computed here, not by the module's pre-hook (which would keep
            # this step's graph alive on the module: release_weight_norm_graphs)
            x = F.linear(x, effective_weight(lin), lin.bias)
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

    # -- batched, device-resident form (graph-capturable) -------------------
    def interval_time_grid(self, total_nb_images, nb_sample_timestep, n_intervals=None):
        """The reference's per-interval time grids, built once on the host exactly as
        compute_consecutive_relative_pose builds them (torch.linspace(t_k, t_k+1, n+1)[:-1],
        Δt = grid[1] - grid[0]): ([K, n] steps, [K] Δt) for the intervals k -> k+1,
        k < K (default K = total_nb_images - 1)."""
        K = total_nb_images - 1 if n_intervals is None else n_intervals
        steps, dts = [], []
        for k in range(K):
            t0 = k / (total_nb_images - 1) * 2 - 1
            t1 = (k + 1.0) / (total_nb_images - 1) * 2 - 1
            g = torch.linspace(t0, t1, nb_sample_timestep + 1)[:-1]
            steps.append(g)
            dts.append(g[1] - g[0])
        dev = self._device()
        return torch.stack(steps).to(dev), torch.stack(dts).to(dev)

    def batched_relative_poses(self, steps, dts, extra_t=None):
        """Every consecutive relative pose at once: one MotionNetwork forward over all
        K*n time steps, then the reference's Euler recurrence (neus_fields.py:146-165)
        T <- R_s T + V_s, R <- R R_s run for all K intervals together (n batched 3x3
        steps instead of K*n host-launched ones).  steps [K, n], dts [K] -> [K, 4, 4]."""
        K, n = steps.shape
        t = steps.reshape(-1, 1)
        if extra_t is not None:  # more time queries in the same network evaluation (returned as well)
            t = torch.cat([t, extra_t.reshape(-1, 1).to(t.dtype)])
        omega, vel = self.forward(t)
        extra = (omega[K * n:], vel[K * n:]) if extra_t is not None else None
        omega, vel = omega[:K * n], vel[:K * n]
        if omega.is_cuda:  # the recurrence forward and backward in one launch each (cn_euler_chain)
            P = _EulerChainFn.apply(omega, vel, dts.reshape(K).contiguous(), K, n)
            return P if extra is None else (P, extra)
        dt = dts.view(K, 1, 1)
        Rs = euler_angles_to_matrix(omega.view(K, n, 3) * dt, "XYZ")  # [K, n, 3, 3]
        Vs = vel.view(K, n, 3) * dt
        R = torch.eye(3, device=steps.device).expand(K, 3, 3)
        T = torch.zeros(K, 3, 1, device=steps.device)
        for s in range(n):
            T = Rs[:, s] @ T + Vs[:, s, :, None]
            R = R @ Rs[:, s]
        top = torch.cat([R, T], -1)  # [K, 3, 4]
        row = torch.eye(4, device=steps.device)[3:4].expand(K, 1, 4)  # no host scalar copy: capturable
        P = torch.cat([top, row], 1)
        return P if extra is None else (P, extra)


class _EulerChainFn(torch.autograd.Function):
    """All K consecutive relative poses from the motion network's velocities: the
    reference's Euler recurrence (neus_fields.py:146-165) as one HIP thread per interval
    (cn_euler_chain), and its reverse recurrence for d omega, d vel (cn_euler_chain_bwd)
    -- instead of ~150 tiny 3x3 launches forward and backward."""

    @staticmethod
    def forward(ctx, omega, vel, dts, K, n):
        from . import ops  # noqa: F401  (the library is loaded by ops)
        from . import _lib
        P = torch.empty(K, 4, 4, device=omega.device, dtype=torch.float32)
        stream = torch.cuda.current_stream().cuda_stream
        _lib.call("cn_euler_chain", K, n, omega.data_ptr(), omega.stride(0), vel.data_ptr(), vel.stride(0),
                  dts.data_ptr(), P.data_ptr(), stream)
        ctx.save_for_backward(omega, vel, dts)
        ctx.Kn = (K, n)
        return P

    @staticmethod
    def backward(ctx, dP):
        from . import _lib
        omega, vel, dts = ctx.saved_tensors
        K, n = ctx.Kn
        dP = dP.contiguous()
        domega = torch.empty(K * n, 3, device=omega.device, dtype=torch.float32)
        dvel = torch.empty(K * n, 3, device=omega.device, dtype=torch.float32)
        stream = torch.cuda.current_stream().cuda_stream
        _lib.call("cn_euler_chain_bwd", K, n, omega.data_ptr(), omega.stride(0), vel.data_ptr(), vel.stride(0),
                  dts.data_ptr(), dP.data_ptr(), domega.data_ptr(), dvel.data_ptr(), stream)
        return domega, dvel, None, None, None


class _Mat4Chain(torch.autograd.Function):
    """Running products C_j = A_j ... A_0 of A [n, 4, 4] (cn_mat4_chain_fwd / _bwd): one
    launch each way instead of a 4x4 GEMM launch per product and two per product back."""

    @staticmethod
    def forward(ctx, A):
        from . import _lib
        A = A.contiguous()
        C = torch.empty_like(A)
        _lib.call("cn_mat4_chain_fwd", A.shape[0], A.data_ptr(), C.data_ptr(),
                  torch.cuda.current_stream(A.device).cuda_stream)
        ctx.save_for_backward(A, C)
        return C

    @staticmethod
    def backward(ctx, dC):
        from . import _lib
        A, C = ctx.saved_tensors
        dA = torch.empty_like(A)
        _lib.call("cn_mat4_chain_bwd", A.shape[0], A.data_ptr(), C.data_ptr(), dC.contiguous().data_ptr(),
                  dA.data_ptr(), torch.cuda.current_stream(A.device).cuda_stream)
        return dA


def mat4_chain(A):
    """[n, 4, 4] -> the running products [A_0, A_1 A_0, ..., A_{n-1} ... A_0] (fp32, device)."""
    return _Mat4Chain.apply(A)


def masked_chain(P, lo, hi):
    """w2c of the frames lo -> hi from consecutive relative poses P [K, 4, 4]:
    P[hi-1] @ ... @ P[lo] (= compute_w2c_mappings(rel[lo:hi])[-1], neus_fields.py:174-186),
    with lo / hi device integer tensors: every interval outside [lo, hi) enters as the
    identity, so the shapes (and a captured graph) do not depend on the indices."""
    K = P.shape[0]
    k = torch.arange(K, device=P.device)
    m = ((k >= lo) & (k < hi)).view(K, 1, 1)
    eye = torch.eye(4, device=P.device)
    return mat4_chain(torch.where(m, P, eye))[K - 1]


def _allreduce_sum(x, group):
    """Sum a detached scalar over the data-parallel ranks (the global normalisers of
    SURVEY.md §8e); identity without a process group."""
    if group is None:
        return x
    import torch.distributed as dist
    x = x.clone()
    dist.all_reduce(x, op=dist.ReduceOp.SUM, group=group)
    return x


def _world(group):
    if group is None:
        return 1
    import torch.distributed as dist
    return dist.get_world_size(group)


def scene_flow_loss(pts, normals, sdf_flows, weights, angular_velocity, velocity, group=None):
    """SDF scene-flow consistency (train.py:467-477): the scene flow ω × p + v of
    every sample must satisfy the level-set equation ∇sdf · flow + ∂sdf/∂t = 0;
    L1, weighted by the detached render weights over their global sum.  With a
    process group, Σw is all-reduced before the divide and the rank's term is
    scaled by the world size, so the mean of the ranks' gradients is the gradient
    of the single-GPU loss over all rays."""
    pts = pts.reshape(-1, 3)
    normals = normals.reshape(-1, 3)
    sdf_flows = sdf_flows.reshape(-1)
    w = weights.reshape(-1).detach()
    omega = angular_velocity.reshape(1, 3).expand(pts.shape[0], 3)
    vel = velocity.reshape(1, 3).expand(pts.shape[0], 3)
    flow = torch.cross(omega, pts, dim=-1) + vel
    lhs = torch.sum(flow * normals, dim=-1)
    den = _allreduce_sum(torch.sum(w), group)
    return _world(group) * torch.sum(torch.abs(lhs + sdf_flows) * w) / (den + 1e-10)


def _rows(t, c):
    """t viewed as [M, c] rows of a common leading dimension (the renderer's outputs are
    column slices of its [M, 4] buffers), and that leading dimension."""
    v = t.reshape(-1, c)
    if v.stride(-1) != 1 or (v.shape[0] > 1 and v.stride(0) < c):
        v = v.contiguous()
    return v, (v.stride(0) if v.shape[0] > 1 else c)


class _Stage1Terms(torch.autograd.Function):
    """cn_stage1_fwd / cn_stage1_bwd: the per-sample work of the stage-1 losses in one
    HIP pass each way (train.py:467-477 scene-flow residual sums, the per-ray weighted
    point sums the flow projection of train.py:484-495 reduces to, and the world points
    of the SDF-consistency query, train.py:502-504).  Outputs (num, sumw, ray_acc, x):
    num = Σ|(ω × p + v)·n + f| w and sumw = Σw over the rank's samples (w detached, as
    the reference's weights.detach()); ray_acc [R, 4] = (Σ_s w p, Σ_s w); x [M, 4] =
    (cw2 (p, 1), t_world).  x carries gradient to cw2 and the points only when
    x_grad (sdf_consistency_enable_pose_grad, train.py:496)."""

    @staticmethod
    def forward(ctx, pts, normals, flows, weights, mv, cw2, t_world, x_grad):
        from . import _lib
        R, S = weights.shape
        p, ldp = _rows(pts, 3)
        n, ldn = _rows(normals, 3)
        f, ldf = _rows(flows, 1)
        w = weights.contiguous()
        mv = mv.contiguous()
        cw2 = cw2.contiguous()
        dev = w.device
        sums = torch.empty(2, device=dev, dtype=torch.float32)
        ray_acc = torch.empty(R, 4, device=dev, dtype=torch.float32)
        x = torch.empty(R * S, 4, device=dev, dtype=torch.float32)
        ws = torch.empty(_lib.load().cn_stage1_workspace_bytes(R) // 4, device=dev, dtype=torch.float32)
        stream = torch.cuda.current_stream(dev).cuda_stream
        _lib.call("cn_stage1_fwd", R, S, p.data_ptr(), ldp, n.data_ptr(), ldn, f.data_ptr(), ldf, w.data_ptr(),
                  mv.data_ptr(), cw2.data_ptr(), float(t_world), ray_acc.data_ptr(), x.data_ptr(), 4,
                  sums.data_ptr(), ws.data_ptr(), stream)
        ctx.save_for_backward(p, n, f, w, mv, cw2)
        ctx.meta = (R, S, ldp, ldn, ldf, bool(x_grad), (pts.shape, normals.shape, flows.shape))
        num, sumw = sums[0:1], sums[1:2]
        ctx.mark_non_differentiable(sumw)
        if not x_grad:
            ctx.mark_non_differentiable(x)
        return num, sumw, ray_acc, x

    @staticmethod
    def backward(ctx, g_num, _g_sumw, g_ray, g_x):
        from . import _lib
        p, n, f, w, mv, cw2 = ctx.saved_tensors
        R, S, ldp, ldn, ldf, x_grad, (pshape, nshape, fshape) = ctx.meta
        dev = w.device
        need = ctx.needs_input_grad
        g_num = torch.zeros(1, device=dev) if g_num is None else g_num.contiguous()
        g_ray = None if g_ray is None else g_ray.contiguous()
        g_x = g_x.contiguous() if (x_grad and g_x is not None) else None
        dG = torch.empty(R * S, 4, device=dev, dtype=torch.float32)
        dw = torch.empty(R, S, device=dev, dtype=torch.float32) if (need[3] and g_ray is not None) else None
        dp = torch.empty(R * S, 3, device=dev, dtype=torch.float32) if need[0] else None
        dmc = torch.empty(18, device=dev, dtype=torch.float32)
        ws = torch.empty(_lib.load().cn_stage1_workspace_bytes(R) // 4, device=dev, dtype=torch.float32)
        ptr = lambda t: 0 if t is None else t.data_ptr()
        stream = torch.cuda.current_stream(dev).cuda_stream
        _lib.call("cn_stage1_bwd", R, S, p.data_ptr(), ldp, n.data_ptr(), ldn, f.data_ptr(), ldf, w.data_ptr(),
                  mv.data_ptr(), cw2.data_ptr(), g_num.data_ptr(), ptr(g_ray), ptr(g_x), 4, dG.data_ptr(), 4,
                  dG[:, 3:].data_ptr(), 4, ptr(dw), ptr(dp), 3, dmc.data_ptr(), ws.data_ptr(), stream)
        dnormals = dG[:, :3].reshape(nshape) if need[1] else None
        dflows = dG[:, 3:].reshape(fshape) if need[2] else None
        dpts = dp.reshape(pshape) if dp is not None else None
        dmv = dmc[:6] if need[4] else None
        dcw2 = None
        if need[5] and g_x is not None:
            dcw2 = torch.cat([dmc[6:].view(3, 4), torch.zeros(1, 4, device=dev)], 0)
        return dpts, dnormals, dflows, dw, dmv, dcw2, None, None


def stage1_terms_fused(pts, normals, sdf_flows, weights, angular_velocity, velocity, cw2, t_world, x_grad,
                       group=None):
    """The fused stage-1 pass (cn_stage1_fwd/bwd) -> (sdf_loss, pbar [R, 3], wbar [R, 1],
    x [M, 4]): sdf_loss as scene_flow_loss, the per-ray sums project_flow_sums takes and
    the world points (with the world time step) of the SDF-consistency re-query."""
    R = weights.shape[0]
    mv = torch.cat([angular_velocity.reshape(3), velocity.reshape(3)])
    num, sumw, ray_acc, x = _Stage1Terms.apply(pts, normals, sdf_flows, weights.reshape(R, -1), mv, cw2, t_world,
                                               x_grad)
    den = _allreduce_sum(sumw, group)
    sdf_loss = (_world(group) * num / (den + 1e-10)).reshape(())
    return sdf_loss, ray_acc[:, :3], ray_acc[:, 3:], x


def project_flow(pts, weights, w2c, ref_camera_mat, scale_mat, normalized_pixels, img_hw):
    """Forward optical flow to reference frames (train.py:484-495): the
    weight-averaged sample point of each ray, mapped by the relative pose w2c
    [T, 4, 4] (or [4, 4]) and projected with the reference cameras ref_camera_mat
    [T, 4, 4] (or [1, 4, 4]); returns pixel offsets [T, R, 2] (or [R, 2]).
    The reference maps every sample and then averages; by linearity
    Σ_s w (R p + t) = R (Σ_s w p) + (Σ_s w) t, so the per-ray sums are formed once
    and each frame costs O(R), not O(R·S) (no [T, R·S, 3] intermediate)."""
    R = normalized_pixels.shape[0]
    w = weights.reshape(R, -1, 1)
    pbar = torch.sum(w * pts.reshape(R, -1, 3), dim=1)   # [R, 3]
    wbar = torch.sum(w, dim=1)                           # [R, 1]
    return project_flow_sums(pbar, wbar, w2c, ref_camera_mat, scale_mat, normalized_pixels, img_hw)


def project_flow_sums(pbar, wbar, w2c, ref_camera_mat, scale_mat, normalized_pixels, img_hw):
    """project_flow from the per-ray sums pbar = Σ_s w p [R, 3], wbar = Σ_s w [R, 1]."""
    single = w2c.dim() == 2
    if single:
        w2c, ref_camera_mat = w2c[None], ref_camera_mat.reshape(1, 4, 4)
    wp = torch.einsum("tij,rj->tri", w2c[:, :3, :3], pbar) + wbar[None] * w2c[:, None, :3, 3]  # [T, R, 3]
    KS = scale_mat.reshape(-1, 4, 4)[0, :3, :3] @ ref_camera_mat[:, :3, :3]  # [T, 3, 3]
    pix = torch.einsum("tij,trj->tri", KS, wp)
    pix = pix[..., :2] / pix[..., 2:3]
    flow = pix - normalized_pixels
    h, w_ = img_hw
    flow = torch.stack([flow[..., 0] * (w_ / 2), flow[..., 1] * (h / 2)], -1)
    return flow[0] if single else flow


def affine_points(pts, m):
    """(m[:3, :3] @ pts.T + m[:3, 3:]).T for pts [N, 3] as three fused multiply-adds over
    the rows (a [3, 3] x [3, N] matrix product is a skinny GEMM; this is a stream)."""
    out = torch.addcmul(m[:3, 3], pts[:, 0:1], m[:3, 0])
    out = torch.addcmul(out, pts[:, 1:2], m[:3, 1])
    return torch.addcmul(out, pts[:, 2:3], m[:3, 2])


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


def flow_rgb_loss(flow_fw, sampled_pixel, ref_img, rgb_gt, group=None):
    """Photometric loss of the reference frame warped by the predicted flow
    (train.py:506-515), masked to correspondences inside the image.  Batched over T
    reference frames: flow_fw [T, R, 2], ref_img [T, 3, H, W] -> per-frame losses [T]
    (or [R, 2] / [1, 3, H, W] -> a scalar).  Σvalid is all-reduced with a process group."""
    single = flow_fw.dim() == 2
    if single:
        flow_fw = flow_fw[None]
    T = flow_fw.shape[0]
    corr = sampled_pixel[None] + flow_fw  # [T, R, 2]
    with torch.no_grad():  # ((corr >= 0) & (corr < [W, H])).all(dim=1)
        cx, cy = corr[..., 0], corr[..., 1]
        valid = ((cx >= 0) & (cx < ref_img.shape[3]) & (cy >= 0) & (cy < ref_img.shape[2])).unsqueeze(-1)
    # warp_pixel's uv: [T, 2, R, 1] -> grid [T, R, 1, 2] -> [T, 3, R, 1]
    warped = warp_pixel(ref_img, corr.permute(0, 2, 1).unsqueeze(-1))[..., 0].permute(0, 2, 1)  # [T, R, 3]
    num = torch.sum(torch.abs(warped - rgb_gt[None]) * valid, dim=(1, 2))
    den = _allreduce_sum(torch.sum(valid, dim=(1, 2)).float(), group)
    out = _world(group) * num / (den + 1e-10)
    return out[0] if single else out


def world_points(pts, cw2):
    """Sample points mapped into the world (canonical) frame for the SDF
    consistency re-query (train.py:497-505)."""
    return affine_points(pts.reshape(-1, 3), cw2)
