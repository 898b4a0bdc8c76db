"""NeuSRenderer on the HIP kernels (reference: model/neus_renderer.py:107-591).

forward() keeps the reference signature and output dict.  Inside:
  coarse z + stratified jitter           cn_coarse_z            (neus_renderer.py:466-483)
  4 x [NeuS up-sample + merge + SDF]     cn_up_sample_merge,    (neus_renderer.py:492-525)
                                         SDF MLP on new points
  render_core: SDF fwd + ∇ₓSDF + colour  _SDFFieldFn, _ColorFieldFn (neus_renderer.py:337-358)
  alpha compositing                      _CompositeFn           (neus_renderer.py:360-420)
Every step is a HIP launch on the current stream; the only host work is
launch bookkeeping.  `t_rand` comes from torch's device RNG (the reference
draws it on the CPU, neus_renderer.py:482); tests inject it via `t_rand=`.
"""
from __future__ import annotations

import torch
import torch.nn as nn

from . import ops
from .fields import _empty

# the sampler as one C call (cn_sample: coarse z, the up-sampling rounds and their SDF queries composed in
# C++); False: launch by launch from Python (sample_z_composed)
SAMPLE_NATIVE = True
# the forward without gradient (evaluation, inference) as one C call (cn_render_fwd) where the feature head folds;
# False: launch by launch from Python
RENDER_NATIVE = True


class _PointsFn(torch.autograd.Function):
    """Section midpoints along the rays (neus_renderer.py:337-350):
    pts_time = [rays_o + rays_d * mid_z, t]; backward gives the ray gradients."""

    @staticmethod
    def forward(ctx, rays_o, rays_d, z, time_step, near, far, n_coarse):
        R, S = z.shape
        pts = torch.empty(R * S, 4, device=z.device)
        ops.points(rays_o, rays_d, z, time_step, pts, mid=True, near=near, far=far, n_coarse=n_coarse)
        ctx.save_for_backward(z, near, far)
        ctx.n_coarse = n_coarse
        return pts

    @staticmethod
    def backward(ctx, dpts):
        z, near, far = ctx.saved_tensors
        R = z.shape[0]
        want_o, want_d = ctx.needs_input_grad[0], ctx.needs_input_grad[1]
        if dpts is None or not (want_o or want_d):
            return (None,) * 7
        if dpts.stride(1) != 1:
            dpts = dpts.contiguous()
        do = torch.empty(R, 3, device=z.device) if want_o else None
        dd = torch.empty(R, 3, device=z.device) if want_d else None
        ops.points_bwd(z, dpts, do, dd, mid=True, near=near, far=far, n_coarse=ctx.n_coarse)
        return do, dd, None, None, None, None, None


class _CompositeFn(torch.autograd.Function):
    """(z, sdf, ∇ₓSDF, rgb, rays_d, inv_s) -> (colour, weighted z, weights, cdf)."""

    @staticmethod
    def forward(ctx, z, sdf, G, rgb, rays_d, inv_s, near, far, n_coarse, car):
        ctx.set_materialize_grads(False)
        R, S = z.shape
        dev = z.device
        car = ops.device_scalar(car, dev)  # cos_anneal_ratio: float or device tensor (no host sync)
        color = _empty(R, 3, dev)
        depth = _empty(R, 1, dev)
        weights = _empty(R, S, dev)
        cdf = _empty(R, S, dev)
        ops.composite_fwd(z, sdf, G, rgb, rays_d, inv_s, near, far, n_coarse, car, color, depth, weights, cdf)
        ctx.save_for_backward(z, sdf, G, rgb, rays_d, inv_s, near, far)
        ctx.n_coarse, ctx.car = n_coarse, car
        return color, depth, weights, cdf

    @staticmethod
    def backward(ctx, dcolor, ddepth, dweights, dcdf):
        # z is sampled under no_grad in the reference (neus_renderer.py:492-525): no gradient
        z, sdf, G, rgb, rays_d, inv_s, near, far = ctx.saved_tensors
        R, S = z.shape
        M, dev = R * S, z.device
        dsdf = _empty(M, 1, dev)
        dG = _empty(M, 4, dev)
        drgb = _empty(M, 3, dev)
        dinv = torch.empty(R, device=dev)
        c = lambda t: None if t is None else t.contiguous()  # noqa: E731
        drays_d = torch.empty(R, 3, device=dev) if ctx.needs_input_grad[4] else None
        ops.composite_bwd(z, sdf, G, rgb, rays_d, inv_s, near, far, ctx.n_coarse, ctx.car, c(dcolor), c(ddepth),
                          c(dweights), c(dcdf), dsdf, dG, drgb, dinv, drays_d)
        dinv_s = dinv.sum().reshape(inv_s.shape) if ctx.needs_input_grad[5] else None
        return (None, dsdf if ctx.needs_input_grad[1] else None, dG if ctx.needs_input_grad[2] else None,
                drgb if ctx.needs_input_grad[3] else None, drays_d, dinv_s, None, None, None, None)


class _RenderTrainFn(torch.autograd.Function):
    """render_core under autograd (neus_renderer.py:307-450) as two C calls, cn_render_train_fwd / cn_render_bwd:
    the points, the SDF field with ∇ₓSDF, the colour network with the folded feature head and the compositing,
    and their backward with the gradient sums autograd makes between _PointsFn, _SDFFieldFn, _ColorFieldFn and
    _CompositeFn -- bitwise that composition (RENDER_NATIVE off).
    (rays_o, rays_d, inv_s, z, time_step, near, far, car, n_coarse, layouts and packs, *sdf params, *colour params)
    -> (sdf [M,1], ∇ₓSDF [M,4], points [M,4], colour [R,3], weighted z [R,1], weights [R,S], cdf [R,S])."""

    @staticmethod
    def forward(ctx, rays_o, rays_d, inv_s, z, time_step, near, far, car, n_coarse, sdf_lay, sdf_pk, col_lay, col_pk,
                *params):
        ctx.set_materialize_grads(False)
        sn, k1 = ops.sdf_net(sdf_lay, sdf_pk)
        cn, k2 = ops.color_net(col_lay, col_pk)
        inv_s = inv_s.contiguous()
        out, state, d = ops.render_train_fwd(sn, cn, rays_o, rays_d, near, far, time_step, inv_s, car, n_coarse, z)
        # the descriptor points into the inputs, the networks' images and the sdf / ∇ₓSDF outputs: hold them
        ctx.native = (sn, cn, k1, k2, state, d, (rays_o, rays_d, inv_s, z, time_step, near, far, car))
        ctx.save_for_backward(out["sdf"], out["grad"])
        ctx.lays, ctx.inv_shape = (sdf_lay, col_lay), inv_s.shape
        ctx.pose = ctx.needs_input_grad[0] or ctx.needs_input_grad[1]
        if not ctx.pose:
            ctx.mark_non_differentiable(out["pts"])
        return out["sdf"], out["grad"], out["pts"], out["color"], out["depth"], out["weights"], out["cdf"]

    @staticmethod
    def backward(ctx, dsdf, dgrad, dpts, dcolor, ddepth, dweights, dcdf):
        sn, cn, k1, k2, state, d, inputs = ctx.native
        ctx.native = None
        saved = ctx.saved_tensors  # (sdf, ∇ₓSDF: read by the compositing's backward)
        sdf_lay, col_lay = ctx.lays
        dev = state.device
        R = inputs[3].shape[0]
        c = lambda t: None if t is None else t.contiguous()  # noqa: E731
        sdf_dWs = [torch.empty(sdf_lay.out_dim[l], sdf_lay.in_dim[l], device=dev) for l in range(sdf_lay.n_lin)]
        sdf_dbs = [torch.empty(sdf_lay.out_dim[l], device=dev) for l in range(sdf_lay.n_lin)]
        col_dWs = [torch.empty(col_lay.out_dim[l], col_lay.in_dim[l], device=dev) for l in range(col_lay.n_lin)]
        col_dbs = [torch.empty(col_lay.out_dim[l], device=dev) for l in range(col_lay.n_lin)]
        dinv = torch.empty(R, device=dev)
        do = torch.empty(R, 3, device=dev) if ctx.pose else None
        dd = torch.empty(R, 3, device=dev) if ctx.pose else None
        ops.render_bwd(d, state, dcolor=c(dcolor), ddepth=c(ddepth), dweights=c(dweights), dcdf=c(dcdf), dsdf=c(dsdf),
                       dgrad=c(dgrad), dpts=c(dpts) if ctx.pose else None, sdf_dWs=sdf_dWs, sdf_dbs=sdf_dbs,
                       col_dWs=col_dWs, col_dbs=col_dbs, dinv_s=dinv, drays_o=do, drays_d=dd)
        del k1, k2, state, inputs, saved
        dinv_s = dinv.sum().reshape(ctx.inv_shape) if ctx.needs_input_grad[2] else None
        grads = []
        for w, b in zip(sdf_dWs, sdf_dbs):
            grads += [w, b]
        for w, b in zip(col_dWs, col_dbs):
            grads += [w, b]
        return (do if ctx.needs_input_grad[0] else None, dd if ctx.needs_input_grad[1] else None, dinv_s) + \
            (None,) * 10 + tuple(grads)


class NeuSRenderer(nn.Module):
    """Reference: model/neus_renderer.py:107-135 (constructor) and 453-584 (forward)."""

    def __init__(self, nerf, sdf_network, deviation_network, color_network, motion_network, n_samples,
                 n_importance, n_outside, up_sample_steps, perturb, n_max_network_queries,
                 importance_sampling_start, naive_render):
        super().__init__()
        self.nerf = nerf
        self.sdf_network = sdf_network
        self.deviation_network = deviation_network
        self.color_network = color_network
        self.motion_network = motion_network
        self.n_samples = n_samples
        self.n_importance = n_importance
        self.n_outside = n_outside
        self.up_sample_steps = up_sample_steps
        self.perturb = perturb
        self.n_max_network_queries = n_max_network_queries
        self.importance_sampling_start = importance_sampling_start
        self.naive_render = naive_render
        if n_outside > 0:
            raise NotImplementedError("n_outside > 0 (NeRF++ background) is out of scope; every config uses 0")
        if naive_render:
            raise NotImplementedError("naive_render (logistic up-sampler) is out of scope; every config uses False")
        # opt-in: keep forward()'s SDF weight images (effective weights + packed GEMM images)
        # in last_sdf_pack for a second SDF query of the same step; the caller must clear it
        # (it holds the step's autograd graph)
        self.expose_sdf_pack = False
        self.last_sdf_pack = None

    def set_mfma_dtype(self, dtype: str):
        """"fp32" (default: exact fp32 MFMA products, the |Δ| <= 1e-4 parity path),
        "bf16x6" (fp32 GEMMs on the bf16 MFMA: both operands split into three bf16
        terms, six term products accumulated in fp32; same parity bar) or
        "bf16" (config C3, "bf16 MLP MFMA": every MLP GEMM rounds its operands to
        bf16 and accumulates in fp32; activations, epilogues, sampling and
        compositing stay fp32)."""
        if dtype not in ("fp32", "bf16", "bf16x6"):
            raise ValueError(f"mfma dtype {dtype!r}")
        self.sdf_network.mfma_dtype = dtype
        self.color_network.mfma_dtype = dtype
        return self

    def _can_fold(self):
        """The feature head folds into the colour network when the colour network reads
        the SDF feature as its last input block and the SDF's hidden width equals the
        feature width (every shipped config; set fold_feature=False to disable)."""
        if not getattr(self, "fold_feature", True):
            return False
        lay, cl = self.sdf_network.layout(), self.color_network.layout()
        L8 = lay.n_lin - 1
        return lay.in_dim[L8] == lay.HL == cl.F and lay.out_dim[L8] == 1 + cl.F

    # -- sampling ------------------------------------------------------------
    @torch.no_grad()
    def sample_z(self, rays_o, rays_d, time_step, near, far, n_samples, n_importance, t_rand, sdf_packed):
        """Coarse + hierarchical z-values [R, n_samples + n_importance] (neus_renderer.py:466-525): one
        cn_sample call (SAMPLE_NATIVE), or launch by launch (sample_z_composed: the same kernels, the same
        bits) when the kernel timer attributes every launch."""
        if not SAMPLE_NATIVE or ops._timer is not None or n_importance <= 0:
            return self.sample_z_composed(rays_o, rays_d, time_step, near, far, n_samples, n_importance, t_rand,
                                          sdf_packed)
        from . import fields  # local: avoid a cycle at import
        R = rays_o.shape[0]
        k = n_importance // self.up_sample_steps
        z = _empty(R, n_samples + self.up_sample_steps * k, rays_o.device)
        net, keep = ops.sdf_net(self.sdf_network.layout(), sdf_packed[2], layered=not fields.FUSED_SDF_QUERY)
        ops.sample(net, rays_o.detach(), rays_d.detach(), near, far, t_rand, time_step.detach(), n_samples,
                   n_importance, self.up_sample_steps, z)
        del keep
        return z

    def sample_z_composed(self, rays_o, rays_d, time_step, near, far, n_samples, n_importance, t_rand, sdf_packed):
        """sample_z launch by launch from Python (the composition cn_sample makes in C++)."""
        R, dev = rays_o.shape[0], rays_o.device
        z = _empty(R, n_samples, dev)
        ops.coarse_z(near, far, n_samples, t_rand, z)
        if n_importance <= 0:
            return z
        sdfn = self.sdf_network
        lay = sdfn.layout()
        pk = sdf_packed[2]
        from .fields import sdf_forward  # local: avoid a cycle at import
        pts = torch.empty(R * n_samples, 4, device=dev)
        ops.points(rays_o, rays_d, z, time_step, pts)
        sdf = sdf_forward(lay, pk, pts, want_feat=False, want_grad=False, keep=False)["sdf"].view(R, n_samples)
        k = n_importance // self.up_sample_steps
        for i in range(self.up_sample_steps):
            n = z.shape[1]
            last = (i + 1) == self.up_sample_steps
            z_out = _empty(R, n + k, dev)
            z_new = _empty(R, k, dev)
            sdf_out = None if last else _empty(R, n + k, dev)
            new_dst = None if last else torch.empty(R * k, dtype=torch.int32, device=dev)
            ops.up_sample_merge(z, sdf, k, 64 * 2 ** i, z_out, z_new, sdf_out, new_dst)
            if not last:
                pts = torch.empty(R * k, 4, device=dev)
                ops.points(rays_o, rays_d, z_new, time_step, pts)
                sdf_forward(lay, pk, pts, want_feat=False, want_grad=False, keep=False, sdf_out=sdf_out,
                            dst=new_dst)
            z, sdf = z_out, sdf_out
        return z

    # -- forward -------------------------------------------------------------
    def forward(self, rays_o, rays_d, ray_d_norm, time_step, near, far, perturb_overwrite=-1, background_rgb=None,
                cos_anneal_ratio=0.0, it=-1, eval=False, t_rand=None, z_vals=None):
        """Reference signature (neus_renderer.py:453) plus two test hooks: `t_rand`
        injects the stratified jitter, `z_vals` [R, S] skips the sampler and renders
        at the given sample positions (the render_core seam)."""
        R = len(rays_o)
        dev = rays_o.device
        if it >= self.importance_sampling_start:
            n_samples, n_importance = self.n_samples, self.n_importance
        else:
            n_samples, n_importance = self.n_samples + self.n_importance, 0
        rays_o = rays_o.contiguous().float()
        rays_d = rays_d.contiguous().float()  # differentiable: pose gradients flow through these
        near = near.contiguous().float()
        far = far.contiguous().float()
        time_step = time_step.reshape(-1)[:1].contiguous().float()
        if not eval and t_rand is None:
            t_rand = torch.rand([R, n_samples], device=dev)
        if eval:
            t_rand = None
        if t_rand is not None:
            t_rand = t_rand.contiguous().float()
        if z_vals is not None:
            z_vals = z_vals.contiguous().float()

        sdf_packed = self.sdf_network.params_and_pack()
        fold = self._can_fold()
        # the SDF feature head folded into the colour network's first layer (both linear,
        # neus_renderer.py:352-358): no feature GEMM forward, the SDF's last adjoint is
        # elementwise backward, one weight gradient fewer (RenderingNetwork.params_and_pack)
        col_packed = self.color_network.params_and_pack(
            fold_feature=(sdf_packed[0][-1], sdf_packed[1][-1]) if fold else None)
        self.last_sdf_pack = sdf_packed if self.expose_sdf_pack else None
        if RENDER_NATIVE and fold and not torch.is_grad_enabled() and background_rgb is None and ops._timer is None:
            return self._forward_native(rays_o, rays_d, ray_d_norm, time_step, near, far, n_samples, n_importance,
                                        t_rand, z_vals, sdf_packed, col_packed, cos_anneal_ratio, eval)
        if z_vals is None:
            z = self.sample_z(rays_o, rays_d, time_step, near, far, n_samples, n_importance, t_rand, sdf_packed)
        else:
            z = z_vals
        S = z.shape[1]

        # render_core (neus_renderer.py:307-450)
        if RENDER_NATIVE and fold and torch.is_grad_enabled() and background_rgb is None and ops._timer is None:
            return self._forward_train_native(rays_o, rays_d, ray_d_norm, time_step, near, far, n_samples, z,
                                              sdf_packed, col_packed, cos_anneal_ratio, eval)
        if rays_o.requires_grad or rays_d.requires_grad:  # pose optimisation (eval.py:51-82, joint pose training)
            pts_time = _PointsFn.apply(rays_o, rays_d, z, time_step, near, far, n_samples)
        else:
            pts_time = torch.empty(R * S, 4, device=dev)
            ops.points(rays_o, rays_d, z, time_step, pts_time, mid=True, near=near, far=far, n_coarse=n_samples)
        sdf, feat, G = self.sdf_network.field(pts_time, want_feat="hidden" if fold else True, want_grad=True,
                                              packed=sdf_packed)
        rgb = self.color_network.color(pts_time, G, rays_d, S, feat, packed=col_packed)
        inv_s = self.deviation_network(torch.zeros([1, 3], device=dev))[:, :1].clip(1 / 1e3, 1 / 1e-3)
        car = ops.device_scalar(cos_anneal_ratio, dev)  # a device scalar: graph replays read the current ratio
        color, depth, weights, cdf = _CompositeFn.apply(z, sdf, G, rgb, rays_d, inv_s, near, far, n_samples, car)
        weighted_z_vals = depth.detach().clone()
        depth_pred = depth / ray_d_norm if eval else depth
        if background_rgb is not None:
            color = color + background_rgb * (1.0 - weights.sum(dim=-1, keepdim=True))
        normals = G[:, :3].reshape(R, S, 3)
        sdf_flows = G[:, 3:].reshape(R, S, 1)
        s_val = (1.0 / inv_s).expand(R * S, 1).reshape(R, S).mean(dim=-1, keepdim=True)
        with torch.no_grad():
            weight_inside = weights.sum(dim=-1).detach()
            weight_outside = weights.new_zeros(R)
        return {
            "sdf": sdf,
            "color_fine": color,
            "depth_pred": depth_pred,
            "weighted_z_vals": weighted_z_vals,
            "s_val": s_val,
            "cdf_fine": cdf,
            "weight_sum": weights.sum(dim=-1, keepdim=True),
            "weight_max": torch.max(weights, dim=-1, keepdim=True)[0],
            "normals": normals,
            "sdf_flows": sdf_flows,
            "sampled_points": pts_time[:, :3].reshape(R, S, 3),
            "weights": weights,
            "inside_sphere": torch.ones_like(weights),
            "weight_inside": weight_inside,
            "weight_outside": weight_outside,
        }

    def _forward_train_native(self, rays_o, rays_d, ray_d_norm, time_step, near, far, n_samples, z, sdf_packed,
                              col_packed, cos_anneal_ratio, eval):
        """render_core under autograd as _RenderTrainFn (cn_render_train_fwd / cn_render_bwd): the outputs of the
        path below, the same bits forward and backward."""
        R, S, dev = rays_o.shape[0], z.shape[1], rays_o.device
        inv_s = self.deviation_network(torch.zeros([1, 3], device=dev))[:, :1].clip(1 / 1e3, 1 / 1e-3)
        car = ops.device_scalar(cos_anneal_ratio, dev)
        params = []
        for w, b in zip(sdf_packed[0], sdf_packed[1]):
            params += [w, b]
        for w, b in zip(col_packed[0], col_packed[1]):
            params += [w, b]
        sdf, G, pts_time, color, depth, weights, cdf = _RenderTrainFn.apply(
            rays_o, rays_d, inv_s, z, time_step, near, far, car, n_samples, self.sdf_network.layout(), sdf_packed[2],
            self.color_network.layout(), col_packed[2], *params)
        weighted_z_vals = depth.detach().clone()
        depth_pred = depth / ray_d_norm if eval else depth
        normals = G[:, :3].reshape(R, S, 3)
        sdf_flows = G[:, 3:].reshape(R, S, 1)
        s_val = (1.0 / inv_s).expand(R * S, 1).reshape(R, S).mean(dim=-1, keepdim=True)
        with torch.no_grad():
            weight_inside = weights.sum(dim=-1).detach()
            weight_outside = weights.new_zeros(R)
        return {
            "sdf": sdf,
            "color_fine": color,
            "depth_pred": depth_pred,
            "weighted_z_vals": weighted_z_vals,
            "s_val": s_val,
            "cdf_fine": cdf,
            "weight_sum": weights.sum(dim=-1, keepdim=True),
            "weight_max": torch.max(weights, dim=-1, keepdim=True)[0],
            "normals": normals,
            "sdf_flows": sdf_flows,
            "sampled_points": pts_time[:, :3].reshape(R, S, 3),
            "weights": weights,
            "inside_sphere": torch.ones_like(weights),
            "weight_inside": weight_inside,
            "weight_outside": weight_outside,
        }

    def _forward_native(self, rays_o, rays_d, ray_d_norm, time_step, near, far, n_samples, n_importance, t_rand,
                        z_vals, sdf_packed, col_packed, cos_anneal_ratio, eval):
        """forward without gradient as one cn_render_fwd call (the sampler, the fields with the folded feature
        head and the compositing composed in C++: the same launches as the path below, the same bits)."""
        R, dev = rays_o.shape[0], rays_o.device
        sn, k1 = ops.sdf_net(self.sdf_network.layout(), sdf_packed[2])
        cn, k2 = ops.color_net(self.color_network.layout(), col_packed[2])
        inv_s = self.deviation_network(torch.zeros([1, 3], device=dev))[:, :1].clip(1 / 1e3, 1 / 1e-3).contiguous()
        car = ops.device_scalar(cos_anneal_ratio, dev)
        o = ops.render_fwd(sn, cn, rays_o, rays_d, near, far, time_step, inv_s, car, n_samples, n_importance,
                           self.up_sample_steps, t_rand=t_rand, z_in=z_vals)
        del k1, k2
        S = o["z"].shape[1]
        depth = o["depth"].view(R, 1)
        weights = o["weights"]
        G = o["grad"]
        return {
            "sdf": o["sdf"].view(R * S, 1),
            "color_fine": o["color"],
            "depth_pred": depth / ray_d_norm if eval else depth,
            "weighted_z_vals": depth.clone(),
            "s_val": (1.0 / inv_s).expand(R * S, 1).reshape(R, S).mean(dim=-1, keepdim=True),
            "cdf_fine": o["cdf"],
            "weight_sum": weights.sum(dim=-1, keepdim=True),
            "weight_max": torch.max(weights, dim=-1, keepdim=True)[0],
            "normals": G[:, :3].reshape(R, S, 3),
            "sdf_flows": G[:, 3:].reshape(R, S, 1),
            "sampled_points": o["pts"][:, :3].reshape(R, S, 3),
            "weights": weights,
            "inside_sphere": torch.ones_like(weights),
            "weight_inside": weights.sum(dim=-1),
            "weight_outside": weights.new_zeros(R),
        }

    def extract_geometry(self, bound_min, bound_max, resolution, threshold=0.0):
        raise NotImplementedError("mesh extraction (PyMCubes) is out of scope (SURVEY.md §2)")
