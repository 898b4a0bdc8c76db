"""Generate golden vectors by running the REFERENCE implementation (this container only).

    python tests/golden/make_golden.py      # needs /root/reference; writes tests/golden/*.npz

The reference hot-path modules (model/neus_embedder.py, model/neus_fields.py,
model/neus_renderer.py, utils_poses/pose_pytorch3d.py) are loaded by path with
the shims SURVEY.md §8c lists: stub `mcubes` / `icecream`, `Tensor.cuda` as the
identity, and empty parent packages so model/__init__.py (which needs cv2 /
imageio / CUDA at import) is bypassed.  Nothing from the reference is copied
into the fixtures except numbers: inputs, weights generated from seeds,
outputs and gradients.  The reference's own files never travel to the GPU box;
these .npz files do.
"""
from __future__ import annotations

import importlib.util
import os
import sys
import types

import numpy as np
import torch

REF = os.environ.get("COPENERF_REFERENCE", "/root/reference")
OUT = os.path.dirname(os.path.abspath(__file__))

SDF_CFG = dict(d_in=4, d_out=257, d_hidden=256, n_layers=8, skip_in=[4], multires=6, bias=0.5, scale=1.0,
               geometric_init=True, weight_norm=True)
COL_CFG = dict(d_feature=256, mode="idr", d_in=11, d_out=3, d_hidden=256, n_layers=4, weight_norm=True,
               multires_view=4, squeeze_out=True, use_negative_ray_vector=False)
REN_CFG = dict(n_samples=64, n_importance=64, n_outside=0, up_sample_steps=4, perturb=1.0,
               n_max_network_queries=64000, importance_sampling_start=0, naive_render=False)


def load_reference():
    sys.dont_write_bytecode = True
    for name in ("mcubes", "icecream"):
        sys.modules.setdefault(name, types.ModuleType(name))
    sys.modules["icecream"].ic = print
    torch.Tensor.cuda = lambda self, *a, **k: self
    for pkg in ("model", "utils_poses"):
        p = types.ModuleType(pkg)
        p.__path__ = []
        sys.modules[pkg] = p

    def load(modname, rel):
        spec = importlib.util.spec_from_file_location(modname, os.path.join(REF, rel))
        mod = importlib.util.module_from_spec(spec)
        sys.modules[modname] = mod
        spec.loader.exec_module(mod)
        return mod

    load("model.neus_embedder", "model/neus_embedder.py")
    load("utils_poses.pose_pytorch3d", "utils_poses/pose_pytorch3d.py")
    fields = load("model.neus_fields", "model/neus_fields.py")
    rend = load("model.neus_renderer", "model/neus_renderer.py")
    return fields, rend


def build_nets(fields, rend, seed, d_hidden_sdf=256, d_hidden_col=256, var=0.3):
    torch.manual_seed(seed)
    sdf = fields.SDFNetwork(**dict(SDF_CFG, d_hidden=d_hidden_sdf))
    col = fields.RenderingNetwork(**dict(COL_CFG, d_hidden=d_hidden_col))
    dev = fields.SingleVarianceNetwork(var)
    r = rend.NeuSRenderer(None, sdf, dev, col, None, **REN_CFG)
    return sdf, col, dev, r


def make_rays(R, seed):
    """Rays from a camera outside the geometric-init sphere (radius 0.5) looking at it,
    as 4x4 pixel patches so the smoothness losses apply."""
    g = torch.Generator().manual_seed(seed)
    o = torch.tensor([0.05, -0.03, 1.6])
    jitter = (torch.rand(R, 2, generator=g) - 0.5) * 0.5
    d = torch.cat([jitter, -torch.ones(R, 1)], -1)
    norm = d.norm(dim=-1, keepdim=True)
    rays_d = d / norm
    return o.expand(R, 3).contiguous(), rays_d.contiguous(), norm


def state(mod):
    return {k: v.detach().numpy().astype(np.float32) for k, v in mod.state_dict().items()}


def run_render(r, rays_o, rays_d, norm, t, near, far, t_rand, car, eval_mode):
    captured = {}
    orig_core = r.render_core

    def core(*a, **k):
        captured["z_vals"] = a[4].detach().clone()
        return orig_core(*a, **k)

    r.render_core = core
    orig_rand = torch.rand
    torch.rand = lambda *a, **k: t_rand.clone()
    try:
        out = r(rays_o, rays_d, norm, t, near, far, cos_anneal_ratio=car, it=0, eval=eval_mode)
    finally:
        torch.rand = orig_rand
        r.render_core = orig_core
    return out, captured["z_vals"]


def train_loss(out, rgb_gt, edge, smooth):
    rgb = out["color_fine"]
    loss = torch.sum(torch.abs(rgb - rgb_gt)) / float(rgb.shape[0])
    loss = loss + 0.1 * torch.mean((torch.linalg.norm(out["normals"].reshape(-1, 3), ord=2, dim=-1) - 1.0) ** 2)
    d = out["depth_pred"].view(-1, 4, 4, 1)
    img = rgb_gt.view(-1, 4, 4, 3)
    return loss + 1.0 * edge(d, img) + 1e-4 * smooth(d)


def make_losses():
    # restated from model/losses.py:7-38 (that file cannot be imported on a CPU-only torch:
    # it builds an SSIM module on CUDA at import, losses.py:72)
    l1 = lambda x: torch.mean(torch.abs(x))  # noqa: E731
    bw = lambda x: torch.exp(-torch.abs(x).sum(-1) / 0.1).unsqueeze(-1)  # noqa: E731

    def smooth(d):
        return (l1(d[:, :, :-1] - d[:, :, 1:]) + l1(d[:, :-1, :] - d[:, 1:, :]) + l1(d[:, :-1, :-1] - d[:, 1:, 1:]) +
                l1(d[:, 1:, :-1] - d[:, :-1, 1:])) / 4

    def edge(d, w):
        return (l1(bw(w[:, :, :-1] - w[:, :, 1:]) * (d[:, :, :-1] - d[:, :, 1:])) +
                l1(bw(w[:, :-1, :] - w[:, 1:, :]) * (d[:, :-1, :] - d[:, 1:, :])) +
                l1(bw(w[:, :-1, :-1] - w[:, 1:, 1:]) * (d[:, :-1, :-1] - d[:, 1:, 1:])) +
                l1(bw(w[:, 1:, :-1] - w[:, :-1, 1:]) * (d[:, 1:, :-1] - d[:, :-1, 1:]))) / 4
    return edge, smooth


def render_case(fields, rend, name, *, seed, R, dh_sdf, dh_col, eval_mode, car, full_grads, far=3.0):
    sdf, col, dev, r = build_nets(fields, rend, seed, dh_sdf, dh_col)
    rays_o, rays_d, norm = make_rays(R, seed + 1)
    g = torch.Generator().manual_seed(seed + 2)
    t_rand = torch.rand(R, REN_CFG["n_samples"], generator=g)
    rgb_gt = torch.rand(R, 3, generator=g)
    t = torch.tensor([0.25])
    near = torch.full((R, 1), 0.01)
    farr = torch.full((R, 1), far)
    out, z = run_render(r, rays_o, rays_d, norm, t, near, farr, t_rand, car, eval_mode)
    edge, smooth = make_losses()
    rec = {"rays_o": rays_o, "rays_d": rays_d, "rays_d_norm": norm, "t": t, "near": near, "far": farr,
           "t_rand": t_rand, "rgb_gt": rgb_gt, "car": np.float32(car), "eval": np.int32(eval_mode),
           "seed": np.int32(seed), "dh_sdf": np.int32(dh_sdf), "dh_col": np.int32(dh_col),
           "variance": dev.variance.detach(), "z_vals": z}
    for k in ("color_fine", "depth_pred", "weighted_z_vals", "weights", "sdf", "normals", "sdf_flows",
              "cdf_fine", "s_val", "sampled_points", "weight_sum", "weight_max"):
        rec["out_" + k] = out[k].detach()
    params = [("sdf." + k, p) for k, p in sdf.named_parameters()] + \
             [("col." + k, p) for k, p in col.named_parameters()] + [("dev.variance", dev.variance)]
    if not eval_mode:
        loss = train_loss(out, rgb_gt, edge, smooth)
        grads = torch.autograd.grad(loss, [p for _, p in params])
        rec["loss"] = loss.detach()
        gen = torch.Generator().manual_seed(1234)
        for (k, p), gr in zip(params, grads):
            put_grad(rec, k, gr, full_grads, gen)
    # parameters are rebuilt from the seed by the tests; checksums pin that
    for (k, p) in params:
        put_param(rec, k, p)
    np.savez_compressed(os.path.join(OUT, name + ".npz"),
                        **{k: (v.numpy() if torch.is_tensor(v) else v) for k, v in rec.items()})
    print("wrote", name, sorted(rec)[:6], "...")


def pretrained_case(fields, rend, name="render_pretrained", seed=690, R=256):
    """The reference's shipped pretrained SDF (pretrained_sdf/model.pt, loaded with
    weights_only=True) rendered from a camera at the origin looking down -z
    (near/far 0.01/5.0 as the Co3D config): a trained, non-spherical surface.
    The SDF weights travel in the fixture (sdfw.*) so the GPU test can load them."""
    sdf, col, dev, r = build_nets(fields, rend, seed)
    sd = torch.load(os.path.join(REF, "pretrained_sdf", "model.pt"), map_location="cpu", weights_only=True)
    sdf.load_state_dict(sd, strict=True)
    g = torch.Generator().manual_seed(seed + 1)
    d = torch.cat([(torch.rand(R, 2, generator=g) - 0.5) * 1.0, -torch.ones(R, 1)], -1)
    norm = d.norm(dim=-1, keepdim=True)
    rays_d = (d / norm).contiguous()
    rays_o = torch.zeros(R, 3)
    t_rand = torch.rand(R, REN_CFG["n_samples"], generator=g)
    rgb_gt = torch.rand(R, 3, generator=g)
    t = torch.tensor([0.0])
    near, far = torch.full((R, 1), 0.01), torch.full((R, 1), 5.0)
    out, z = run_render(r, rays_o, rays_d, norm, t, near, far, t_rand, 0.5, False)
    edge, smooth = make_losses()
    rec = {"rays_o": rays_o, "rays_d": rays_d, "rays_d_norm": norm, "t": t, "near": near, "far": far,
           "t_rand": t_rand, "rgb_gt": rgb_gt, "car": np.float32(0.5), "eval": np.int32(0),
           "seed": np.int32(seed), "dh_sdf": np.int32(256), "dh_col": np.int32(256),
           "variance": dev.variance.detach(), "z_vals": z}
    for k, v in sd.items():
        rec["sdfw." + k] = v.detach()
    for k in ("color_fine", "depth_pred", "weighted_z_vals", "weights", "sdf", "normals", "sdf_flows",
              "cdf_fine", "s_val", "sampled_points", "weight_sum", "weight_max"):
        rec["out_" + k] = out[k].detach()
    params = [("sdf." + k, p) for k, p in sdf.named_parameters()] + \
             [("col." + k, p) for k, p in col.named_parameters()] + [("dev.variance", dev.variance)]
    loss = train_loss(out, rgb_gt, edge, smooth)
    grads = torch.autograd.grad(loss, [p for _, p in params])
    rec["loss"] = loss.detach()
    gen = torch.Generator().manual_seed(1234)
    for (k, p), gr in zip(params, grads):
        put_grad(rec, k, gr, False, gen)
    np.savez_compressed(os.path.join(OUT, name + ".npz"),
                        **{k: (v.numpy() if torch.is_tensor(v) else v) for k, v in rec.items()})
    print("wrote", name)


def put_grad(rec, key, gr, full, gen):
    if full or gr.numel() <= 512:
        rec["grad." + key] = gr
    else:
        idx = torch.randperm(gr.numel(), generator=gen)[:256]
        rec["gradidx." + key] = idx.int()
        rec["gradval." + key] = gr.reshape(-1)[idx]
        rec["gradnorm." + key] = gr.norm()
        rec["gradsum." + key] = gr.sum()


def put_param(rec, key, p):
    rec["psum." + key] = p.detach().double().sum().float()
    rec["psq." + key] = (p.detach().double() ** 2).sum().float()


def seams_case(fields, rend):
    rec = {}
    # up_sample / sample_pdf seam (neus_renderer.py:178-224, 39-70)
    sdf, col, dev, r = build_nets(fields, rend, 7)
    g = torch.Generator().manual_seed(11)
    R = 32
    for n, inv_s in ((64, 64.0), (80, 128.0), (96, 256.0), (112, 512.0)):
        z = torch.sort(torch.rand(R, n, generator=g) * 2.9 + 0.05, -1)[0]
        sd = 0.6 - z + 0.2 * torch.sin(7 * z + torch.rand(R, 1, generator=g) * 6)  # crosses zero
        rays_o = torch.zeros(R, 3)
        rays_d = torch.tensor([[0.0, 0.0, -1.0]]).expand(R, 3)
        nz = r.up_sample(rays_o, rays_d, z, sd, 16, inv_s)
        zc, _ = r.cat_z_vals(rays_o, rays_d, torch.tensor([0.0]), z, nz, sd, last=True)
        rec[f"up{n}_z"], rec[f"up{n}_sdf"], rec[f"up{n}_new"], rec[f"up{n}_cat"] = z, sd, nz, zc
        rec[f"up{n}_invs"] = torch.tensor(inv_s)
    # SDF field seam at full width: sdf, feature, gradient and the create_graph double backward
    M = 256
    x = torch.cat([(torch.rand(M, 3, generator=g) - 0.5) * 1.6, torch.full((M, 1), 0.25)], -1)
    out = sdf(x)
    grad = sdf.gradient(x).squeeze(1)
    a = torch.randn(M, 1, generator=g)
    B = torch.randn(M, 256, generator=g) * 0.01
    C = torch.randn(M, 4, generator=g)
    L = (a * out[:, :1]).sum() + (B * out[:, 1:]).sum() + (C * grad).sum()
    params = list(sdf.named_parameters())
    grads = torch.autograd.grad(L, [p for _, p in params])
    rec.update({"mlp_x": x, "mlp_sdf": out[:, :1], "mlp_feat": out[:, 1:], "mlp_grad": grad, "mlp_a": a,
                "mlp_B": B, "mlp_C": C})
    gen = torch.Generator().manual_seed(99)
    for (k, p), gr in zip(params, grads):
        put_grad(rec, "mlp." + k, gr, False, gen)
        put_param(rec, "mlp." + k, p)
    # colour seam (neus_fields.py:346-374)
    Mc = 256
    pts = x[:Mc]
    dirs = torch.nn.functional.normalize(torch.randn(Mc, 3, generator=g), dim=-1)
    feat = torch.randn(Mc, 256, generator=g) * 0.3
    gg = torch.randn(Mc, 4, generator=g)
    rgb = col(pts, gg, dirs, feat)
    D = torch.randn(Mc, 3, generator=g)
    cparams = list(col.named_parameters())
    feat.requires_grad_(True)
    gg.requires_grad_(True)
    rgb2 = col(pts, gg, dirs, feat)
    Lc = (D * rgb2).sum()
    cg = torch.autograd.grad(Lc, [p for _, p in cparams] + [feat, gg])
    rec.update({"col_pts": pts, "col_dirs": dirs, "col_feat": feat.detach(), "col_g": gg.detach(), "col_rgb": rgb,
                "col_D": D, "col_dfeat": cg[-2], "col_dg": cg[-1]})
    for (k, p), gr in zip(cparams, cg[:-2]):
        put_grad(rec, "colnet." + k, gr, False, gen)
        put_param(rec, "colnet." + k, p)
    np.savez_compressed(os.path.join(OUT, "seams.npz"),
                        **{k: (v.detach().numpy() if torch.is_tensor(v) else v) for k, v in rec.items()})
    print("wrote seams")


MOTION_CFG = dict(d_out=6, d_in=1, d_hidden=256, n_layers=4, skip_in=[2], multires=6, bias=0.5, scale=1.0,
                  geometric_init=False, weight_norm=True)


def motion_case(fields):
    """MotionNetwork (neus_fields.py:79-190): seeded weights, forward, relative
    camera poses and world-to-camera chain, for the default config
    (default.yaml:113-123) and for geometric_init=True."""
    rec = {}
    for tag, gi in (("", False), ("geo.", True)):
        torch.manual_seed(681)
        m = fields.MotionNetwork(**dict(MOTION_CFG, geometric_init=gi))
        for k, v in m.state_dict().items():
            rec[tag + "sd." + k] = v.detach().numpy()
        t = torch.linspace(-1.0, 1.0, 9).view(-1, 1)
        w, v = m(t)
        rec[tag + "t"] = t.numpy()
        rec[tag + "omega"] = w.detach().numpy()
        rec[tag + "vel"] = v.detach().numpy()
        dt, rel = m.compute_relative_camera_pose(target_cam_idx=2, final_ref_cam_idx=5, total_nb_images=10,
                                                 nb_sample_timestep=10)
        rec[tag + "dt"] = np.float32(dt)
        rec[tag + "rel"] = torch.stack(rel).detach().numpy()
        rec[tag + "w2c"] = m.compute_w2c_mappings(rel).detach().numpy()
    np.savez_compressed(os.path.join(OUT, "motion.npz"), **rec)
    print("wrote motion")


def load_reference_trainer():
    """model/common.py and model/poses_retriever.py loaded by path, and the methods of
    model.training.Trainer that train.py calls per iteration (training.py:101-124,
    377-558) executed from the reference's own source text: training.py itself cannot
    be imported here (cv2 / imageio / torchvision are absent), so its
    class body is parsed and only the listed methods are compiled, unmodified, in a
    namespace holding the names they use (torch, np, F, the common.py functions)."""
    import ast
    load_reference()

    def load(modname, rel):
        spec = importlib.util.spec_from_file_location(modname, os.path.join(REF, rel))
        mod = importlib.util.module_from_spec(spec)
        sys.modules[modname] = mod
        spec.loader.exec_module(mod)
        return mod

    common = load("model.common", "model/common.py")
    poses = load("model.poses_retriever", "model/poses_retriever.py")
    src = open(os.path.join(REF, "model", "training.py")).read()
    tree = ast.parse(src)
    cls = next(n for n in tree.body if isinstance(n, ast.ClassDef) and n.name == "Trainer")
    keep = {"__init__", "near_far_from_sphere", "get_cos_anneal_ratio", "get_patch_indices", "process_data_dict",
            "process_data_reference", "process_data", "get_world_cameraOrigin_cameraRay", "compute_loss",
            "backpropagation", "anneal"}
    cls.body = [f for f in cls.body if isinstance(f, ast.FunctionDef) and f.name in keep]
    mod = ast.Module(body=[cls], type_ignores=[])
    ns = {"torch": torch, "np": np, "F": torch.nn.functional, "arange_pixels": common.arange_pixels,
          "origin_to_world": common.origin_to_world, "image_points_to_world": common.image_points_to_world,
          "transform_to_world": common.transform_to_world}
    exec(compile(mod, os.path.join(REF, "model", "training.py"), "exec"), ns)
    return common, poses, ns["Trainer"]


def trainer_case():
    """Rows a1-a5 of SURVEY.md §8 and the Trainer API from the reference's own code:
    arange_pixels, Exp / make_c2w, PoseRetriever (forward + gradients), the patch ids of
    a seeded get_patch_indices, process_data's rays for a posed camera, near / far,
    cos_anneal_ratio and compute_loss."""
    common, poses, RefTrainer = load_reference_trainer()
    rec = {}
    h, w = 12, 16
    p, pn = common.arange_pixels((h, w), 1)
    rec["arange_p"], rec["arange_pn"] = p, pn
    g = torch.Generator().manual_seed(31)
    rs = torch.cat([torch.zeros(1, 3), (torch.rand(4, 3, generator=g) - 0.5) * 0.6])
    ts = (torch.rand(5, 3, generator=g) - 0.5)
    rec["exp_r"], rec["exp_t"] = rs, ts
    rec["exp_R"] = torch.stack([common.Exp(r) for r in rs])
    rec["c2w"] = torch.stack([common.make_c2w(r, t) for r, t in zip(rs, ts)])
    pr = poses.PoseRetriever(5)
    with torch.no_grad():
        pr.r.copy_(rs)
        pr.t.copy_(ts)
    mats = torch.stack([pr(i) for i in range(5)])
    G = torch.randn(5, 4, 4, generator=g)
    gr, gt = torch.autograd.grad((mats * G).sum(), [pr.r, pr.t])
    rec.update({"pose_mats": mats.detach(), "pose_G": G, "pose_dr": gr, "pose_dt": gt})
    # the Trainer: cfg as default.yaml's training section (n_training_points = 64 here)
    cfg = dict(n_training_points=64, rgb_weight=[1.0, 1.0], eikonal_weight=[0.1, 0.1], sdf_weight=[0.1, 0.1],
               flow_rgb_weight=[7.5, 7.5], sdf_consistency_weight=[0.0, 1.0],
               edge_aware_smoothness_weight=[1.0, 0.0], smoothness_weight=[1e-4, 0.0])
    cfg_all = {"rendering": {"depth_range": [0.01, 5.0]}}
    tr = RefTrainer(None, None, None, cfg, device=torch.device("cpu"), total_nb_images=5, cfg_all=cfg_all,
                    logger=None, gt_depths=None, world_cam_idx=2, train_dataset=None)
    torch.manual_seed(5)
    rec["patch_idx"] = tr.get_patch_indices(h, w, 4, 64)
    rec["patch_seed"] = np.int32(5)
    img = torch.rand(1, 3, h, w, generator=g)
    fx = 0.9 * w
    K = torch.tensor([[[2 * fx / w, 0, 0, 0], [0, -2 * fx / h, 0, 0], [0, 0, -1, 0], [0, 0, 0, 1]]])
    scale = torch.eye(4)[None].clone()
    scale[0, 0, 0] = scale[0, 1, 1] = scale[0, 2, 2] = 1.25  # a non-trivial scale_mat
    data = {"img": img, "img.camera_mat": K, "img.scale_mat": scale, "img.idx": torch.tensor([3]),
            "img.ref_imgs": img.clone(), "img.ref_idxs": [torch.tensor([4])]}
    world_mat = pr(3).detach()
    torch.manual_seed(6)
    out = tr.process_data(data, world_mat, it=1, epoch=0, patch_size=4)
    names = ("img", "ref_img", "p", "pn", "rays_o", "rays_d", "rays_d_norm", "rgb_gt", "camera_mat", "scale_mat")
    for n, v in zip(names, out):
        rec["pd_" + n] = v
    rec["pd_seed"] = np.int32(6)
    rec["pd_world_mat"] = world_mat
    near, far = tr.near_far_from_sphere(out[4], out[5])
    rec["near"], rec["far"] = near, far
    rec["car_its"] = np.array([0, 1000, 25000, 50000, 80000], np.int64)
    rec["car"] = np.array([tr.get_cos_anneal_ratio(i, 50000) for i in rec["car_its"]], np.float64)
    # compute_loss on fixed terms
    rr = torch.rand(64, 3, generator=g)
    terms = torch.rand(6, generator=g)  # gradient, sdf, flow_rgb, sdf_consistency, edge-aware, smoothness
    d = tr.compute_loss(data, rr, out[7], *terms.unbind(0))
    rec["cl_rgb"], rec["cl_terms"] = rr, terms
    for k in ("loss", "loss_rgb", "l2_mean"):
        rec["cl_" + k] = d[k].detach()
    np.savez_compressed(os.path.join(OUT, "trainer.npz"),
                        **{k: (v.detach().numpy() if torch.is_tensor(v) else v) for k, v in rec.items()})
    print("wrote trainer")


def main():
    fields, rend = load_reference()
    motion_case(fields)
    trainer_case()
    torch.set_num_threads(8)
    render_case(fields, rend, "render_small_train", seed=678, R=16, dh_sdf=64, dh_col=64, eval_mode=False,
                car=0.5, full_grads=True)
    render_case(fields, rend, "render_small_eval", seed=679, R=16, dh_sdf=64, dh_col=64, eval_mode=True,
                car=1.0, full_grads=True)
    render_case(fields, rend, "render_full_train", seed=680, R=32, dh_sdf=256, dh_col=256, eval_mode=False,
                car=0.5, full_grads=False)
    seams_case(fields, rend)
    pretrained_case(fields, rend)


def main_motion_only():
    fields, _ = load_reference()
    motion_case(fields)


def main_pretrained_only():
    fields, rend = load_reference()
    torch.set_num_threads(8)
    pretrained_case(fields, rend)


if __name__ == "__main__":
    if "--trainer-only" in sys.argv:
        trainer_case()
    elif "--motion-only" in sys.argv:
        main_motion_only()
    elif "--pretrained-only" in sys.argv:
        main_pretrained_only()
    else:
        main()
