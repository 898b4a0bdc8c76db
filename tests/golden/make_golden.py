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

# The reference is untrusted public content: every source file this generator executes (imported
# module, or a block AST-extracted from train.py / training.py) is pinned by its sha256, and nothing
# runs if a file differs from the snapshot the fixtures were generated from.
PINNED = {
    "model/neus_embedder.py": "a949926f2c29c2ec1dd374505c2c994c1e822a60a6d6a165971a665bfe84739d",
    "utils_poses/pose_pytorch3d.py": "6026fda1c4defbf2603b1140ec7e8a93e9ed6fdc35187cafd72e5262a0874705",
    "model/neus_fields.py": "16292e97bde411fb7376294125ea03f31eee4fdc79145e9d0a63404ba75237c7",
    "model/neus_renderer.py": "6b0642436284c2a188b9ca52701af133711e543bbc2d2d354f802c2c8d7a9da8",
    "model/training.py": "3c99029d001d73e5864224b3a8bc6bec7ff90b9f7a3d401d5801ec799495319d",
    "train.py": "145aa03d8103d27fd00ba9e6255fa03b1d78313da3a88b671373e162acc16ab6",
    "model/checkpoints.py": "a0040bb837453b91baa4eb403962cfb1298130de463a6dbcebdb450483ad18fc",
    "model/poses_retriever.py": "92881188beb3d744e224de2ecb4f30654f0ebb4e5e8242930e197ef71be19392",
    "model/common.py": "09fc4fef0377091323e9a1a94e639ec434fed1df79af2f0befe2505f6131a656",
}


def _ref_text(rel):
    """The text of a pinned reference source file (refuses a file whose hash differs)."""
    import hashlib
    path = os.path.join(REF, rel)
    data = open(path, "rb").read()
    got = hashlib.sha256(data).hexdigest()
    if PINNED.get(rel) != got:
        raise RuntimeError(f"{path}: sha256 {got} is not the pinned one; refusing to execute it")
    return data.decode()


def _ref_path(rel):
    _ref_text(rel)
    return os.path.join(REF, rel)

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
        spec = importlib.util.spec_from_file_location(modname, _ref_path(rel))
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
        spec = importlib.util.spec_from_file_location(modname, _ref_path(rel))
        mod = importlib.util.module_from_spec(spec)
        sys.modules[modname] = mod
        spec.loader.exec_module(mod)
        return mod

    common = load("model.common", "model/common.py")
    poses = load("model.poses_retriever", "model/poses_retriever.py")
    src = _ref_text("model/training.py")
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


def load_reference_stage1_block():
    """The stage-1 loss block of the reference's training loop (train.py:467-517: the
    `if not self.query_in_canonical_space:` statement inside Trainer.train) and
    Trainer.warp_pixel (train.py:235-244), parsed from train.py's own source text and
    compiled unmodified: train.py cannot be imported here (tensorboardX, dataloading,
    cv2 are absent).  The block runs as the body of a function whose locals are the
    training loop's variables it reads; the stub `self` carries the attributes it uses.
    `pts_map` is one of them: a frame without a valid reference frame (the last one) never
    assigns it in the block, and train.py:504 then takes only its shape from the previous
    iteration's value (a loop local of Trainer.train); the first iteration on such a frame
    would raise UnboundLocalError."""
    import ast
    src = _ref_text("train.py")
    tree = ast.parse(src)
    cls = next(n for n in tree.body if isinstance(n, ast.ClassDef) and n.name == "Trainer")
    warp = next(f for f in cls.body if isinstance(f, ast.FunctionDef) and f.name == "warp_pixel")
    train_fn = next(f for f in cls.body if isinstance(f, ast.FunctionDef) and f.name == "train")
    block = next(n for n in ast.walk(train_fn) if isinstance(n, ast.If) and isinstance(n.test, ast.UnaryOp)
                 and isinstance(n.test.op, ast.Not) and ast.unparse(n.test.operand) == "self.query_in_canonical_space")
    names = ["self", "render_out", "query_time_step", "image_idx", "ref_image_idx_list", "nb_valid_next_time_step",
             "ref_camera_mat_list", "scale_mat", "normalized_sampled_pixel", "img", "rgb_pred", "sampled_pixel",
             "rgb_gt", "ref_image_list", "sdf", "flow_loss", "flow_rgb_loss", "sdf_consistency_loss", "sdf_loss",
             "pts_map"]
    ret = ast.parse("return sdf_loss, flow_rgb_loss, sdf_consistency_loss").body
    fn = ast.FunctionDef(name="stage1_block", args=ast.arguments(
        posonlyargs=[], args=[ast.arg(arg=n) for n in names], kwonlyargs=[], kw_defaults=[], defaults=[]),
        body=[block] + ret, decorator_list=[], returns=None, type_params=[])
    mod = ast.fix_missing_locations(ast.Module(body=[warp, fn], type_ignores=[]))
    ns = {"torch": torch, "np": np}
    exec(compile(mod, os.path.join(REF, "train.py"), "exec"), ns)
    return ns["warp_pixel"], ns["stage1_block"]


STAGE1_CASES = (  # (tag, image_idx, random_ref_interval, sdf_consistency_enable_pose_grad)
    ("before", 2, (1, 2, 3), False), ("world", 4, (1, 2, 3), False), ("after", 6, (1, 2, 3), False),
    ("last", 7, (1, 2, 3), False), ("iv1510", 2, (1, 5, 10), False), ("posegrad_before", 2, (1, 2, 3), True),
    ("posegrad_after", 6, (1, 5, 10), True))


def stage1_case(fields):
    """Rows a22 / (f)1 of SURVEY.md §8: sdf_loss, flow_rgb_loss and sdf_consistency_loss
    of one stage-1 iteration, and their gradients, from the reference's own code
    (load_reference_stage1_block) for frames before / at / after the world camera (n = 8,
    world 4) and the last frame, ref intervals (1, 2, 3) and (1, 5, 10), with and without
    sdf_consistency_enable_pose_grad.  The renderer outputs the block reads are inputs
    here (rays through 4x4-patch pixels of a 24x32 frame, points at depth 0.8..1.6, random
    weights / normals / sdf flows; the renderer itself is pinned by the render_* fixtures):
    gradients are taken with respect to them, the motion network and the SDF network."""
    warp_pixel, block = load_reference_stage1_block()
    import types as _t
    n_images, world, H, W, R, S = 8, 4, 24, 32, 32, 8
    rec = {"n_images": np.int32(n_images), "world": np.int32(world), "H": np.int32(H), "W": np.int32(W)}
    torch.manual_seed(681)
    motion = fields.MotionNetwork(**MOTION_CFG)
    with torch.no_grad():  # non-trivial velocities
        g = torch.Generator().manual_seed(682)
        for p in motion.parameters():
            p.add_(0.05 * torch.randn(p.shape, generator=g))
    torch.manual_seed(683)
    sdf_net = fields.SDFNetwork(**dict(SDF_CFG, d_hidden=64))
    for k, v in motion.state_dict().items():
        rec["motion." + k] = v.detach()
    for k, v in sdf_net.state_dict().items():
        rec["sdfnet." + k] = v.detach()
    g = torch.Generator().manual_seed(684)
    fx = 0.9 * W
    K = torch.tensor([[2 * fx / W, 0, 0, 0], [0, -2 * fx / H, 0, 0], [0, 0, -1, 0], [0, 0, 0, 1.0]])
    frames = torch.rand(n_images, 3, H, W, generator=g) * 0.8 + 0.1
    rec["K"], rec["frames"] = K, frames
    for tag, image, intervals, pose_grad in STAGE1_CASES:
        # pixels of R/16 4x4 patches; rays through them from the origin (world_mat = I in stage 1)
        corner = torch.stack([torch.randint(0, W - 4, (R // 16,), generator=g),
                              torch.randint(0, H - 4, (R // 16,), generator=g)], -1)
        off = torch.stack(torch.meshgrid(torch.arange(4), torch.arange(4), indexing="xy"), -1).reshape(16, 2)
        pix = (corner[:, None, :] + off[None]).reshape(R, 2).float()
        pixn = torch.stack([pix[:, 0] / (W - 1) * 2 - 1, pix[:, 1] / (H - 1) * 2 - 1], -1)
        d = torch.stack([pixn[:, 0] / K[0, 0], pixn[:, 1] / K[1, 1], -torch.ones(R)], -1)
        z = 0.8 + 0.8 * torch.rand(R, S, generator=g)
        pts = (d[:, None, :] * z[..., None]).reshape(R, S, 3)
        wts = torch.rand(R, S, generator=g)
        wts = wts / wts.sum(-1, keepdim=True) * 0.9
        leaves = {"sampled_points": pts, "weights": wts,
                  "normals": torch.nn.functional.normalize(torch.randn(R * S, 3, generator=g), dim=-1),
                  "sdf_flows": 0.1 * torch.randn(R * S, 1, generator=g),
                  "sdf": 0.05 * torch.randn(R * S, 1, generator=g)}
        leaves = {k: v.clone().requires_grad_(k != "sampled_points") for k, v in leaves.items()}
        render_out = dict(leaves)
        refs = [image + j for j in intervals]
        ref_imgs = [torch.ones(1, 3, H, W) * 10e5 if r >= n_images else frames[r][None] for r in refs]  # dataset.py:243
        ref_K = [torch.ones(1, 4, 4) * 10e5 if r >= n_images else K[None] for r in refs]               # dataset.py:289
        ref_idx = torch.tensor(refs)
        nxt = ref_idx / (n_images - 1) * 2 - 1
        nb_valid = len(nxt[nxt <= 1.0])
        t = image / (n_images - 1) * 2 - 1
        cfg = {"training": {"flow_rgb_weight": [7.5, 7.5], "sdf_consistency_weight": [0.0, 1.0],
                            "sdf_consistency_enable_pose_grad": pose_grad}}
        self_ = _t.SimpleNamespace(device=torch.device("cpu"), motion_network=motion, cfg=cfg, total_nb_images=n_images,
                                   query_in_canonical_space=False,
                                   nb_sample_timestep=10, world_cam_idx=world, sdf_network=sdf_net,
                                   world_time_step=world / (n_images - 1) * 2 - 1)
        self_.warp_pixel = lambda src_frame, uv, normalize_pix=True, _s=self_: warp_pixel(_s, src_frame, uv, normalize_pix)
        zero = lambda: torch.tensor(0.0)  # noqa: E731
        rgb_gt = torch.rand(R, 3, generator=g)
        l_sdf, l_flow, l_cons = block(self_, render_out, torch.tensor([t]).float(), torch.tensor([image]), ref_idx,
                                      nb_valid, torch.cat(ref_K), torch.eye(4)[None], pixn, torch.zeros(1, 3, H, W),
                                      torch.zeros(R, 3), pix, rgb_gt, torch.cat(ref_imgs), leaves["sdf"], zero(), zero(),
                                      zero(), zero(), torch.zeros(R * S, 3))
        total = 0.1 * l_sdf + 7.5 * l_flow + 0.3 * l_cons
        wrt = ([("out." + k, v) for k, v in leaves.items() if v.requires_grad] +
               [("motion." + k, p) for k, p in motion.named_parameters()] +
               [("sdfnet." + k, p) for k, p in sdf_net.named_parameters()])
        grads = torch.autograd.grad(total, [v for _, v in wrt], allow_unused=True)
        c = f"{tag}."
        rec.update({c + "image": np.int32(image), c + "intervals": np.array(intervals, np.int32),
                    c + "pose_grad": np.int32(pose_grad), c + "pix": pix, c + "pixn": pixn, c + "rgb_gt": rgb_gt,
                    c + "sdf_loss": l_sdf.detach(), c + "flow_rgb_loss": l_flow.detach(),
                    c + "sdf_consistency_loss": torch.as_tensor(l_cons).detach()})
        for k, v in leaves.items():
            rec[c + "in." + k] = v.detach()
        gen = torch.Generator().manual_seed(685)
        for (k, _), gr in zip(wrt, grads):
            if gr is None:
                rec["grad." + c + k] = torch.zeros(0)
            else:  # large motion-network gradients: 256 sampled entries + norm + sum
                put_grad(rec, c + k, gr, k.startswith("out."), gen)
        print(f"stage1 {tag}: sdf {l_sdf.item():.6f} flow {l_flow.item():.6f} cons {float(l_cons):.6f}")
    np.savez_compressed(os.path.join(OUT, "stage1.npz"),
                        **{k: (v.detach().numpy() if torch.is_tensor(v) else v) for k, v in rec.items()})
    print("wrote stage1")


def checkpoint_case(fields, rend):
    """what train.py checkpoints.  train.py:47-54 builds
    DataParallel(NeuSRenderer(None, sdf, dev, col, motion)) and train.py:94 registers it
    with the reference's CheckpointIO as `model`, beside the two Adam optimizers
    (train.py:58-59); save_checkpoint (train.py:158-167) adds epoch_it / it /
    depth_range.  Recorded: the module.-prefixed state-dict keys and shapes at the
    default.yaml widths (state_keys.json), and a checkpoint file written by the
    reference's own CheckpointIO (model/checkpoints.py) at 64-wide networks after one
    Adam step of each optimizer (ref_checkpoint.pt: tensors, ints and floats only, so
    torch.load(weights_only=True) reads it)."""
    import json
    import tempfile
    ckio = importlib.util.spec_from_file_location("model.checkpoints", _ref_path("model/checkpoints.py"))
    ckmod = importlib.util.module_from_spec(ckio)
    ckio.loader.exec_module(ckmod)

    def build(width):
        torch.manual_seed(700)
        sdf = fields.SDFNetwork(**dict(SDF_CFG, d_hidden=width))
        col = fields.RenderingNetwork(**dict(COL_CFG, d_hidden=width, d_feature=width))
        dev = fields.SingleVarianceNetwork(0.3)
        motion = fields.MotionNetwork(**dict(MOTION_CFG, d_hidden=width))
        r = rend.NeuSRenderer(None, sdf, dev, col, motion, **REN_CFG)
        return torch.nn.DataParallel(r), sdf, dev, col, motion

    dp, *_ = build(256)
    keys = {k: list(v.shape) for k, v in dp.state_dict().items()}
    json.dump({"source": "DataParallel(NeuSRenderer) of train.py:47-54 at default.yaml widths", "keys": keys},
              open(os.path.join(OUT, "state_keys.json"), "w"), indent=0)
    dp, sdf, dev, col, motion = build(64)
    opt = torch.optim.Adam(list(sdf.parameters()) + list(dev.parameters()) + list(col.parameters()), lr=1e-3)
    mopt = torch.optim.Adam(motion.parameters(), lr=5e-4)
    g = torch.Generator().manual_seed(701)
    for o, mods in ((opt, (sdf, dev, col)), (mopt, (motion,))):
        for m in mods:
            for p in m.parameters():
                p.grad = torch.randn(p.shape, generator=g) * 0.01
        o.step()
    with tempfile.TemporaryDirectory() as d:
        io = ckmod.CheckpointIO(d, model=dp, optimizer=opt, motion_optimizer=mopt)
        io.save("model.pt", lastest_checkpoint=True, epoch_it=12, it=3456, depth_range=[0.01, 5.0])
        raw = open(os.path.join(d, "models", "weights", "model.pt"), "rb").read()
    open(os.path.join(OUT, "ref_checkpoint.pt"), "wb").write(raw)
    print("wrote state_keys.json, ref_checkpoint.pt", len(keys), "keys,", len(raw), "bytes")


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
    stage1_case(fields)
    checkpoint_case(fields, rend)


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
    elif "--stage1-only" in sys.argv:
        stage1_case(load_reference()[0])
    elif "--checkpoint-only" in sys.argv:
        checkpoint_case(*load_reference())
    elif "--motion-only" in sys.argv:
        main_motion_only()
    elif "--pretrained-only" in sys.argv:
        main_pretrained_only()
    else:
        main()
