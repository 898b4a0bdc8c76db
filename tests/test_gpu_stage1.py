"""The training step of copenerf.train_step.SyntheticTrainer against the CPU oracle's
restatement (oracle.stage1_losses is pinned to the reference's own stage-1 block by
tests/test_stage1_golden.py) on identical sample positions, in three workloads:
  stage1     the MotionNetwork losses of train.py:467-517 (scene-flow SDF loss, flow-RGB
             warp, SDF consistency at the world camera) with the Co3D configs' options:
             sdf_consistency_enable_pose_grad (the consistency term reaches the motion
             network) and random_ref_interval [1, 5, 10];
  canonical  query in canonical space with learnable SE(3) poses (train.py:425-431,
             config C3's joint pose optimisation: ray gradients into r, t);
  hybrid     both at once (not a reference workload: the reference applies the stage-1
             losses only outside canonical space; kept as the widest coverage of the
             backward: pose, motion and field gradients in one step);
for frames before, at and after the world camera and the last frame (no valid reference
frame).  Gradients of the poses, the motion network and the fields are compared in every
GEMM mode: fp32 and bf16x6 at 2e-3 of the gradient scale (fields) and 5e-3 (poses /
motion); bf16 (config C3, operands rounded to 8 bits) as the relative L2 error of each
gradient tensor at about twice the error measured on the GPU (COPENERF_PARITY_LOG
collects the measured values)."""
import json
import os

import pytest
import torch

from helpers import oracle_params, smooth_frames
from oracle import neus_oracle as O

pytestmark = pytest.mark.gpu
DEV = "cuda"
N_IMAGES = 8  # world camera n // 2 = 4 (world_idx 'mid', train.py:85)
R, H, W = 128, 48, 64
# (loss rel., fields, poses / motion): fp32 modes: max |Δ| over the gradient's max |g|;
# bf16 (operands rounded to 8 bits): relative L2 error of each gradient tensor
# bf16 at about twice the largest error measured over these cases on an MI355X
# (profiles/r3_stage1_parity.jsonl: loss 8.2e-4, fields 6.6e-2, pose / motion 4.9e-2)
BARS = {"fp32": (1e-4, 2e-3, 5e-3), "bf16x6": (1e-4, 2e-3, 5e-3), "bf16": (2e-3, 1.3e-1, 1e-1)}
SCEN = {"hybrid": (True, True, {}),
        "stage1": (False, True, {"sdf_consistency_enable_pose_grad": True, "random_ref_interval": (1, 5, 10)}),
        "canonical": (True, False, {})}
CASES = ([("hybrid", i, m, R) for i in (2, 4, 6, 7) for m in ("fp32", "bf16x6", "bf16")] +
         [("stage1", i, m, R) for i in (2, 6, 7) for m in ("bf16x6", "bf16")] +
         [("canonical", i, m, R) for i in (2, 5) for m in ("bf16x6", "bf16")] +
         [("canonical", 2, "bf16", 1024)])  # the shipped n_training_points (default.yaml)


def _trainer(mode, start_it, joint_pose=True, stage1=True, train_cfg=None, rays=R):
    from copenerf.train_step import SyntheticTrainer
    tr = SyntheticTrainer(DEV, rays=rays, H=H, W=W, seed=11, joint_pose=joint_pose, stage1=stage1, n_images=N_IMAGES,
                          start_it=start_it, schedule="reference", mfma_dtype=mode, depth_range=(0.01, 3.0),
                          train_cfg=train_cfg)
    tr.images = smooth_frames(N_IMAGES, H, W, DEV)  # see smooth_frames: a well-conditioned flow-RGB gradient
    return tr


def _cpu_copy(mod, cls_args):
    m = type(mod)(**cls_args)
    m.load_state_dict({k: v.detach().cpu() for k, v in mod.state_dict().items()})
    return m


def _err(got, ref, name, l2=False):
    assert got is not None, name
    got = got.detach().cpu()
    if l2:
        return (got - ref).norm().item() / (ref.norm().item() + 1e-12)
    return (got - ref).abs().max().item() / (ref.abs().max().item() + 1e-12)


@pytest.mark.parametrize("scenario,image,mode,rays", CASES)
def test_training_step_matches_oracle(scenario, image, mode, rays):
    errs = _step_errors(scenario, image, mode, rays)
    l_bar, f_bar, pm_bar = BARS[mode]
    worst_f = max(v for k, v in errs.items() if k.startswith(("sdf.", "col.", "dev.")))
    worst_pm = max([v for k, v in errs.items() if k.startswith(("pose", "motion"))] or [0.0])
    logp = os.environ.get("COPENERF_PARITY_LOG")
    if logp:
        with open(logp, "a") as f:
            f.write(json.dumps({"scenario": scenario, "image": image, "mode": mode, "rays": rays,
                                "loss": errs["loss"], "fields": worst_f, "pose_motion": worst_pm,
                                "worst_field": max((k for k in errs if k.startswith(("sdf.", "col.", "dev."))),
                                                   key=errs.get)}) + "\n")
    assert errs["loss"] <= l_bar + errs["_loss_abs_slack"], errs["loss"]
    for k, e in errs.items():
        if k not in ("loss", "_loss_abs_slack"):
            assert e <= (pm_bar if k.startswith(("pose", "motion")) else f_bar), (k, e)


def _step_errors(scenario, image, mode, rays):
    """The HIP training step against the oracle on identical samples: the loss's relative error and
    each gradient's error (fp32 modes: max |Δ| over max |g|; bf16: relative L2)."""
    from copenerf.rays import PoseRetriever, world_rays
    from copenerf.train_step import MOTION_CFG
    joint_pose, stage1, tcfg = SCEN[scenario]
    # iteration it uses frame (it - 1) % n; it ~ 30000: cos_anneal_ratio 0.6, consistency weight 0.3
    start = 30000 + (image - 30000 % N_IMAGES) % N_IMAGES
    tr = _trainer(mode, start, joint_pose, stage1, tcfg, rays)
    tr.begin_iteration()
    it, img = tr.it, tr.image_index(tr.it)
    assert img == image
    batch = tr.make_batch()
    # ---- oracle (CPU) on the same pixels, poses, weights and sample positions
    P, Pc, var, leaves = oracle_params(tr.sdf, tr.col, tr.var)
    pixn, pix = batch["pixn"].cpu(), batch["pix"].cpu()
    K = tr.K.cpu()
    pose_leaves, motion_c = [], None
    world_mat = torch.eye(4)
    if joint_pose:
        poses_c = PoseRetriever(N_IMAGES)
        poses_c.load_state_dict({k: v.detach().cpu() for k, v in tr.poses.state_dict().items()})
        pose_leaves = [poses_c.r, poses_c.t]
        if img != tr.world_cam_idx:
            world_mat = poses_c(img)
    if stage1:
        motion_c = _cpu_copy(tr.motion, MOTION_CFG)
    o, d, n = world_rays(pixn, K, world_mat, torch.eye(4))
    # train.py:440: the frame's time in stage 1, the world camera's time in canonical space
    t = torch.tensor([(img if stage1 else tr.world_cam_idx) / (N_IMAGES - 1) * 2 - 1])
    near, far = torch.full((rays, 1), 0.01), torch.full((rays, 1), 3.0)
    t_rand = torch.rand(rays, 64, generator=torch.Generator().manual_seed(img))
    torch.set_num_threads(8)
    z = O.hierarchical_z(P, o.detach(), d.detach(), t, near, far, 64, 64, 4, t_rand)
    v = tr.sched.values(it, img)
    car = v["car"]
    ref = O.render_core(P, Pc, var, o, d, n, t, z, (far[0, 0] - near[0, 0]) / 64, car)
    rgb_gt = batch["rgb_gt"].cpu()
    lw, sw = v["loss_w"], v["stage1_w"]
    loss_ref = O.train_loss(ref, rgb_gt, w_rgb=lw[0], w_eik=lw[1], w_edge=lw[2], w_smooth=lw[3])
    if stage1:
        l_sdf, l_flow, l_cons = O.stage1_losses(
            ref, motion_c, lambda x: O.sdf_mlp(P, x)[:, :1], image_idx=img, n_images=N_IMAGES,
            world_cam_idx=tr.world_cam_idx, nb_sample_timestep=10, rgb_gt=rgb_gt, sampled_pixel=pix,
            normalized_pixel=pixn, camera_mats=tr.camera_mats.cpu(), ref_images=tr.images.cpu(),
            scale_mat=torch.eye(4)[None], img_hw=(H, W), ref_intervals=tr.cfg["random_ref_interval"],
            consistency_pose_grad=tr.cfg["sdf_consistency_enable_pose_grad"])
        loss_ref = loss_ref + sw[0] * l_sdf + sw[1] * l_flow + sw[2] * l_cons
    motion_leaves = list(motion_c.parameters()) if stage1 else []
    ref_leaves = pose_leaves + motion_leaves + list(leaves.values())
    gref = torch.autograd.grad(loss_ref, ref_leaves, allow_unused=True)
    # ---- HIP path: the trainer's own iteration with the oracle's sample positions
    loss = tr.iteration(batch, z_vals=z.to(DEV))
    l2 = mode == "bf16"
    errs = {"loss": abs(loss.item() - loss_ref.item()) / abs(loss_ref.item())}
    np_ = len(pose_leaves)
    if joint_pose and img != tr.world_cam_idx:  # the world camera's rays use the identity: no pose gradient
        errs["pose r"] = _err(tr.poses.r.grad[img], gref[0][img], "pose r", l2)
        errs["pose t"] = _err(tr.poses.t.grad[img], gref[1][img], "pose t", l2)
    if stage1:
        for (name, p), gr in zip(tr.motion.named_parameters(), gref[np_:np_ + len(motion_leaves)]):
            if gr is None:
                assert p.grad is None or not p.grad.any(), name
                continue
            errs["motion." + name] = _err(p.grad, gr, "motion." + name, l2)
    keys = list(leaves)
    fields = ([("sdf." + k, p) for k, p in tr.sdf.named_parameters()] +
              [("col." + k, p) for k, p in tr.col.named_parameters()] + [("dev.variance", tr.var.variance)])
    off = np_ + len(motion_leaves)
    for name, p in fields:
        errs[name] = _err(p.grad, gref[off + keys.index(name)], name, l2)
    errs["_loss_abs_slack"] = 1e-6 / abs(loss_ref.item())
    return errs


def test_stage1_terms_are_masked_not_branched():
    """Frame = world camera: the SDF-consistency term is zero (train.py:497), and the
    last frame has no valid reference frame: flow-RGB is zero (train.py:421, 506)."""
    tr = _trainer("bf16x6", 30000 + (7 - 30000 % N_IMAGES) % N_IMAGES)
    tr.begin_iteration()
    assert tr.image_index(tr.it) == 7
    batch = tr.make_batch()
    out = tr.renderer(batch["rays_o"], batch["rays_d"], batch["norm"], tr.query_time(),
                      torch.full((R, 1), 0.01, device=DEV), torch.full((R, 1), 3.0, device=DEV),
                      cos_anneal_ratio=tr.sched.car, it=tr.it)
    _, l_flow, l_cons = tr.stage1_terms(out, batch)
    assert l_flow.item() == 0.0 and l_cons.item() > 0
    tr.sched.set(tr.it, tr.world_cam_idx)
    _, l_flow, l_cons = tr.stage1_terms(out, batch)
    assert l_cons.item() == 0.0 and l_flow.item() > 0


@pytest.mark.parametrize("joint_pose,stage1", [(True, False), (False, True), (True, True)])
def test_synthetic_trainer_modes_step(joint_pose, stage1):
    """The C3-style training step runs and updates the poses / motion network."""
    from copenerf.train_step import SyntheticTrainer
    tr = SyntheticTrainer(DEV, rays=1024, joint_pose=joint_pose, stage1=stage1, schedule="reference",
                          start_it=30000, mfma_dtype="bf16")
    r0 = tr.poses.r.detach().clone() if joint_pose else None
    m0 = tr.motion.lin0.bias.detach().clone() if stage1 else None
    for _ in range(3):
        loss = tr.step()
    assert torch.isfinite(loss).item()
    tr.check_finite()
    if joint_pose:
        assert not torch.equal(tr.poses.r.detach(), r0)
    if stage1:
        assert not torch.equal(tr.motion.lin0.bias.detach(), m0)
    for p in tr.all_params:
        assert torch.isfinite(p).all()


def test_euler_chain_kernel_matches_torch_recurrence():
    """cn_euler_chain / _bwd (all K relative poses, neus_fields.py:146-165) against the
    torch recurrence of MotionNetwork.batched_relative_poses on the CPU: poses and the
    motion network's parameter gradients."""
    from copenerf.motion import MotionNetwork
    from copenerf.train_step import MOTION_CFG
    torch.manual_seed(5)
    m = MotionNetwork(**MOTION_CFG)
    with torch.no_grad():  # non-trivial velocities
        for p in m.parameters():
            p.add_(0.05 * torch.randn_like(p))
    mc = MotionNetwork(**MOTION_CFG).to(DEV)
    mc.load_state_dict({k: v.to(DEV) for k, v in m.state_dict().items()})
    steps, dts = m.interval_time_grid(10, 10)
    P_ref = m.batched_relative_poses(steps, dts)
    P = mc.batched_relative_poses(steps.to(DEV), dts.to(DEV))
    torch.testing.assert_close(P.cpu(), P_ref, rtol=1e-5, atol=2e-6)
    G = torch.randn(P_ref.shape, generator=torch.Generator().manual_seed(6))
    g_ref = torch.autograd.grad((P_ref * G).sum(), list(m.parameters()))
    g = torch.autograd.grad((P * G.to(DEV)).sum(), list(mc.parameters()))
    for a, b in zip(g, g_ref):
        assert _err(a, b, "motion grad") <= 1e-4


def _rounded(t):
    return t.bfloat16().float() if (t is not None and t.dtype == torch.float32) else t


@pytest.mark.parametrize("variant", ["images", "fp32_operands", "sigma_bf16", "second_order_bf16", "bias_sum_bf16"])
def test_bf16_image_error_sources(variant, monkeypatch):
    """Where the bf16 mode's operand images (round 4) add error, on the stage-1 case
    with the largest field error (frame 6): the image path, the same step with fp32 operands rounded
    on load (round 3's numerics: _img_mode off), and that step with ONE of the images' roundings put
    back -- σ recovered from the rounded activation (MUL / TANGENT / BWD_SOFTPLUS aux0), the
    second-order term's s and u̇ rounded (BWD_SOFTPLUS / the elementwise last adjoint's aux1, aux2),
    or the weight gradients' bias sums over rounded adjoints (Y0).  Each within the bf16 bars; the
    measured errors go to COPENERF_PARITY_LOG (profiles/r5_bf16_sources.jsonl)."""
    from copenerf import fields, ops
    if variant != "images":
        monkeypatch.setattr(fields, "_img_mode", lambda pk, lay: False)
    lin, adj, wq_add = ops.linear, ops.softplus_adjoint, ops.WgradQueue.add
    if variant == "sigma_bf16":
        def linear(*a, **kw):
            if a[5] in (ops.EPI_MUL, ops.EPI_TANGENT, ops.EPI_BWD_SOFTPLUS) and kw.get("aux_beta", 0.0):
                kw["aux0"] = _rounded(kw.get("aux0"))
            return lin(*a, **kw)
        monkeypatch.setattr(ops, "linear", linear)
    elif variant == "second_order_bf16":
        def linear(*a, **kw):
            if a[5] == ops.EPI_BWD_SOFTPLUS:
                kw["aux1"], kw["aux2"] = _rounded(kw.get("aux1")), _rounded(kw.get("aux2"))
            return lin(*a, **kw)

        def softplus_adjoint(*a, **kw):
            kw["aux1"], kw["aux2"] = _rounded(kw.get("aux1")), _rounded(kw.get("aux2"))
            return adj(*a, **kw)
        monkeypatch.setattr(ops, "linear", linear)
        monkeypatch.setattr(ops, "softplus_adjoint", softplus_adjoint)
    elif variant == "bias_sum_bf16":
        def add(self, Y0, X0, *a, **kw):
            return wq_add(self, _rounded(Y0), X0, *a, **kw)
        monkeypatch.setattr(ops.WgradQueue, "add", add)
    errs = _step_errors("stage1", 6, "bf16", R)
    fk = sorted((k for k in errs if k.startswith(("sdf.", "col.", "dev."))), key=errs.get, reverse=True)
    worst_pm = max([v for k, v in errs.items() if k.startswith(("pose", "motion"))] or [0.0])
    rec = {"variant": variant, "loss": errs["loss"], "fields": errs[fk[0]], "pose_motion": worst_pm,
           "top_fields": {k: round(errs[k], 5) for k in fk[:4]}}
    print(rec)
    logp = os.environ.get("COPENERF_PARITY_LOG")
    if logp:
        with open(logp, "a") as f:
            f.write(json.dumps(rec) + "\n")
    l_bar, f_bar, pm_bar = BARS["bf16"]
    assert errs["loss"] <= l_bar and errs[fk[0]] <= f_bar and worst_pm <= pm_bar, rec
