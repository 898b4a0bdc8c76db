"""The Trainer drop-in (copenerf.trainer, exported as model.Trainer) and the ray
generation of SURVEY.md §8 rows a1-a5 against fixtures produced by the
reference's own code (tests/golden/make_golden.py trainer_case: model/common.py,
model/poses_retriever.py and the Trainer methods of model/training.py)."""
import os
import sys

import pytest
import torch

from helpers import fixture

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def fx():
    return fixture("trainer")


def _trainer(device="cpu", **kw):
    sys.path.insert(0, os.path.join(ROOT, "cope-nerf_amd"))
    from model import Trainer  # the drop-in import train.py uses (train.py:102: mdl.Trainer)
    cfg = dict(n_training_points=64, rgb_weight=[1.0, 1.0], eikonal_weight=[0.1, 0.1], sdf_weight=[0.1, 0.1],
               flow_rgb_weight=[7.5, 7.5], sdf_consistency_weight=[0.0, 1.0],
               edge_aware_smoothness_weight=[1.0, 0.0], smoothness_weight=[1e-4, 0.0])
    return Trainer(None, None, None, cfg, device=torch.device(device), total_nb_images=5,
                   cfg_all={"rendering": {"depth_range": [0.01, 5.0]}}, logger=None, gt_depths=None, world_cam_idx=2,
                   train_dataset=None, **kw)


def test_arange_pixels_rows(fx):
    from copenerf.rays import pixels_from_indices
    h, w = 12, 16
    p, pn = pixels_from_indices(torch.arange(h * w), h, w)
    assert torch.equal(p, fx["arange_p"][0])
    assert torch.equal(pn, fx["arange_pn"][0])


def test_exp_make_c2w_pose_retriever(fx):
    from copenerf.rays import Exp, PoseRetriever, make_c2w
    for i in range(fx["exp_r"].shape[0]):
        torch.testing.assert_close(Exp(fx["exp_r"][i]), fx["exp_R"][i], rtol=0, atol=1e-7)
        torch.testing.assert_close(make_c2w(fx["exp_r"][i], fx["exp_t"][i]), fx["c2w"][i], rtol=0, atol=1e-7)
    pr = PoseRetriever(5)
    with torch.no_grad():
        pr.r.copy_(fx["exp_r"])
        pr.t.copy_(fx["exp_t"])
    mats = torch.stack([pr(i) for i in range(5)])
    torch.testing.assert_close(mats.detach(), fx["pose_mats"], rtol=0, atol=1e-7)
    gr, gt = torch.autograd.grad((mats * fx["pose_G"]).sum(), [pr.r, pr.t])
    torch.testing.assert_close(gr, fx["pose_dr"], rtol=1e-6, atol=1e-6)
    torch.testing.assert_close(gt, fx["pose_dt"], rtol=1e-6, atol=1e-6)
    # the device-index form (graph-capturable) is the same arithmetic
    for i in range(5):
        torch.testing.assert_close(pr.pose_at(torch.tensor([i])).detach(), fx["pose_mats"][i], rtol=0, atol=1e-7)


def test_patch_indices_follow_the_reference_rng(fx):
    tr = _trainer()
    torch.manual_seed(int(fx["patch_seed"]))
    assert torch.equal(tr.get_patch_indices(12, 16, 4, 64), fx["patch_idx"])
    # the device variant: same structure (whole 4x4 patches, distinct corners)
    from copenerf.rays import get_patch_indices
    idx = get_patch_indices(12, 16, 4, 64, generator=torch.Generator().manual_seed(0)).view(-1, 16)
    corners = idx[:, 0]
    assert corners.unique().numel() == corners.numel()
    offs = torch.tensor([r * 16 + c for r in range(4) for c in range(4)])
    assert torch.equal(idx - corners[:, None], offs.expand_as(idx))


def test_process_data_rays_match_reference(fx):
    tr = _trainer()
    data = {"img": fx["pd_img"], "img.camera_mat": fx["pd_camera_mat"], "img.scale_mat": fx["pd_scale_mat"],
            "img.idx": torch.tensor([3]), "img.ref_imgs": fx["pd_ref_img"], "img.ref_idxs": [torch.tensor([4])]}
    torch.manual_seed(int(fx["pd_seed"]))
    out = tr.process_data(data, fx["pd_world_mat"], it=1, epoch=0, patch_size=4)
    names = ("img", "ref_img", "p", "pn", "rays_o", "rays_d", "rays_d_norm", "rgb_gt", "camera_mat", "scale_mat")
    for n, v in zip(names, out):
        ref = fx["pd_" + n]
        if n in ("p", "pn", "rgb_gt", "img", "ref_img"):
            assert torch.equal(v, ref.reshape(v.shape)), n
        else:
            torch.testing.assert_close(v, ref.reshape(v.shape), rtol=0, atol=1e-6, msg=lambda m: f"{n}: {m}")
    near, far = tr.near_far_from_sphere(out[4], out[5])
    assert torch.equal(near, fx["near"]) and torch.equal(far, fx["far"])
    for it, car in zip(fx["car_its"].tolist(), fx["car"].tolist()):
        assert float(tr.get_cos_anneal_ratio(it, 50000)) == car


def test_compute_loss_matches_reference(fx):
    tr = _trainer()
    terms = fx["cl_terms"].unbind(0)
    d = tr.compute_loss({}, fx["cl_rgb"], fx["pd_rgb_gt"], *terms)
    for k in ("loss", "loss_rgb", "l2_mean"):
        torch.testing.assert_close(d[k], fx["cl_" + k], rtol=1e-6, atol=1e-7)
    with pytest.raises(AssertionError, match="Nan loss found"):
        tr.compute_loss({}, fx["cl_rgb"], fx["pd_rgb_gt"], torch.tensor(float("nan")), *terms[1:])
    trd = _trainer(nan_check="deferred")
    trd.compute_loss({}, fx["cl_rgb"], fx["pd_rgb_gt"], torch.tensor(float("nan")), *terms[1:])
    with pytest.raises(AssertionError, match="Nan loss found"):
        trd.check_finite()


def test_train_py_iteration_sequence_on_cpu():
    """train.py:433-438, 441-444, 526-532 through `from model import Trainer`, with the
    CPU oracle standing in for the HIP renderer (the renderer is GPU-only; the
    GPU twin of this test, test_gpu_trainer.py, runs the HIP NeuSRenderer)."""
    from helpers import build_modules, oracle_params
    from oracle import neus_oracle as O
    tr = _trainer()
    mods = build_modules(3, 64, 64)
    P, Pc, var, leaves = oracle_params(*mods)

    def eff(prefix, n):  # effective weights rebuilt from the (g, v) leaves every iteration
        W = [torch._weight_norm(leaves[f"{prefix}lin{l}.weight_v"], leaves[f"{prefix}lin{l}.weight_g"], 0)
             for l in range(n)]
        return W, [leaves[f"{prefix}lin{l}.bias"] for l in range(n)]
    opt = torch.optim.Adam(list(leaves.values()), lr=1e-3)
    motion_opt = torch.optim.Adam([torch.nn.Parameter(torch.zeros(1))], lr=5e-4)
    tr.optimizer, tr.motion_optimizer = opt, motion_opt
    g = torch.Generator().manual_seed(1)
    h, w = 24, 32
    fx_ = 0.9 * w
    K = torch.tensor([[[2 * fx_ / w, 0, 0, 0], [0, -2 * fx_ / h, 0, 0], [0, 0, -1, 0], [0, 0, 0, 1]]])
    data = {"img": torch.rand(1, 3, h, w, generator=g), "img.camera_mat": K, "img.scale_mat": torch.eye(4)[None],
            "img.idx": torch.tensor([1]), "img.ref_imgs": torch.rand(1, 3, h, w, generator=g),
            "img.ref_idxs": [torch.tensor([2])]}
    world_mat = torch.eye(4)
    world_mat[2, 3] = 1.6  # camera outside the unit sphere of the geometric init
    before = {k: v.detach().clone() for k, v in leaves.items()}
    for it in (1, 2):
        (img, ref_img, p, pn, rays_o, rays_d, rays_d_norm, rgb_gt, camera_mat, scale_mat) = tr.process_data(
            data, world_mat, it=it, epoch=0, patch_size=4)
        near, far = tr.near_far_from_sphere(rays_o, rays_d)
        car = tr.get_cos_anneal_ratio(it, 50000)
        P.W, P.b = eff("sdf.", len(P.W))
        Pc.W, Pc.b = eff("col.", len(Pc.W))
        out = O.render(P, Pc, var, rays_o, rays_d, rays_d_norm, torch.tensor([0.0]), near, far, car=float(car),
                       t_rand=torch.rand(rays_o.shape[0], 64, generator=g))
        normals = out["normals"].view(-1, 3)
        gradient_loss = torch.mean((torch.linalg.norm(normals, ord=2, dim=-1) - 1.0) ** 2)
        d = out["depth_pred"].view(-1, 4, 4, 1)
        gt = rgb_gt.view(-1, 4, 4, 3)
        edge, smooth = 0.5 * O.edge_smoothness(d, gt), 0.5 * O.smoothness(d)
        z = torch.zeros(())
        loss_dict = tr.compute_loss(data, out["color_fine"], rgb_gt, gradient_loss, z, z, z, edge, smooth, it=it)
        tr.backpropagation(loss_dict, train_motion_network=False)
        assert torch.isfinite(loss_dict["loss"])
    assert all(not torch.equal(before[k], v.detach()) for k, v in leaves.items() if k.endswith("bias"))


def test_checkpoint_roundtrip(tmp_path):
    """CheckpointIO (model/checkpoints.py layout): save, then a strict reload of the
    module state dicts plus the scalars."""
    sys.path.insert(0, os.path.join(ROOT, "cope-nerf_amd"))
    from model import CheckpointIO
    from helpers import build_modules
    sdf, col, dev = build_modules(4, 64, 64)
    ck = CheckpointIO(str(tmp_path), model=sdf)
    ck.save("model.pt", True, epoch_it=3, it=42)
    sdf2, _, _ = build_modules(5, 64, 64)
    ck2 = CheckpointIO(str(tmp_path), model=sdf2)
    scalars = ck2.load(os.path.join(str(tmp_path), "models", "weights", "model.pt"))
    assert scalars == {"epoch_it": 3, "it": 42}
    for (k, a), (_, b) in zip(sdf.state_dict().items(), sdf2.state_dict().items()):
        assert torch.equal(a, b), k
