"""Stage-1 motion model against golden vectors from the reference's
MotionNetwork (tests/golden/motion.npz, made by tests/golden/make_golden.py):
seeded weights, forward, relative camera poses, world-to-camera chain; and
the scene-flow loss against the oracle."""
import torch

from helpers import fixture
from oracle import neus_oracle as O

CFG = dict(d_out=6, d_in=1, d_hidden=256, n_layers=4, skip_in=[2], multires=6, bias=0.5, scale=1.0,
           weight_norm=True)


def test_motion_network_matches_reference():
    from copenerf.motion import MotionNetwork
    fx = fixture("motion")
    for tag, gi in (("", False), ("geo.", True)):
        torch.manual_seed(681)
        m = MotionNetwork(**dict(CFG, geometric_init=gi))
        sd = m.state_dict()
        keys = sorted(k[len(tag) + 3:] for k in fx if k.startswith(tag + "sd."))
        assert sorted(sd.keys()) == keys
        for k in keys:
            assert torch.equal(sd[k], fx[tag + "sd." + k]), (tag, k)
        w, v = m(fx[tag + "t"])
        torch.testing.assert_close(w, fx[tag + "omega"], rtol=1e-5, atol=1e-6)
        torch.testing.assert_close(v, fx[tag + "vel"], rtol=1e-5, atol=1e-6)
        dt, rel = m.compute_relative_camera_pose(target_cam_idx=2, final_ref_cam_idx=5, total_nb_images=10,
                                                 nb_sample_timestep=10)
        assert abs(float(dt) - float(fx[tag + "dt"])) <= 1e-7
        torch.testing.assert_close(torch.stack(rel), fx[tag + "rel"], rtol=1e-5, atol=1e-6)
        torch.testing.assert_close(m.compute_w2c_mappings(rel), fx[tag + "w2c"], rtol=1e-5, atol=1e-6)


def test_scene_flow_loss_matches_oracle():
    from copenerf.motion import scene_flow_loss
    g = torch.Generator().manual_seed(3)
    M = 4096
    pts, n = torch.randn(M, 3, generator=g), torch.randn(M, 3, generator=g)
    fl, w = torch.randn(M, 1, generator=g), torch.rand(M, generator=g)
    om, vel = torch.randn(1, 3, generator=g), torch.randn(1, 3, generator=g)
    a = scene_flow_loss(pts, n, fl, w, om, vel)
    b = O.scene_flow_loss(pts, n, fl, w, om, vel)
    torch.testing.assert_close(a, b, rtol=1e-6, atol=1e-7)


def test_euler_xyz_is_a_rotation_product():
    from copenerf.motion import euler_angles_to_matrix
    e = torch.tensor([[0.3, -0.2, 0.7]])
    R = euler_angles_to_matrix(e, "XYZ")[0]
    torch.testing.assert_close(R @ R.T, torch.eye(3), atol=1e-6, rtol=0)
    cx, sx = torch.cos(e[0, 0]), torch.sin(e[0, 0])
    Rx = torch.tensor([[1.0, 0, 0], [0, cx, -sx], [0, sx, cx]])
    torch.testing.assert_close(euler_angles_to_matrix(torch.tensor([[0.3, 0.0, 0.0]]), "XYZ")[0], Rx)
