"""Which piece of the joint-pose / stage-1 step is not HIP-graph capturable?  Captures
small pieces separately (each in a fresh private graph) and prints the outcome."""
import os
import sys
import traceback

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "cope-nerf_amd"), ROOT, os.path.join(ROOT, "tests")]


def try_capture(name, fn):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()  # warm-up
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    try:
        with torch.cuda.graph(g):
            fn()
        print(f"{name}: OK", flush=True)
        return True
    except Exception as e:  # noqa: BLE001
        print(f"{name}: FAIL {type(e).__name__}: {str(e).splitlines()[0]}", flush=True)
        traceback.print_exc(limit=4)
        return False


def main():
    from copenerf.rays import PoseRetriever, inv4x4, world_rays, intrinsics_ndc
    dev = "cuda"
    pr = PoseRetriever(6).to(dev)
    idx = torch.tensor([2], device=dev)
    K = intrinsics_ndc(50, 50, 64, 48, device=dev)
    I = torch.eye(4, device=dev)
    pixn = torch.rand(64, 2, device=dev)

    def pose_fb():
        m = pr.pose_at(idx)
        m.sum().backward()

    def inv_fb():
        m = pr.pose_at(idx)
        inv4x4(m).sum().backward()

    def rays_fb():
        o, d, n = world_rays(pixn, K, pr.pose_at(idx), I)
        (o.sum() + d.sum()).backward()
    ok = [try_capture("pose_at fwd+bwd", pose_fb), try_capture("inv4x4 fwd+bwd", inv_fb),
          try_capture("world_rays fwd+bwd", rays_fb)]
    from copenerf.motion import MotionNetwork, masked_chain
    from copenerf.train_step import MOTION_CFG
    mn = MotionNetwork(**MOTION_CFG).to(dev)
    steps, dts = mn.interval_time_grid(6, 10)

    def motion_fb():
        P = mn.batched_relative_poses(steps, dts)
        P.sum().backward()

    def chain_fb():
        P = mn.batched_relative_poses(steps, dts)
        c = masked_chain(P, idx, idx + 2)
        c.sum().backward()

    def gs_fb():
        img = torch.rand(3, 3, 48, 64, device=dev)
        grid = (torch.rand(3, 64, 1, 2, device=dev) * 2 - 1).requires_grad_(True)
        torch.nn.functional.grid_sample(img, grid, mode="bilinear", padding_mode="border", align_corners=True).sum().backward()
    ok += [try_capture("motion poses fwd+bwd", motion_fb), try_capture("masked_chain fwd+bwd", chain_fb),
           try_capture("grid_sample fwd+bwd", gs_fb)]
    print("all ok" if all(ok) else "some failed", flush=True)


if __name__ == "__main__":
    main()
