"""Full-image inference rendering (render_visdata / render_eval loop,
model/training.py:157-300) on the HIP renderer against the CPU oracle, with the
reference's pretrained SDF; chunking invariance."""
import pytest
import torch

from helpers import REN_CFG, build_modules, fixture, load_pretrained_sdf, oracle_params
from oracle import neus_oracle as O

pytestmark = pytest.mark.gpu
DEV = "cuda"


def test_render_image_matches_oracle_and_is_chunk_invariant():
    from copenerf import NeuSRenderer
    from copenerf.inference import arange_pixels, render_image
    from copenerf.rays import intrinsics_ndc, world_rays
    fx = fixture("render_pretrained")
    h, w = 24, 32
    mods = build_modules(int(fx["seed"]), device=DEV)
    load_pretrained_sdf(mods[0], fx)
    sdf, col, dev = mods
    r = NeuSRenderer(None, sdf, dev, col, None, **REN_CFG).to(DEV)
    K = intrinsics_ndc(0.9 * w, 0.9 * w, w, h, device=DEV)
    I = torch.eye(4, device=DEV)
    t = torch.tensor([0.0], device=DEV)
    a = render_image(r, K, I, I, (h, w), t, chunk=256)
    b = render_image(r, K, I, I, (h, w), t, chunk=h * w)
    for k in a:
        assert torch.equal(a[k], b[k]), k
    # oracle on the same rays (eval mode: no jitter, depth / |d|)
    mods_cpu = build_modules(int(fx["seed"]))
    load_pretrained_sdf(mods_cpu[0], fx)
    P, Pc, var, _ = oracle_params(*mods_cpu)
    _, pix = arange_pixels(h, w)
    o, d, n = world_rays(pix, K.cpu(), I.cpu(), I.cpu())
    torch.set_num_threads(8)
    R = o.shape[0]
    ref = O.render(P, Pc, var, o, d, n, torch.tensor([0.0]), torch.full((R, 1), 0.01), torch.full((R, 1), 5.0),
                   car=1.0, eval_mode=True)
    err = torch.maximum((a["rgb"].reshape(-1, 3).cpu() - ref["color_fine"].detach()).abs().max(1)[0],
                        (a["depth"].reshape(-1).cpu() - ref["depth_pred"].detach().reshape(-1)).abs())
    assert (err > 1e-4).float().mean().item() <= 0.02, err.max().item()
    assert err.median().item() <= 1e-5
    wn = (ref["normals"] * ref["weights"][:, :, None]).sum(1)
    nerr = (a["normal"].reshape(-1, 3).cpu() - wn.detach()).abs().max(1)[0]
    assert (nerr > 1e-3).float().mean().item() <= 0.02


def test_render_image_at_the_bench_chunk_size():
    """The bench's chunk (65,536 rays x 128 samples: 8.4 M rows per cn_render_fwd call, [M, 256] fp32 buffers
    above 4 GiB) renders bitwise what 4,096-ray chunks render, and matches the oracle on pixels spread over the
    whole image -- incl. rays past the first 32,768 of a chunk, whose sample rows sit beyond 4 GiB into those
    buffers (the row bound relaxed in commit 3c48c3c, cn_pipeline.hip)."""
    from copenerf import NeuSRenderer
    from copenerf.inference import arange_pixels, render_image
    from copenerf.rays import intrinsics_ndc, world_rays
    fx = fixture("render_pretrained")
    h, w = 256, 320  # 81,920 rays: one 65,536-ray chunk and a 16,384-ray tail
    mods = build_modules(int(fx["seed"]), device=DEV)
    load_pretrained_sdf(mods[0], fx)
    sdf, col, dev = mods
    r = NeuSRenderer(None, sdf, dev, col, None, **REN_CFG).to(DEV)
    r.set_mfma_dtype("bf16x6")  # the bench's GEMM mode (bench.py --config infer)
    K = intrinsics_ndc(0.9 * w, 0.9 * w, w, h, device=DEV)
    I = torch.eye(4, device=DEV)
    t = torch.tensor([0.0], device=DEV)
    big = render_image(r, K, I, I, (h, w), t, chunk=65536)
    small = render_image(r, K, I, I, (h, w), t, chunk=4096)
    for k in big:
        assert torch.equal(big[k], small[k]), k
    assert torch.isfinite(big["rgb"]).all() and big["rgb"].abs().sum() > 0
    # the oracle on 384 pixels: every 213th of the image, so a third of them lie past ray 32,768 of the first chunk
    sel = torch.arange(0, h * w, 213)
    mods_cpu = build_modules(int(fx["seed"]))
    load_pretrained_sdf(mods_cpu[0], fx)
    P, Pc, var, _ = oracle_params(*mods_cpu)
    _, pix = arange_pixels(h, w)
    o, d, n = world_rays(pix[sel], K.cpu(), I.cpu(), I.cpu())
    torch.set_num_threads(8)
    R = o.shape[0]
    assert (sel >= 32768).sum() > R // 3 and (sel < 65536).sum() > R // 2
    ref = O.render(P, Pc, var, o, d, n, torch.tensor([0.0]), torch.full((R, 1), 0.01), torch.full((R, 1), 5.0),
                   car=1.0, eval_mode=True)
    rgb = big["rgb"].reshape(-1, 3)[sel.to(DEV)].cpu()
    depth = big["depth"].reshape(-1)[sel.to(DEV)].cpu()
    err = torch.maximum((rgb - ref["color_fine"].detach()).abs().max(1)[0],
                        (depth - ref["depth_pred"].detach().reshape(-1)).abs())
    print(f"chunk 65536 vs oracle: median {err.median().item():.2e}, max {err.max().item():.2e}, "
          f"> 1e-4: {(err > 1e-4).float().mean().item():.4f}")
    # the same flip statistics as the test above (a last-ulp sdf difference may move an importance sample)
    assert (err > 1e-4).float().mean().item() <= 0.02, err.max().item()
    assert err.median().item() <= 1e-5
