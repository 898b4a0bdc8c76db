"""The C ABI library loads, exports exactly what include/copenerf.h declares,
and rejects bad arguments before touching the GPU (no device needed)."""
import ctypes
import os
import re

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "copenerf.h")


def _declared():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(cn_[a-z0-9_]+)\s*\(", src)))


def test_header_and_binding_agree():
    from copenerf import _lib
    assert set(_declared()) == set(_lib.SIGNATURES), set(_declared()) ^ set(_lib.SIGNATURES)


def test_library_exports_every_declared_symbol():
    from copenerf import _lib
    lib = _lib.load()
    for name in _declared():
        assert hasattr(lib, name), name
    m = re.search(r"#define CN_ABI_VERSION (\d+)", open(HEADER).read())
    assert lib.cn_abi_version() == int(m.group(1)) == _lib.ABI_VERSION


def test_struct_layouts_match_header_order():
    from copenerf import _lib
    src = open(HEADER).read()
    for cname, py in (("cn_linear_desc", _lib.LinearDesc), ("cn_wgrad_desc", _lib.WgradDesc),
                      ("cn_sdf_mlp_desc", _lib.SdfMlpDesc), ("cn_sdf_net", _lib.SdfNet),
                      ("cn_sample_desc", _lib.SampleDesc), ("cn_color_net", _lib.ColorNet),
                      ("cn_render_desc", _lib.RenderDesc), ("cn_mlp_desc", _lib.MlpDesc),
                      ("cn_render_grads", _lib.RenderGrads)):
        body = re.search(r"typedef struct %s \{(.*?)\} %s;" % (cname, cname), src, re.S).group(1)
        body = re.sub(r"/\*.*?\*/", "", body, flags=re.S)
        names = []
        for decl in body.split(";"):
            decl = decl.strip()
            if not decl:
                continue
            decl = re.sub(r"^(const\s+)?\w+\s*\**", "", decl)
            names += [re.sub(r"\[[\w\s+-]+\]", "", n.strip(" *")) for n in decl.split(",")]
        assert names == [f[0] for f in py._fields_], (cname, names)
    assert ctypes.sizeof(_lib.LinearDesc) % 8 == 0


def test_argument_validation_without_gpu():
    from copenerf import _lib
    lib = _lib.load()
    assert lib.cn_linear(None, None) == -1
    assert b"null desc" in lib.cn_last_error()
    d = _lib.LinearDesc()
    d.A, d.B, d.out0 = 16, 16, 16
    d.M, d.N, d.K = 8, 8, 30  # K not a multiple of 32
    assert lib.cn_linear(ctypes.byref(d), None) == -2
    assert b"multiple of 32" in lib.cn_last_error()
    assert lib.cn_row_head(1, 300, 16, 4, 16, 4, None, 1, 0, 16, 1, None, None) == -5
    assert lib.cn_up_sample_merge(1, 300, 16, 1.0, 16, 16, 16, 16, None, None, None) == -5
    w = _lib.WgradDesc()
    assert lib.cn_wgrad(ctypes.byref(w), None) == -1
    assert lib.cn_wgrad_batch(None, 1, None) == -1
    ws2 = (_lib.WgradDesc * 2)()
    assert lib.cn_wgrad_batch(ws2, 2, None) == -1  # checked before anything launches
    assert lib.cn_wgrad_batch(ws2, 0, None) == 0
    assert lib.cn_wgrad_workspace_bytes(524288, 256, 256) >= 4 * 256 * 256
    ws = lib.cn_train_loss_workspace_bytes(4096, 4)
    assert ws >= 8 * (4096 // 16 // 256)
    assert lib.cn_train_loss(4096, 5, 0, 16, 16, 16, None, 0, 16, 0.1, 16, 16, 16, None, 0, None, 16, ws,
                             None) == -5
    assert b"patch 5" in lib.cn_last_error()
    # ABI v4: the softplus-derivative epilogues need aux_beta; no epilogue writes out1
    d = _lib.LinearDesc()
    d.A, d.B, d.out0, d.aux0 = 16, 16, 16, 16
    d.M, d.N, d.K, d.lda, d.ldb, d.ld_out0, d.ld_aux0 = 8, 8, 32, 32, 32, 8, 8
    d.epilogue = _lib.EPI_MUL
    assert lib.cn_linear(ctypes.byref(d), None) == -1
    assert b"aux_beta" in lib.cn_last_error()
    d.aux_beta, d.out1 = 100.0, 16
    assert lib.cn_linear(ctypes.byref(d), None) == -1
    assert b"out1" in lib.cn_last_error()
    # ABI v10 bf16 images: BWD_SOFTPLUS takes its three aux operands in one format
    d = _lib.LinearDesc()
    d.A, d.B, d.out0_b, d.aux0, d.aux1, d.aux2 = 16, 16, 16, 16, 16, 16
    d.M, d.N, d.K, d.lda, d.ldb, d.ld_out0_b, d.ld_aux0, d.ld_aux1, d.ld_aux2 = 8, 256, 256, 256, 256, 256, 256, 256, 256
    d.epilogue, d.mfma_dtype, d.aux_beta, d.a_bf16, d.aux0_bf16 = _lib.EPI_BWD_SOFTPLUS, 1, 100.0, 1, 1
    assert lib.cn_linear(ctypes.byref(d), None) == -5
    assert b"all bf16 images or all fp32" in lib.cn_last_error()
    d.mfma_dtype = 2  # images only in the bf16 MFMA mode
    assert lib.cn_linear(ctypes.byref(d), None) == -5
    assert b"CN_MFMA_BF16" in lib.cn_last_error()
    # cn_softplus_adjoint's in_bf16 is a 3-bit mask; cn_rgb_head_bwd's bf16 dZ needs 8-byte alignment
    assert lib.cn_softplus_adjoint(8, 256, None, 0, 16, 256, 100.0, None, None, None, 0, None, 0, 0.0, 16, 256,
                                   1, 9, None, None, 1.0, None, 0, None) == -1
    assert b"3-bit mask" in lib.cn_last_error()
    assert lib.cn_rgb_head_bwd(8, 256, 16, 16, 16, 256, 16, 18, 256, 1, 16, 16, 16, 1 << 20, None) == -3
    # ABI v11: the fused sampler query takes the 8 x 256 SDF network only
    assert lib.cn_sdf_mlp(None, None) == -1
    m = _lib.SdfMlpDesc()
    m.u0 = m.tail = m.sdf = m.head_w = m.head_b = 16
    m.n_layers, m.hidden, m.kpad0 = 8, 128, 64
    assert lib.cn_sdf_mlp(ctypes.byref(m), None) == -5
    assert b"8 x 256" in lib.cn_last_error()



def _fake_net(mode=1, dh=256, multires=6, skip=4):
    """A cn_sdf_net of SDFNetwork(d_hidden=dh, n_layers=8, skip_in=[skip]) with placeholder (aligned,
    never dereferenced) pointers: host planning only."""
    from copenerf import _lib
    n = _lib.SdfNet()
    E = 4 * (1 + 2 * multires)
    n.n_lin, n.skip, n.multires, n.scale, n.beta, n.threshold, n.mfma_dtype = 9, skip, multires, 1.0, 100.0, 20.0, mode
    kq = 64 if mode == 1 else 32
    for l in range(9):
        n.out_dim[l] = 257 if l == 8 else (dh - E if l + 1 == skip else dh)
        n.in_dim[l] = E if l == 0 else n.out_dim[l - 1] + (E if l == skip else 0)
    for l in range(8):
        n.W[l], n.bias[l] = 4096, 4096
        n.w_rows[l] = -(-n.out_dim[l] // 128) * 128
        n.w_cols[l] = 64 if l == 0 else -(-n.in_dim[l] // kq) * kq
    n.head_w = n.head_b = 4096
    return n


def test_composed_entry_points_plan_without_gpu():
    """ABI v12: cn_sdf_query / cn_sample validate and size their workspace on the host."""
    from copenerf import _lib
    lib = _lib.load()
    assert lib.cn_sdf_query(None, 1, 16, 4, 16, None, 16, 1 << 20, None) == -1
    assert lib.cn_sdf_query_workspace_bytes(None, 10) == 0
    assert lib.cn_sample(None, None, 0, None) == -1
    n = _fake_net()
    M = 262144
    assert lib.cn_sdf_query_workspace_bytes(ctypes.byref(n), M) == 2 * M * 64 * 2  # fused: the two bf16 images
    n.flags = 1  # layered: U0 fp32 [M][64], the skip input's bf16 image, two bf16 ping-pong buffers
    assert lib.cn_sdf_query_workspace_bytes(ctypes.byref(n), M) == M * 64 * 4 + 3 * M * 256 * 2
    n.flags = 0
    x = _fake_net(mode=0)  # fp32 buffers
    assert lib.cn_sdf_query_workspace_bytes(ctypes.byref(x), M) == M * 64 * 4 + 3 * M * 256 * 4
    x.in_dim[3] = 200  # inconsistent widths
    assert lib.cn_sdf_query(ctypes.byref(x), 4, 4096, 4, 4096, None, 4096, 1 << 30, None) == -2
    assert b"lin3 takes 200" in lib.cn_last_error()
    d = _lib.SampleDesc()
    d.R, d.n_samples, d.n_importance, d.up_sample_steps = 4096, 64, 64, 4
    d.rays_o = d.rays_d = d.near = d.far = d.time_step = d.z = 4096
    d.net = ctypes.pointer(n)
    R, k = 4096, 16
    want = 4 * (R * 128 * 4) + R * 64 * 16 + 2 * R * k * 4 + 2 * (R * 64) * 64 * 2
    assert lib.cn_sample_workspace_bytes(ctypes.byref(d)) == want
    assert lib.cn_sample(ctypes.byref(d), 4096 * 256, want - 1, None) == -2
    assert b"workspace" in lib.cn_last_error()
    d.n_importance = 3  # fewer than one sample per round
    assert lib.cn_sample(ctypes.byref(d), 4096 * 256, want, None) == -2
    d.n_importance = 64
    n.w_rows[2] = 128  # an image too small for its layer
    assert lib.cn_sample(ctypes.byref(d), 4096 * 256, want, None) == -2
    assert b"layer 2 image" in lib.cn_last_error()


def test_render_fwd_checks_without_gpu():
    """ABI v13: cn_render_fwd validates both networks and the fold on the host."""
    from copenerf import _lib
    lib = _lib.load()
    assert lib.cn_render_fwd(None, None, 0, None) == -1
    assert lib.cn_render_fwd_workspace_bytes(None) == 0
    n = _fake_net()
    for l in range(8):
        n.Wt[l], n.wt_rows[l], n.wt_cols[l] = 4096, 256, 256
    n.head_wp = 4096
    c = _lib.ColorNet()
    c.n_lin, c.d_feature, c.multires_view, c.mfma_dtype = 5, 256, 4, 1
    dims = [4 + 27 + 4 + 256, 256, 256, 256, 256]
    for l in range(5):
        c.in_dim[l], c.out_dim[l] = dims[l], (3 if l == 4 else 256)
    for l in range(4):
        c.W[l], c.w_rows[l], c.w_cols[l], c.bias[l] = 4096, 256, (256 + 64 if l == 0 else 256), 4096
    c.head_w = c.head_b = 4096
    d = _lib.RenderDesc()
    d.R, d.n_samples, d.n_importance, d.up_sample_steps = 4096, 64, 64, 4
    for k in ("rays_o", "rays_d", "near", "far", "time_step", "inv_s", "cos_anneal_ratio", "z", "pts", "sdf", "grad",
              "rgb", "color", "depth", "weights", "cdf"):
        setattr(d, k, 4096)
    d.sdf_net, d.color_net = ctypes.pointer(n), ctypes.pointer(c)
    M = 4096 * 128
    ws = lib.cn_render_fwd_workspace_bytes(ctypes.byref(d))
    assert ws >= M * 256 * 2 * 7  # at least the kept activations
    assert lib.cn_render_fwd(ctypes.byref(d), 4096 * 256, ws - 1, None) == -2
    d.up_sample_steps = 0  # importance samples without rounds
    assert lib.cn_render_fwd_workspace_bytes(ctypes.byref(d)) == 0
    assert lib.cn_render_fwd(ctypes.byref(d), 4096 * 256, ws, None) == -2
    d.up_sample_steps = 4
    c.mfma_dtype = 2
    assert lib.cn_render_fwd(ctypes.byref(d), 4096 * 256, ws, None) == -1
    assert b"modes differ" in lib.cn_last_error()
    c.mfma_dtype, c.d_feature = 1, 128  # no fold: the colour network's feature is not the SDF's hidden layer
    c.in_dim[0] = 4 + 27 + 4 + 128
    c.w_cols[0] = 128 + 64
    assert lib.cn_render_fwd(ctypes.byref(d), 4096 * 256, ws, None) == -5


def test_uniform_philox_checks_without_gpu():
    """ABI v14: cn_uniform_philox refuses null pointers; n = 0 draws nothing."""
    from copenerf import _lib
    lib = _lib.load()
    assert lib.cn_uniform_philox(10, None, 4096, None) == -1
    assert lib.cn_uniform_philox(0, None, None, None) == 0
    d = _lib.SampleDesc()
    d.R, d.n_samples, d.n_importance, d.up_sample_steps = 4096, 64, 0, 4
    d.near = d.far = d.z = 4096
    assert lib.cn_sample_workspace_bytes(ctypes.byref(d)) == 0  # no draws: no workspace
    d.philox = 4096
    assert lib.cn_sample_workspace_bytes(ctypes.byref(d)) == 4096 * 64 * 4  # the drawn jitter


def test_mlp_entry_points_check_and_plan_without_gpu():
    """ABI v14: cn_mlp_fwd / cn_mlp_bwd size the kept state and the backward's workspace on the host and
    refuse incomplete descriptors before anything launches."""
    from copenerf import _lib
    lib = _lib.load()
    assert lib.cn_mlp_fwd(None, None, 0, None) == -1
    assert lib.cn_mlp_state_bytes(None) == 0 and lib.cn_mlp_bwd_workspace_bytes(None) == 0
    n = _fake_net()  # bf16 images, d_hidden 256, skip 4
    M = 65536
    d = _lib.MlpDesc()
    d.M, d.x, d.sdf, d.net = M, 4096, 4096, ctypes.pointer(n)
    # U_0 fp32 [M][64], U_1 .. U_7 bf16 images (the skip input's too), U_8 fp32
    want = M * 64 * 4 + 7 * M * 256 * 2 + M * 256 * 4
    assert lib.cn_mlp_state_bytes(ctypes.byref(d)) == want
    assert lib.cn_mlp_fwd(ctypes.byref(d), 4096 * 256, want - 1, None) == -2
    f = _fake_net(mode=0)
    d.net = ctypes.pointer(f)
    assert lib.cn_mlp_state_bytes(ctypes.byref(d)) == M * 64 * 4 + 8 * M * 256 * 4
    d.net = ctypes.pointer(n)
    d.dsdf = 4096
    assert lib.cn_mlp_bwd(ctypes.byref(d), 4096 * 256, want, 4096 * 256, 1 << 40, None) == -1
    assert b"neither" in lib.cn_last_error()
    d.dx = 4096
    assert lib.cn_mlp_bwd(ctypes.byref(d), 4096 * 256, want, 4096 * 256, 1 << 40, None) == -2
    assert b"transposed image 0" in lib.cn_last_error()
    for l in range(8):
        n.Wt[l], n.wt_rows[l], n.wt_cols[l] = 4096, 256, 256
    n.head_wp = 4096
    dx_only = lib.cn_mlp_bwd_workspace_bytes(ctypes.byref(d))
    assert dx_only == 2 * M * 256 * 4 + 2 * M * 64 * 4  # two fp32 adjoints, PE, P0
    for l in range(9):
        d.dW[l], d.db[l] = 4096, 4096
    d.db[3] = None
    assert lib.cn_mlp_bwd(ctypes.byref(d), 4096 * 256, want, 4096 * 256, 1 << 40, None) == -1
    assert b"db[3]" in lib.cn_last_error()
    d.db[3] = 4096
    full = lib.cn_mlp_bwd_workspace_bytes(ctypes.byref(d))
    assert full >= 7 * M * 256 * 2 + M * 256 * 4 + 2 * M * 64 * 4  # Z_7 .. Z_1 images, Z_0, PE, P0
    assert lib.cn_mlp_bwd(ctypes.byref(d), 4096 * 256, want, 4096 * 256, full - 1, None) == -2
    assert b"workspace" in lib.cn_last_error()


def test_product_path_refuses_cpu_tensors():
    from copenerf import SDFNetwork
    torch.manual_seed(0)
    net = SDFNetwork(d_in=4, d_out=257, d_hidden=64, n_layers=8, skip_in=[4], multires=6)
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        net.sdf(torch.zeros(8, 4))


def test_kernel_name_queries_follow_the_launch_choice():
    """cn_linear_kernel_name / cn_wgrad_kernel_name (no device access): C2's hidden-layer
    SOFTPLUS on the 256x256 bf16x6 tile, the colour network's RELU with a rowv on the 256x128
    tile, 256x256 and 256x64 bf16x6 weight gradients on the stage rings -- the rocprofv3 symbols the
    bench's launch classes report."""
    from copenerf import _lib, ops
    d = _lib.LinearDesc()
    d.M, d.N, d.K, d.K1, d.ldb, d.epilogue, d.tile, d.mfma_dtype = 524288, 256, 256, 256, 256, 1, 0, 2
    assert ops.kernel_name(_lib.load().cn_linear_kernel_name, d) == \
        "void cn::linear_kernel<4, 2, 2, 4, 16, 1, 2, 1, false, 2>(cn::LinearArgs)"
    d.epilogue, d.rowv = 2, 16
    assert ops.kernel_name(_lib.load().cn_linear_kernel_name, d) == \
        "void cn::linear_kernel<4, 2, 2, 2, 32, 1, 2, 2, true, 2>(cn::LinearArgs)"
    w = _lib.WgradDesc()
    w.M, w.N, w.K, w.npairs, w.mfma_dtype = 524288, 256, 256, 2, 2
    w.ldy0 = w.ldx0 = w.ldy1 = w.ldx1 = 256
    assert ops.kernel_name(_lib.load().cn_wgrad_kernel_name, w) == "void cn::wgrad_x6r_kernel<2>(cn::WgradBatch)"
    w.K, w.ldx0, w.ldx1 = 64, 64, 64  # a K = 64 first layer: the narrow stage ring
    assert ops.kernel_name(_lib.load().cn_wgrad_kernel_name, w) == "void cn::wgrad_x6n_kernel<3>(cn::WgradArgs)"
    w.ldy0 = w.ldy1 = 128  # Y rows not 256-padded: the 128x64 tiles
    assert ops.kernel_name(_lib.load().cn_wgrad_kernel_name, w) == "void cn::wgrad_x6_kernel<2, 1>(cn::WgradArgs)"
    assert _lib.load().cn_linear_kernel_name(d, ctypes.create_string_buffer(8), 8) == -2  # CN_ERR_SHAPE


def test_shape_key_sees_scalars_and_pointer_presence_only():
    """ops._sized memoises the composed entry points' sizing on _lib.shape_key: pointer values must not
    matter, their presence and every scalar (nested networks' too) must."""
    from copenerf import _lib
    n, c = _lib.SdfNet(), _lib.ColorNet()
    d = _lib.RenderDesc()
    d.sdf_net, d.color_net = ctypes.pointer(n), ctypes.pointer(c)
    d.R, n.n_lin, n.beta = 4096, 9, 100.0
    k0 = _lib.shape_key(d)
    d.rays_o = 0x1000
    k1 = _lib.shape_key(d)
    assert k1 != k0
    d.rays_o = 0x2000
    n.W[2] = 0x3000
    k2 = _lib.shape_key(d)
    assert k2 != k1
    n.W[2] = 0x4000
    assert _lib.shape_key(d) == k2
    for obj, field, val in ((d, "R", 2048), (n, "beta", 50.0), (c, "d_feature", 128), (n, "in_dim", None)):
        if val is None:
            getattr(obj, field)[3] += 1
        else:
            old = getattr(obj, field)
            setattr(obj, field, val)
            assert _lib.shape_key(d) != k2, field
            setattr(obj, field, old)
            continue
        assert _lib.shape_key(d) != k2, field
        getattr(obj, field)[3] -= 1
    assert _lib.shape_key(d) == k2
    d.color_net = None
    assert _lib.shape_key(d) != k2
