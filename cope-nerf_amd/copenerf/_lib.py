"""ctypes binding of libcopenerf.so (include/copenerf.h).

This is the reference-side binding of the C ABI: the reference is pure Python,
so the "FFI" it would grow for this path is a ctypes stub exactly like this one
(see INTEGRATION.md).  The library is looked up next to this file; if it is
missing, or cannot be loaded, every hot-path entry point raises -- there is no
CPU fallback on the product path.
"""
from __future__ import annotations

import ctypes
import os
import threading

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_NAME = "libcopenerf.so"
LIB_PATH = os.environ.get("COPENERF_LIB", os.path.join(_HERE, LIB_NAME))

ABI_VERSION = 15

c_f32p = ctypes.c_void_p  # device pointers are passed as integers
c_i32 = ctypes.c_int32
c_i64 = ctypes.c_int64
c_f32 = ctypes.c_float
c_ptr = ctypes.c_void_p

# cn_epilogue
EPI_STORE = 0
EPI_SOFTPLUS = 1
EPI_RELU = 2
EPI_MUL = 3
EPI_TANGENT = 4
EPI_BWD_SOFTPLUS = 5
EPI_BWD_RELU = 6
EPI_SOFTPLUS_HEAD = 8


class WnJob(ctypes.Structure):
    _fields_ = [("v", c_ptr), ("g", c_ptr), ("w", c_ptr), ("dw", c_ptr), ("dv", c_ptr), ("dg", c_ptr),
                ("rows", c_i32), ("cols", c_i32)]


class LinearDesc(ctypes.Structure):
    _fields_ = [
        ("A", c_ptr), ("A2", c_ptr), ("B", c_ptr), ("bias", c_ptr), ("rowv", c_ptr), ("colv", c_ptr),
        ("aux0", c_ptr), ("aux1", c_ptr), ("out0", c_ptr), ("out1", c_ptr), ("out_split", c_ptr),
        ("lda", c_i64), ("lda2", c_i64), ("ldb", c_i64), ("ld_aux0", c_i64), ("ld_aux1", c_i64),
        ("ld_out0", c_i64), ("ld_out1", c_i64), ("ld_split", c_i64),
        ("M", c_i32), ("N", c_i32), ("K", c_i32), ("K1", c_i32),
        ("nzero", c_i32), ("nsplit", c_i32), ("epilogue", c_i32), ("tile", c_i32),
        ("adiv", c_f32), ("odiv", c_f32), ("beta", c_f32), ("threshold", c_f32),
        ("mfma_dtype", c_i32), ("aux_beta", c_f32), ("aux2", c_ptr), ("ld_aux2", c_i64),
        ("aux2_scale", c_f32), ("flags", c_i32),
        ("head_w", c_ptr), ("head_b", c_ptr), ("head_out", c_ptr), ("head_idx", c_ptr),
        ("a_bf16", c_i32), ("aux0_bf16", c_i32), ("aux12_bf16", c_i32), ("out0_b", c_ptr), ("ld_out0_b", c_i64),
        ("out1_b", c_ptr), ("ld_out1_b", c_i64),
    ]


class WgradDesc(ctypes.Structure):
    _fields_ = [
        ("Y0", c_ptr), ("X0", c_ptr), ("Y1", c_ptr), ("X1", c_ptr),
        ("workspace", c_ptr), ("dW", c_ptr), ("db", c_ptr),
        ("ldy0", c_i64), ("ldx0", c_i64), ("ldy1", c_i64), ("ldx1", c_i64), ("ld_dw", c_i64),
        ("workspace_bytes", c_i64),
        ("M", c_i32), ("N", c_i32), ("K", c_i32), ("npairs", c_i32),
        ("n_out", c_i32), ("k_out", c_i32), ("accumulate", c_i32), ("mfma_dtype", c_i32),
        ("y_bf16", c_i32), ("x_bf16", c_i32),
    ]


class PackJob(ctypes.Structure):
    _fields_ = [
        ("src", c_ptr), ("dst", c_ptr), ("src_ld", c_i64), ("dst_ld", c_i64),
        ("rows", c_i32), ("cols", c_i32), ("r0", c_i32), ("r1", c_i32), ("c0", c_i32), ("c1", c_i32),
        ("transpose", c_i32), ("format", c_i32),
    ]


class SdfMlpDesc(ctypes.Structure):
    _fields_ = [
        ("u0", c_ptr), ("tail", c_ptr), ("ld_u0", c_i64), ("ld_t", c_i64),
        ("M", c_i32), ("n_layers", c_i32), ("hidden", c_i32), ("kpad0", c_i32), ("multires", c_i32),
        ("skip_layer", c_i32),
        ("W", c_ptr * 8), ("ldw", c_i64 * 8), ("bias", c_ptr * 8),
        ("head_w", c_ptr), ("head_b", c_ptr), ("sdf", c_ptr), ("idx", c_ptr),
        ("skip_div", c_f32), ("beta", c_f32), ("threshold", c_f32), ("debug", c_ptr), ("format", c_i32),
    ]


SDF_MAX_LIN = 16


class SdfNet(ctypes.Structure):
    _fields_ = [
        ("n_lin", c_i32), ("in_dim", c_i32 * SDF_MAX_LIN), ("out_dim", c_i32 * SDF_MAX_LIN), ("skip", c_i32),
        ("multires", c_i32), ("scale", c_f32), ("beta", c_f32), ("threshold", c_f32), ("mfma_dtype", c_i32),
        ("flags", c_i32),
        ("W", c_ptr * (SDF_MAX_LIN - 1)), ("w_rows", c_i32 * (SDF_MAX_LIN - 1)), ("w_cols", c_i32 * (SDF_MAX_LIN - 1)),
        ("bias", c_ptr * (SDF_MAX_LIN - 1)), ("head_w", c_ptr), ("head_b", c_ptr),
        ("Wt", c_ptr * (SDF_MAX_LIN - 1)), ("wt_rows", c_i32 * (SDF_MAX_LIN - 1)), ("wt_cols", c_i32 * (SDF_MAX_LIN - 1)),
        ("head_wp", c_ptr),
    ]


class ColorNet(ctypes.Structure):
    _fields_ = [
        ("n_lin", c_i32), ("in_dim", c_i32 * SDF_MAX_LIN), ("out_dim", c_i32 * SDF_MAX_LIN), ("d_feature", c_i32),
        ("multires_view", c_i32), ("mfma_dtype", c_i32),
        ("W", c_ptr * (SDF_MAX_LIN - 1)), ("w_rows", c_i32 * (SDF_MAX_LIN - 1)), ("w_cols", c_i32 * (SDF_MAX_LIN - 1)),
        ("bias", c_ptr * (SDF_MAX_LIN - 1)), ("head_w", c_ptr), ("head_b", c_ptr),
        ("Wt", c_ptr * (SDF_MAX_LIN - 1)), ("wt_rows", c_i32 * (SDF_MAX_LIN - 1)), ("wt_cols", c_i32 * (SDF_MAX_LIN - 1)),
        ("Wtf", c_ptr), ("wtf_rows", c_i32), ("wtf_cols", c_i32), ("Wg", c_ptr), ("wg_ld", c_i32), ("Wxt", c_ptr),
        ("wxt_rows", c_i32), ("wxt_cols", c_i32),
    ]


class SampleDesc(ctypes.Structure):
    _fields_ = [
        ("R", c_i32), ("n_samples", c_i32), ("n_importance", c_i32), ("up_sample_steps", c_i32),
        ("rays_o", c_ptr), ("rays_d", c_ptr), ("near", c_ptr), ("far", c_ptr), ("t_rand", c_ptr),
        ("time_step", c_ptr), ("net", ctypes.POINTER(SdfNet)), ("z", c_ptr), ("philox", c_ptr),
    ]


class RenderDesc(ctypes.Structure):
    _fields_ = [
        ("R", c_i32), ("n_samples", c_i32), ("n_importance", c_i32), ("up_sample_steps", c_i32), ("S_in", c_i32),
        ("rays_o", c_ptr), ("rays_d", c_ptr), ("near", c_ptr), ("far", c_ptr), ("t_rand", c_ptr), ("time_step", c_ptr),
        ("z_in", c_ptr), ("inv_s", c_ptr), ("cos_anneal_ratio", c_ptr), ("sdf_net", ctypes.POINTER(SdfNet)),
        ("color_net", ctypes.POINTER(ColorNet)), ("z", c_ptr), ("pts", c_ptr), ("sdf", c_ptr), ("grad", c_ptr),
        ("rgb", c_ptr), ("color", c_ptr), ("depth", c_ptr), ("weights", c_ptr), ("cdf", c_ptr), ("philox", c_ptr),
    ]


class RenderGrads(ctypes.Structure):
    _fields_ = [
        ("dcolor", c_ptr), ("ddepth", c_ptr), ("dweights", c_ptr), ("dcdf", c_ptr), ("dsdf", c_ptr), ("dgrad", c_ptr),
        ("dpts", c_ptr), ("sdf_dW", c_ptr * SDF_MAX_LIN), ("sdf_db", c_ptr * SDF_MAX_LIN),
        ("col_dW", c_ptr * SDF_MAX_LIN), ("col_db", c_ptr * SDF_MAX_LIN), ("dinv_s", c_ptr), ("drays_o", c_ptr),
        ("drays_d", c_ptr),
    ]


class MlpDesc(ctypes.Structure):
    _fields_ = [
        ("M", c_i32), ("x", c_ptr), ("net", ctypes.POINTER(SdfNet)), ("sdf", c_ptr), ("dsdf", c_ptr),
        ("dW", c_ptr * SDF_MAX_LIN), ("db", c_ptr * SDF_MAX_LIN), ("dx", c_ptr),
    ]


# name -> (restype, argtypes); mirrors include/copenerf.h one to one.
SIGNATURES = {
    "cn_abi_version": (c_i32, []),
    "cn_last_error": (ctypes.c_char_p, []),
    "cn_linear": (c_i32, [ctypes.POINTER(LinearDesc), c_ptr]),
    "cn_linear_kernel_name": (c_i32, [ctypes.POINTER(LinearDesc), ctypes.c_char_p, c_i32]),
    "cn_wgrad_kernel_name": (c_i32, [ctypes.POINTER(WgradDesc), ctypes.c_char_p, c_i32]),
    "cn_weight_norm": (c_i32, [ctypes.POINTER(WnJob), c_i32, c_i32, c_ptr]),
    "cn_wgrad_workspace_bytes": (ctypes.c_size_t, [c_i32, c_i32, c_i32]),
    "cn_wgrad": (c_i32, [ctypes.POINTER(WgradDesc), c_ptr]),
    "cn_wgrad_batch": (c_i32, [ctypes.POINTER(WgradDesc), c_i32, c_ptr]),
    "cn_wgrad_batch_workspace_bytes": (ctypes.c_size_t, [ctypes.POINTER(WgradDesc), c_i32, c_ptr]),
    "cn_pack_weights": (c_i32, [ctypes.POINTER(PackJob), c_i32, c_ptr]),
    "cn_row_head": (c_i32, [c_i32, c_i32, c_ptr, c_i64, c_ptr, c_i64, c_ptr, c_i32, c_i32, c_ptr, c_i64,
                            c_ptr, c_ptr]),
    "cn_softplus_adjoint_workspace_bytes": (ctypes.c_size_t, [c_i32, c_i32]),
    "cn_softplus_adjoint": (c_i32, [c_i32, c_i32, c_ptr, c_i64, c_ptr, c_i64, c_f32, c_ptr, c_ptr, c_ptr, c_i64,
                                    c_ptr, c_i64, c_f32, c_ptr, c_i64, c_i32, c_i32, c_ptr, c_ptr, c_f32, c_ptr,
                                    c_i64, c_ptr]),
    "cn_scale_cols": (c_i32, [c_i32, c_i32, c_ptr, c_i64, c_ptr, c_ptr, c_ptr, c_i64, c_f32, c_ptr]),
    "cn_sdf_embed": (c_i32, [c_i32, c_ptr, c_i64, c_i32, c_f32, c_i32, c_ptr, c_i64, c_ptr, c_i64, c_f32,
                             c_i32, c_ptr]),
    "cn_sdf_grad_assemble": (c_i32, [c_i32, c_i32, c_f32, c_ptr, c_i64, c_ptr, c_i64, c_ptr, c_i64, c_ptr,
                                     c_i64, c_ptr]),
    "cn_sdf_tangent_prep": (c_i32, [c_i32, c_i32, c_f32, c_i32, c_ptr, c_i64, c_ptr, c_i64, c_ptr, c_i64,
                                    c_ptr, c_i64, c_f32, c_i32, c_ptr]),
    "cn_color_extras": (c_i32, [c_i32, c_ptr, c_i64, c_ptr, c_i64, c_ptr, c_i64, c_i32, c_i32, c_i32, c_ptr,
                                c_i64, c_ptr]),
    "cn_rgb_head_bwd_workspace_bytes": (ctypes.c_size_t, [c_i32, c_i32]),
    "cn_rgb_head_bwd": (c_i32, [c_i32, c_i32, c_ptr, c_ptr, c_ptr, c_i64, c_ptr, c_ptr, c_i64, c_i32, c_ptr,
                                c_ptr, c_ptr, c_i64, c_ptr]),
    "cn_colsum_workspace_bytes": (ctypes.c_size_t, [c_i32, c_i32]),
    "cn_colsum": (c_i32, [c_i32, c_i32, c_ptr, c_ptr, c_i64, c_f32, c_ptr, c_i32, c_ptr, c_i64, c_ptr]),
    "cn_patch_indices": (c_i32, [c_i32, c_i32, c_i32, c_i32, c_ptr, c_ptr, c_ptr]),
    "cn_euler_chain": (c_i32, [c_i32, c_i32, c_ptr, c_i64, c_ptr, c_i64, c_ptr, c_ptr, c_ptr]),
    "cn_euler_chain_bwd": (c_i32, [c_i32, c_i32, c_ptr, c_i64, c_ptr, c_i64, c_ptr, c_ptr, c_ptr, c_ptr, c_ptr]),
    "cn_coarse_z": (c_i32, [c_i32, c_i32, c_ptr, c_ptr, c_ptr, c_ptr, c_ptr]),
    "cn_uniform_philox": (c_i32, [c_i64, c_ptr, c_ptr, c_ptr]),
    "cn_points": (c_i32, [c_i32, c_i32, c_ptr, c_ptr, c_ptr, c_ptr, c_i32, c_ptr, c_ptr, c_i32, c_ptr, c_ptr]),
    "cn_up_sample_merge": (c_i32, [c_i32, c_i32, c_i32, c_f32, c_ptr, c_ptr, c_ptr, c_ptr, c_ptr, c_ptr,
                                   c_ptr]),
    "cn_composite_fwd": (c_i32, [c_i32, c_i32, c_ptr, c_ptr, c_ptr, c_i64, c_ptr, c_ptr, c_ptr, c_ptr, c_ptr,
                                 c_i32, c_ptr, c_ptr, c_ptr, c_ptr, c_ptr, c_ptr]),
    "cn_composite_bwd": (c_i32, [c_i32, c_i32, c_ptr, c_ptr, c_ptr, c_i64, c_ptr, c_ptr, c_ptr, c_ptr, c_ptr,
                                 c_i32, c_ptr, c_ptr, c_ptr, c_ptr, c_ptr, c_ptr, c_ptr, c_ptr, c_ptr,
                                 c_ptr, c_ptr]),
    "cn_points_bwd": (c_i32, [c_i32, c_i32, c_ptr, c_i32, c_ptr, c_ptr, c_i32, c_ptr, c_i64, c_ptr, c_ptr,
                              c_ptr]),
    "cn_color_extras_bwd": (c_i32, [c_i32, c_i32, c_ptr, c_i64, c_ptr, c_i64, c_i32, c_ptr, c_i32, c_ptr]),
    "cn_train_loss_workspace_bytes": (ctypes.c_size_t, [c_i32, c_i32]),
    "cn_train_loss": (c_i32, [c_i32, c_i32, c_i64, c_ptr, c_ptr, c_ptr, c_ptr, c_i64, c_ptr, c_f32, c_ptr, c_ptr,
                              c_ptr, c_ptr, c_i64, c_ptr, c_ptr, c_i64, c_ptr]),
    "cn_stage1_workspace_bytes": (ctypes.c_size_t, [c_i32]),
    "cn_stage1_fwd": (c_i32, [c_i32, c_i32, c_ptr, c_i64, c_ptr, c_i64, c_ptr, c_i64, c_ptr, c_ptr, c_ptr, c_f32,
                              c_ptr, c_ptr, c_i64, c_ptr, c_ptr, c_ptr]),
    "cn_stage1_bwd": (c_i32, [c_i32, c_i32, c_ptr, c_i64, c_ptr, c_i64, c_ptr, c_i64, c_ptr, c_ptr, c_ptr, c_ptr,
                              c_ptr, c_ptr, c_i64, c_ptr, c_i64, c_ptr, c_i64, c_ptr, c_ptr, c_i64, c_ptr, c_ptr,
                              c_ptr]),
    "cn_mat4_chain_fwd": (c_i32, [c_i32, c_ptr, c_ptr, c_ptr]),
    "cn_mat4_chain_bwd": (c_i32, [c_i32, c_ptr, c_ptr, c_ptr, c_ptr, c_ptr]),
    "cn_sdf_mlp": (c_i32, [ctypes.POINTER(SdfMlpDesc), c_ptr]),
    "cn_sdf_query_workspace_bytes": (ctypes.c_size_t, [ctypes.POINTER(SdfNet), c_i32]),
    "cn_sdf_query": (c_i32, [ctypes.POINTER(SdfNet), c_i32, c_ptr, c_i64, c_ptr, c_ptr, c_ptr, c_i64, c_ptr]),
    "cn_sample_workspace_bytes": (ctypes.c_size_t, [ctypes.POINTER(SampleDesc)]),
    "cn_sample": (c_i32, [ctypes.POINTER(SampleDesc), c_ptr, c_i64, c_ptr]),
    "cn_render_fwd_workspace_bytes": (ctypes.c_size_t, [ctypes.POINTER(RenderDesc)]),
    "cn_render_fwd": (c_i32, [ctypes.POINTER(RenderDesc), c_ptr, c_i64, c_ptr]),
    "cn_render_state_bytes": (ctypes.c_size_t, [ctypes.POINTER(RenderDesc)]),
    "cn_render_bwd_workspace_bytes": (ctypes.c_size_t, [ctypes.POINTER(RenderDesc), c_i32]),
    "cn_render_train_fwd": (c_i32, [ctypes.POINTER(RenderDesc), c_ptr, c_i64, c_ptr]),
    "cn_render_bwd": (c_i32, [ctypes.POINTER(RenderDesc), ctypes.POINTER(RenderGrads), c_ptr, c_i64, c_ptr, c_i64, c_ptr]),
    "cn_mlp_state_bytes": (ctypes.c_size_t, [ctypes.POINTER(MlpDesc)]),
    "cn_mlp_bwd_workspace_bytes": (ctypes.c_size_t, [ctypes.POINTER(MlpDesc)]),
    "cn_mlp_fwd": (c_i32, [ctypes.POINTER(MlpDesc), c_ptr, c_i64, c_ptr]),
    "cn_mlp_bwd": (c_i32, [ctypes.POINTER(MlpDesc), c_ptr, c_i64, c_ptr, c_i64, c_ptr]),
}

_lock = threading.Lock()
_lib = None
_load_error: str | None = None


class LibraryMissing(RuntimeError):
    pass


def load(path: str | None = None):
    """Load (once) and return the ctypes handle; raise LibraryMissing if absent."""
    global _lib, _load_error
    with _lock:
        if _lib is not None:
            return _lib
        p = path or LIB_PATH
        if not os.path.exists(p):
            _load_error = f"{p} not found: build it with `python -c 'import __graft_entry__ as g; g.build()'`"
            raise LibraryMissing(_load_error)
        try:
            lib = ctypes.CDLL(p)
        except OSError as e:  # pragma: no cover - depends on the loader
            _load_error = f"cannot load {p}: {e}"
            raise LibraryMissing(_load_error) from e
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        v = lib.cn_abi_version()
        if v != ABI_VERSION:
            raise LibraryMissing(f"{p}: ABI version {v}, expected {ABI_VERSION}")
        _lib = lib
        return lib


def check(rc: int, name: str) -> None:
    if rc != 0:
        msg = load().cn_last_error()
        raise RuntimeError(f"{name} failed ({rc}): {msg.decode() if msg else ''}")


def call(name: str, *args) -> None:
    lib = load()
    check(getattr(lib, name)(*args), name)


_KEY_PLANS = {}


def _key_plan(T):
    """Per descriptor type: the 8-byte words of its pointer fields (plain and in arrays) and its nested
    descriptor pointers (name, word).  Every other field is a scalar or an array of scalars, compared by its
    bytes (ctypes zero-fills a new structure, padding included)."""
    plan = _KEY_PLANS.get(T)
    if plan is None:
        words, nested = [], []
        for name, typ in T._fields_:
            off = getattr(T, name).offset
            if typ is c_ptr:
                assert off % 8 == 0
                words.append(off // 8)
            elif issubclass(typ, ctypes.Array) and typ._type_ is c_ptr:
                assert off % 8 == 0
                words.extend(off // 8 + i for i in range(typ._length_))
            elif issubclass(typ, ctypes._Pointer):
                assert off % 8 == 0 and issubclass(typ._type_, ctypes.Structure)
                nested.append((name, off // 8))
            else:
                assert issubclass(typ, ctypes._SimpleCData) or (issubclass(typ, ctypes.Array) and
                                                                issubclass(typ._type_, ctypes._SimpleCData)), name
        assert ctypes.sizeof(T) % 8 == 0
        plan = _KEY_PLANS[T] = (np.array(words + [w for _, w in nested], dtype=np.int64), nested)
    return plan


def shape_key(st):
    """What a composed entry point's sizing pass reads of a descriptor: every scalar field, every pointer
    field only as present / absent (the planners see no pointer values -- a buffer's existence is a flag),
    nested descriptors (networks) likewise.  Equal keys give equal workspace / state sizes, so the host
    plans a shape once (ops._sized) instead of on every call.  The key is the structure's bytes with each
    pointer word replaced by its presence (a field-by-field walk cost ~140 us per render descriptor)."""
    words, nested = _key_plan(type(st))
    a = np.frombuffer(bytearray(st), dtype=np.uint64)
    a[words] = a[words] != 0
    sub = tuple(shape_key(getattr(st, name).contents) if a[w] else None for name, w in nested)
    return (type(st).__name__, a.tobytes(), sub)
