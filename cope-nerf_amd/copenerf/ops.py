"""Tensor-level wrappers over the C ABI (one function per entry point).

Every wrapper checks device, dtype and layout on the host, then launches on
torch's current HIP stream.  Buffers are plain 2-D fp32 row-major tensors whose
leading dimension (stride(0)) is passed explicitly, so column views such as
``buf[:, :256]`` can be handed over without copies.
"""
from __future__ import annotations

import ctypes
import math

import torch

from . import _lib
from ._lib import (EPI_BWD_RELU, EPI_BWD_SOFTPLUS, EPI_MUL, EPI_RELU, EPI_SOFTPLUS, EPI_SOFTPLUS_HEAD,  # noqa: F401
                   EPI_STORE, EPI_TANGENT)

SQRT2 = float(math.sqrt(2.0))  # torch's x / np.sqrt(2) divides by the fp32 rounding of this


class KernelTimer:
    """Brackets cn_linear / cn_wgrad launches with HIP events on the launching
    stream (torch's current stream) and keeps (key, events, algorithmic FLOPs)."""

    def __init__(self, detail=False):
        self.records = []
        self.detail = detail  # key launches by shape as well
        self.symbols = {}  # launch class -> rocprofv3 symbol of its kernel (named by the library)

    def start(self):
        e = torch.cuda.Event(enable_timing=True)
        e.record()
        return e

    def stop(self, key, e0, flops, nbytes=0.0):
        e1 = torch.cuda.Event(enable_timing=True)
        e1.record()
        self.records.append((key, e0, e1, flops, nbytes))

    def summary(self):
        torch.cuda.synchronize()
        agg = {}
        for key, e0, e1, fl, nb in self.records:
            a = agg.setdefault(key, {"launches": 0, "ms": 0.0, "flops": 0.0, "bytes": 0.0})
            a["launches"] += 1
            a["ms"] += e0.elapsed_time(e1)
            a["flops"] += fl
            a["bytes"] += nb
        return agg


_timer = None
# cn_linear_desc.flags bit 0 alternated launch to launch (the memory-side cache holds the last
# rows a layer wrote when the next one starts; see include/copenerf.h)
_flip = 0
EPI_NAMES = {0: "store", 1: "softplus", 2: "relu", 3: "mul", 4: "tangent", 5: "bwd_softplus", 6: "bwd_relu",
             8: "softplus_head"}


def set_kernel_timer(t):
    global _timer
    _timer = t


def rup(x: int, m: int) -> int:
    return (x + m - 1) // m * m


def _ptr(t):
    return None if t is None else t.data_ptr()


def _stream():
    return torch.cuda.current_stream().cuda_stream


def _need(t, name, *, ndim=2):
    if t is None:
        return
    if not t.is_cuda:
        raise RuntimeError(f"copenerf: {name} must be a CUDA/HIP tensor (got {t.device}); "
                           "the HIP kernels have no CPU fallback")
    if t.dtype not in (torch.float32, torch.int32, torch.bfloat16):
        raise RuntimeError(f"copenerf: {name} must be float32 (got {t.dtype})")
    if ndim == 2 and (t.dim() != 2 or t.stride(1) != 1):
        raise RuntimeError(f"copenerf: {name} must be a row-major 2-D tensor (shape {tuple(t.shape)}, "
                           f"strides {t.stride()})")


def _ld(t):
    return 0 if t is None else t.stride(0)


def split_bf16x3(W: torch.Tensor) -> torch.Tensor:
    """[N, K] fp32 (K % 16 == 0) -> the chunk-major B image of
    CN_MFMA_F32_BF16X6, bf16 [K/16, N, 48]: entry [c, n, 16 t + j] is term t of
    W[n, 16 c + j], with W = w0 + w1 + w2 (each the RNE bf16 of the remainder;
    |W - Σ| <= 2^-27 |W|)."""
    N, K = W.shape
    if K % 16:
        raise ValueError(f"split_bf16x3: K={K} must be a multiple of 16")
    w0 = W.to(torch.bfloat16)
    r = W - w0.float()
    w1 = r.to(torch.bfloat16)
    w2 = (r - w1.float()).to(torch.bfloat16)
    t = torch.stack([w0, w1, w2], 1).view(N, 3, K // 16, 16)
    return t.permute(2, 0, 1, 3).reshape(K // 16, N, 48).contiguous()


def unsplit_bf16x3(B: torch.Tensor) -> torch.Tensor:
    """The three terms [3, N, K] (bf16) of a split_bf16x3 image."""
    C, N, _ = B.shape
    return B.view(C, N, 3, 16).permute(2, 1, 0, 3).reshape(3, N, C * 16)


FORMATS = {"fp32": 0, "bf16": 1, "bf16x6": 2}


def weight_norm_batch(vs, gs, *, dws=None):
    """cn_weight_norm over lists of (v [rows, cols], g [rows, 1] or [rows]) in one launch:
    forward -> [W]; with dws (the gradients of the W) -> ([dv], [dg])."""
    jobs = (_lib.WnJob * max(1, len(vs)))()
    outs = []
    for i, (v, g) in enumerate(zip(vs, gs)):
        _need(v, "v")
        if not v.is_contiguous() or not g.is_contiguous() or g.numel() != v.shape[0]:
            raise RuntimeError("weight_norm_batch: v [rows, cols] and g [rows] must be contiguous")
        j = jobs[i]
        j.v, j.g, j.rows, j.cols = v.data_ptr(), g.data_ptr(), v.shape[0], v.shape[1]
        if dws is None:
            w = torch.empty_like(v)
            j.w = w.data_ptr()
            outs.append(w)
        else:
            dw = dws[i].contiguous()
            dv, dg = torch.empty_like(v), torch.empty_like(g)
            j.dw, j.dv, j.dg = dw.data_ptr(), dv.data_ptr(), dg.data_ptr()
            outs.append((dv, dg, dw))
    _lib.check(_lib.load().cn_weight_norm(jobs, len(vs), 0 if dws is None else 1, _stream()), "cn_weight_norm")
    if dws is None:
        return outs
    return [o[0] for o in outs], [o[1] for o in outs]


class ImagePacker:
    """Collects cn_pack_job regions of weight images and builds them in one
    cn_pack_weights launch (the per-call weight packing of fields.py)."""

    def __init__(self, mode: str):
        if mode not in FORMATS:
            raise ValueError(f"mode must be one of {tuple(FORMATS)} (got {mode!r})")
        self.mode = mode
        self.jobs = []
        self.keep = []  # sources must stay alive until the launch is queued

    def image(self, rows: int, cols: int, device, fmt: str | None = None) -> torch.Tensor:
        """An uninitialised image of the packer's format: fp32 / bf16 [rows, cols], bf16x6 the
        chunk-major [cols/16, rows, 48] (split_bf16x3's layout)."""
        fmt = fmt or self.mode
        if fmt == "bf16x6":
            if cols % 16:
                raise ValueError(f"pack: bf16x6 image width {cols} must be a multiple of 16")
            return torch.empty(cols // 16, rows, 48, device=device, dtype=torch.bfloat16)
        return torch.empty(rows, cols, device=device, dtype=torch.bfloat16 if fmt == "bf16" else torch.float32)

    def put(self, dst: torch.Tensor, src: torch.Tensor, *, transpose=False, r0=0, r1=None, c0=0, c1=None, fmt=None):
        """Region [r0, r1) x [c0, c1) of dst (default: all of it) = src (or srcᵀ) at (r0, c0), zero elsewhere."""
        fmt = fmt or self.mode
        _need(src, "pack src")
        _need(dst, "pack dst", ndim=dst.dim())
        if src.dtype != torch.float32:
            raise RuntimeError("pack: src must be float32")
        rows, cols = (src.shape[1], src.shape[0]) if transpose else (src.shape[0], src.shape[1])
        j = _lib.PackJob()
        j.src, j.dst = src.data_ptr(), dst.data_ptr()
        j.src_ld = src.stride(0)
        x6 = fmt == "bf16x6"
        d_rows, d_cols = (dst.shape[1], 16 * dst.shape[0]) if x6 else (dst.shape[0], dst.shape[1])
        j.dst_ld = d_rows if x6 else d_cols
        j.rows, j.cols = rows, cols
        j.r0, j.r1 = r0, d_rows if r1 is None else r1
        j.c0, j.c1 = c0, d_cols if c1 is None else c1
        j.transpose, j.format = int(transpose), FORMATS[fmt]
        self.jobs.append(j)
        self.keep.append(src)
        return dst

    def run(self):
        if self.jobs:
            arr = (_lib.PackJob * len(self.jobs))(*self.jobs)
            _lib.check(_lib.load().cn_pack_weights(arr, len(self.jobs), _stream()), "cn_pack_weights")
        self.jobs, self.keep = [], []


# launch-class tags of the kernel timer: linear_kernel<WM, WN, TM, TN, BK, OCC, DEPTH, ...> arguments
# (named by the library itself, cn_linear_kernel_name) -> a short tile name
_TILE_TAGS = {"4, 2, 2, 4, 16, 1, 2": "sq", "4, 2, 1, 4, 32, 1, 2": "tall", "4, 2, 2, 2, 32, 1, 2": "wide",
              "2, 2, 2, 2, 16, 2, 2": "t128", "4, 1, 1, 2, 16, 2, 2": "t1", "4, 2, 2, 4, 32, 1, 2": "sq",
              "2, 2, 2, 2, 64, 2, 1": "t128", "4, 1, 1, 2, 64, 2, 1": "t1"}


def kernel_name(query, d) -> str:
    """The rocprofv3 symbol of the kernel a cn_linear / cn_wgrad descriptor launches, as the
    library decides it (cn_linear_kernel_name / cn_wgrad_kernel_name)."""
    buf = ctypes.create_string_buffer(256)
    n = query(d, buf, 256)
    if n < 0:
        raise RuntimeError(f"kernel name query failed ({n}): {_lib.load().cn_last_error().decode()}")
    return buf.value.decode()


def _tile_tag(name, tile):
    args = name[name.index("<") + 1:].split(", ")[:7]
    return _TILE_TAGS.get(", ".join(args), tile)


def linear(A, B, N, K, out0, epilogue, *, bias=None, A2=None, K1=None, rowv=None, colv=None, aux0=None,
           aux1=None, aux2=None, out_split=None, nsplit=None, nzero=None, adiv=1.0, odiv=1.0, beta=100.0,
           threshold=20.0, aux_beta=0.0, aux2_scale=0.0, tile=None, M=None, kalg=None, out1=None, head_w=None,
           head_b=None, head_out=None, head_idx=None, out0_b=None, out1_b=None):
    """out = epilogue((A|A2) @ B[:N].T / adiv) -- cn_linear.  MUL / TANGENT /
    BWD_SOFTPLUS read softplus' as sg = 1 - exp(-aux_beta * aux0) from the stored
    softplus output aux0 (include/copenerf.h).  kalg: the unpadded
    inner dimension (for the FLOP count of the kernel timer only).  A bfloat16 B
    selects the bf16 MFMA path (A rounded to bf16 on load, fp32 accumulate); K is
    then rounded up to 64, so A's columns up to that must exist (zero padding).
    A [K/16, N, 48] bfloat16 B (split_bf16x3) selects CN_MFMA_F32_BF16X6: the fp32
    GEMM computed from three bf16 terms per operand on the bf16 MFMA.
    EPI_SOFTPLUS_HEAD (the last SDF hidden layer): out0 = softplus activation (or
    None: not stored), out1 = colv * softplus' (or None), head_out[head_idx[m] or m]
    = out0[m] · head_w + head_b.
    tile: None (the library's choice), 1 (128x64), 2 (128x128 only: tests compare the tiles).
    bf16 operand images (bf16 MFMA mode only, ABI v10): A (with A2) may be bfloat16 -- the rounded
    operand itself, read instead of rounded on load; aux0 may be bfloat16 for BWD_RELU (its sign) and
    for MUL / TANGENT / BWD_SOFTPLUS (the activation σ is recovered from), BWD_SOFTPLUS's aux1 / aux2
    too (all three in one dtype);
    out0_b / out1_b (bfloat16, or None) receive the RNE bf16 image of every value written to out0 /
    out1, and out0 may then be None."""
    x6 = B.dim() == 3
    if x6 and (B.dtype != torch.bfloat16 or B.shape[2] != 48 or not B.is_contiguous()):
        raise RuntimeError(f"cn_linear: a 3-D B must be split_bf16x3's [K/16, N, 48] bfloat16 image (got "
                           f"{tuple(B.shape)}, {B.dtype}, strides {B.stride()})")
    if out0 is None and out0_b is None and epilogue != EPI_SOFTPLUS_HEAD:
        raise RuntimeError("cn_linear: out0 (or out0_b) is required")
    bf = B.dtype == torch.bfloat16 and not x6
    for t, n in ((A, "A"), (A2, "A2"), (B, "B"), (out0, "out0"), (aux0, "aux0"), (aux1, "aux1"), (aux2, "aux2"),
                 (out_split, "out_split"), (out1, "out1"), (out0_b, "out0_b"), (out1_b, "out1_b")):
        _need(t, n, ndim=3 if (x6 and t is B) else 2)
        if t is None or t is B:
            continue
        want_b = n in ("out0_b", "out1_b")
        may_b = bf and (n in ("A", "A2") or
                        (n == "aux0" and epilogue in (EPI_BWD_RELU, EPI_MUL, EPI_TANGENT, EPI_BWD_SOFTPLUS)) or
                        (n in ("aux1", "aux2") and epilogue == EPI_BWD_SOFTPLUS))
        if (t.dtype == torch.bfloat16) != want_b and not (may_b and t.dtype == torch.bfloat16):
            raise RuntimeError(f"cn_linear: {n} has dtype {t.dtype} (bfloat16 images: A / A2, the aux0 of MUL / "
                               f"TANGENT / BWD_SOFTPLUS / BWD_RELU, BWD_SOFTPLUS's aux1 / aux2 and out0_b / out1_b, "
                               f"in the bf16 MFMA mode only)")
    a_b = A.dtype == torch.bfloat16
    if A2 is not None and (A2.dtype == torch.bfloat16) != a_b:
        raise RuntimeError("cn_linear: A and A2 must have the same dtype")
    if aux1 is not None and aux2 is not None and aux1.dtype != aux2.dtype:
        raise RuntimeError("cn_linear: aux1 and aux2 must have the same dtype")
    if aux1 is not None and aux0 is not None and aux1.dtype != aux0.dtype:
        raise RuntimeError("cn_linear: BWD_SOFTPLUS's aux0, aux1 and aux2 must have the same dtype")
    if bf:
        K = rup(K, 64)
        K1 = rup(K1, 64) if K1 is not None else None
        if (A.stride(0) < (K1 or K)) or (A2 is not None and A2.stride(0) < K - K1):
            raise RuntimeError(f"cn_linear (bf16): A rows too short for K={K}")
    M = A.shape[0] if M is None else M
    # the epilogue reads bias / colv as float4
    bias = bias if bias is None or bias.data_ptr() % 16 == 0 else bias.clone()
    colv = colv if colv is None or colv.data_ptr() % 16 == 0 else colv.clone()
    if tile is None:
        tile = 1 if max(N, nzero or 0) <= 64 else 0
    bn = 64 if tile == 1 else 128
    b_rows, b_k = (B.shape[1], 16 * B.shape[0]) if x6 else (B.shape[0], B.shape[1])
    if b_rows < rup(N, bn) or b_k < K:
        raise RuntimeError(f"cn_linear: B {tuple(B.shape)} too small for N={N}, K={K} (tile {tile})")
    if any(t is not None and t.shape[0] < M for t in (out0, out1, out0_b, out1_b)):
        raise RuntimeError("cn_linear: an output has fewer rows than A")
    if epilogue == EPI_SOFTPLUS_HEAD:
        _need(head_w, "head_w", ndim=1)
        _need(head_b, "head_b", ndim=1)
        _need(head_out, "head_out", ndim=1)
        if not head_out.is_contiguous():
            raise RuntimeError("cn_linear: head_out must be contiguous")
        if head_w.numel() < N or head_w.stride(0) != 1:
            raise RuntimeError("cn_linear: head_w must be a contiguous [N] vector")
        if head_idx is None and head_out.numel() < M:
            raise RuntimeError("cn_linear: head_out has fewer than M elements")
        if head_idx is not None and (head_idx.dtype != torch.int32 or head_idx.numel() < M):
            raise RuntimeError("cn_linear: head_idx must be int32 with M elements")
        head_w = head_w if head_w.data_ptr() % 16 == 0 else head_w.clone()
    d = _lib.LinearDesc()
    d.A, d.A2, d.B, d.bias = _ptr(A), _ptr(A2), _ptr(B), _ptr(bias)
    d.rowv, d.colv, d.aux0, d.aux1 = _ptr(rowv), _ptr(colv), _ptr(aux0), _ptr(aux1)
    d.out0, d.out1, d.out_split = _ptr(out0), _ptr(out1), _ptr(out_split)
    d.head_w, d.head_b, d.head_out, d.head_idx = _ptr(head_w), _ptr(head_b), _ptr(head_out), _ptr(head_idx)
    d.aux2, d.ld_aux2 = _ptr(aux2), _ld(aux2)
    d.aux_beta, d.aux2_scale = aux_beta, aux2_scale
    d.lda, d.lda2, d.ldb = _ld(A), _ld(A2), (B.shape[1] if x6 else _ld(B))
    d.ld_aux0, d.ld_aux1, d.ld_out0, d.ld_out1, d.ld_split = _ld(aux0), _ld(aux1), _ld(out0), _ld(out1), _ld(out_split)
    d.M, d.N, d.K = M, N, K
    d.K1 = K1 if K1 is not None else K
    d.nzero = nzero if nzero is not None else N
    d.nsplit = nsplit if nsplit is not None else N
    d.epilogue, d.tile = epilogue, tile
    d.adiv, d.odiv, d.beta, d.threshold = adiv, odiv, beta, threshold
    d.mfma_dtype = 2 if x6 else (1 if bf else 0)
    d.a_bf16 = 1 if a_b else 0
    d.aux0_bf16 = 1 if (aux0 is not None and aux0.dtype == torch.bfloat16) else 0
    d.aux12_bf16 = 1 if (aux1 is not None and aux1.dtype == torch.bfloat16) else 0
    d.out0_b, d.ld_out0_b, d.out1_b, d.ld_out1_b = _ptr(out0_b), _ld(out0_b), _ptr(out1_b), _ld(out1_b)
    global _flip
    _flip ^= 1  # consecutive launches walk the rows in opposite directions
    d.flags = _flip
    if _timer is not None:
        e0 = _timer.start()
        _lib.check(_lib.load().cn_linear(d, _stream()), "cn_linear")
        name = kernel_name(_lib.load().cn_linear_kernel_name, d)
        tag = _tile_tag(name, tile) if (x6 or bf) else tile
        key = ("linear", tag, EPI_NAMES[epilogue] + ("+rowv" if rowv is not None else "") +
               ("+imgA" if a_b else "")) + (("bf16",) if bf else ("x6",) if x6 else ())
        _timer.symbols[key] = name
        ka = kalg or K
        # algorithmic HBM bytes: A (unpadded K) and every aux row read once, each output
        # element written once, the weight image once (bf16x6: 3 bf16 terms per weight)
        nb = (2.0 if a_b else 4.0) * M * ka + (6.0 if x6 else 2.0 if bf else 4.0) * N * ka
        nb += M * N * sum(t.element_size() for t in (out0, out1, aux0, aux1, aux2, out0_b, out1_b) if t is not None)
        nb += 4.0 * M * ((rowv is not None) + (head_out is not None) + (head_idx is not None))
        _timer.stop(key + ((M, N, K),) if _timer.detail else key, e0, 2.0 * M * N * ka, nb)
    else:
        _lib.check(_lib.load().cn_linear(d, _stream()), "cn_linear")
    return out0


WGRAD_MODES = {"fp32": 0, "bf16": 1, "bf16x6": 2}


def _wgrad_desc(Y0, X0, N, K, dW, db, Y1, X1, accumulate, mode, workspace=True):
    """The cn_wgrad descriptor of one weight gradient and the workspace it points into (workspace=False:
    none yet -- cn_wgrad_batch callers carve every job's slabs out of one buffer).  A bfloat16 Y0 / X0
    (with Y1 / X1 of the same dtype) is a bf16 operand image (bf16 mode)."""
    if mode not in WGRAD_MODES:
        raise ValueError(f"wgrad: mode must be one of {tuple(WGRAD_MODES)} (got {mode!r})")
    for t, n in ((Y0, "Y0"), (X0, "X0"), (Y1, "Y1"), (X1, "X1"), (dW, "dW")):
        _need(t, n)
    yb, xb = Y0.dtype == torch.bfloat16, X0.dtype == torch.bfloat16
    if (Y1 is not None and (Y1.dtype == torch.bfloat16) != yb) or (X1 is not None and (X1.dtype == torch.bfloat16) != xb):
        raise RuntimeError("wgrad: Y0 / Y1 and X0 / X1 must have the same dtype")
    if (yb or xb) and mode != "bf16":
        raise RuntimeError("wgrad: bfloat16 operand images only in the bf16 mode")
    M = Y0.shape[0]
    lib = _lib.load()
    ws = None
    d = _lib.WgradDesc()
    if workspace:
        nbytes = lib.cn_wgrad_workspace_bytes(M, N, K)
        ws = torch.empty(nbytes // 4 + 1, device=Y0.device, dtype=torch.float32)
        d.workspace, d.workspace_bytes = _ptr(ws), ws.numel() * 4
    d.Y0, d.X0, d.Y1, d.X1 = _ptr(Y0), _ptr(X0), _ptr(Y1), _ptr(X1)
    d.dW, d.db = _ptr(dW), _ptr(db)
    d.ldy0, d.ldx0, d.ldy1, d.ldx1, d.ld_dw = _ld(Y0), _ld(X0), _ld(Y1), _ld(X1), _ld(dW)
    d.M, d.N, d.K = M, N, rup(K, 64)
    d.npairs = 2 if Y1 is not None else 1
    d.n_out, d.k_out = dW.shape[0], dW.shape[1]
    d.accumulate = 1 if accumulate else 0
    d.mfma_dtype = WGRAD_MODES[mode]
    d.y_bf16, d.x_bf16 = int(yb), int(xb)
    return d, ws


def _wgrad_bytes(d, ops_):
    """Algorithmic HBM bytes of a weight gradient: every operand row read once."""
    Y0, X0 = ops_[0], ops_[1]
    return float(d.npairs * d.M * (d.n_out * Y0.element_size() + d.k_out * X0.element_size()))


def _wgrad_key(d, mode):
    # one launch class per kernel instance (1- and 2-pair calls share it, as in rocprof's stats)
    name = kernel_name(_lib.load().cn_wgrad_kernel_name, d)
    key = ("wgrad", name[len("void cn::"):name.index("(")].replace(" ", "")) + \
        (("bf16",) if mode == "bf16" else ("x6",) if mode == "bf16x6" else ())
    _timer.symbols[key] = name
    return key


def wgrad(Y0, X0, N, K, dW, *, db=None, Y1=None, X1=None, accumulate=False, mode="fp32"):
    """dW[:n_out, :k_out] (+)= Y0ᵀX0 (+ Y1ᵀX1), db = colsum(Y0) -- cn_wgrad.
    mode: "fp32" (exact fp32 MFMA), "bf16x6" (fp32 from three bf16 terms per
    operand on the bf16 MFMA) or "bf16" (operands rounded to bf16 on load,
    config C3's reduced-precision mode; Y / X may then be bfloat16 operand images)."""
    d, ws = _wgrad_desc(Y0, X0, N, K, dW, db, Y1, X1, accumulate, mode)
    lib = _lib.load()
    if _timer is not None:
        e0 = _timer.start()
        _lib.check(lib.cn_wgrad(d, _stream()), "cn_wgrad")
        key = _wgrad_key(d, mode)
        M = d.M
        _timer.stop(key + ((M, d.n_out, d.k_out),) if _timer.detail else key, e0,
                    2.0 * M * d.n_out * d.k_out * d.npairs, _wgrad_bytes(d, (Y0, X0)))
    else:
        _lib.check(lib.cn_wgrad(d, _stream()), "cn_wgrad")
    return dW


class WgradQueue(object):
    """Collects a backward pass's 256x256 stage-ring weight gradients and runs them with ONE
    cn_wgrad_batch call at flush(): one launch and one slab reduction instead of a launch, a
    full-chip slab write and a reduction each (other tile classes launch at add()).  The
    queue holds the operand tensors, so their memory stays allocated until the flush; the
    gradients are written by the flush (call it before anything reads them).  Every job's slabs
    come out of one workspace allocated at the flush, sized by the batch's own layout
    (cn_wgrad_batch_workspace_bytes: each job's share of the slices, not a full launch's)."""

    def __init__(self):
        self.jobs = []

    def add(self, Y0, X0, N, K, dW, *, db=None, Y1=None, X1=None, mode="fp32"):
        d, _ = _wgrad_desc(Y0, X0, N, K, dW, db, Y1, X1, False, mode, workspace=False)
        if "WgradBatch" not in kernel_name(_lib.load().cn_wgrad_kernel_name, d):
            # not a stage-ring job (e.g. K = 64 first layers): nothing to share, launch it now
            return wgrad(Y0, X0, N, K, dW, db=db, Y1=Y1, X1=X1, mode=mode)
        self.jobs.append((d, mode, (Y0, X0, Y1, X1)))
        return dW

    def flush(self):
        if not self.jobs:
            return
        # the batch layout (each job's share of the CUs) and the stream are the jobs' device's
        with torch.cuda.device(self.jobs[0][2][0].device):
            self._flush()

    def _flush(self):
        lib = _lib.load()
        n = len(self.jobs)
        arr = (_lib.WgradDesc * n)(*[d for d, _, _ in self.jobs])
        offs = (ctypes.c_int64 * n)()
        total = lib.cn_wgrad_batch_workspace_bytes(arr, n, offs)
        ws = torch.empty(total // 4 + 1, device=self.jobs[0][2][0].device, dtype=torch.float32)
        base = ws.data_ptr()
        for i in range(n):
            arr[i].workspace = base + offs[i]
            arr[i].workspace_bytes = total - offs[i]
        if _timer is not None:
            # the batch's time goes to the class of its first job; the FLOPs of all of them
            e0 = _timer.start()
            _lib.check(lib.cn_wgrad_batch(arr, n, _stream()), "cn_wgrad_batch")
            key = _wgrad_key(self.jobs[0][0], self.jobs[0][1])
            fl = sum(2.0 * d.M * d.n_out * d.k_out * d.npairs for d, _, _ in self.jobs)
            nb = sum(_wgrad_bytes(d, t) for d, _, t in self.jobs)
            _timer.stop(key + (("batch", n),) if _timer.detail else key, e0, fl, nb)
        else:
            _lib.check(lib.cn_wgrad_batch(arr, n, _stream()), "cn_wgrad_batch")
        self.jobs = []


def row_head(A, K, W, b, C, act, out, dst_index=None, ld_out=None):
    """out[dst(m)*ld_out + c] = act(A[m] . W[c] + b[c]); ld_out defaults to C (out [M, C])."""
    _need(A, "A")
    _need(W, "W")
    if dst_index is not None and (dst_index.dtype != torch.int32 or not dst_index.is_contiguous()):
        raise RuntimeError("row_head: dst_index must be contiguous int32")
    if not out.is_contiguous():
        raise RuntimeError("row_head: out must be contiguous")
    _lib.call("cn_row_head", A.shape[0], K, _ptr(A), _ld(A), _ptr(W), _ld(W), _ptr(b), C, act, _ptr(out),
              C if ld_out is None else ld_out, _ptr(dst_index), _stream())
    return out


def scale_cols(X, N, w, out, act_beta=0.0, rowv=None):
    """out = f(X) * w (* rowv[m]); f(X) = X (act_beta 0) or 1 - exp(-act_beta X): softplus'
    of stored activations."""
    _need(X, "X")
    _need(out, "out")
    if rowv is not None and (not rowv.is_contiguous() or rowv.numel() != X.shape[0]):
        raise RuntimeError("scale_cols: rowv must be a contiguous [M] tensor")
    _lib.call("cn_scale_cols", X.shape[0], N, _ptr(X), _ld(X), _ptr(w), _ptr(rowv), _ptr(out), _ld(out),
              float(act_beta), _stream())
    return out


def softplus_adjoint(act, N, out, *, act_beta, D=None, rowv=None, colv=None, aux1=None, aux2=None, aux2_scale=0.0,
                     cs_out=None, rs_out=None, cs_div=1.0):
    """out = (D + rowv (x) colv) * sg(act) + aux1 * aux2 * aux2_scale * (1 - sg) / sg -- cn_softplus_adjoint;
    cs_out[n] = Σ_m (rowv[m] act[m][n] + aux2[m][n]) / cs_div when given (lin8's sdf-row gradient),
    rs_out[0] = Σ_m rowv[m] / cs_div (its bias gradient)."""
    for t, n in ((act, "act"), (out, "out"), (D, "D"), (aux1, "aux1"), (aux2, "aux2")):
        _need(t, n)
        if t is not None and t.dtype not in (torch.float32, torch.bfloat16):
            raise RuntimeError(f"softplus_adjoint: {n} must be float32 or a bfloat16 operand image")
    if aux1 is not None and aux2 is not None and aux1.dtype != aux2.dtype:
        raise RuntimeError("softplus_adjoint: aux1 and aux2 must have the same dtype")
    isb = lambda t: t is not None and t.dtype == torch.bfloat16  # noqa: E731
    in_bf16 = (1 if isb(D) else 0) | (2 if isb(act) else 0) | (4 if isb(aux1) else 0)
    if rowv is not None and (not rowv.is_contiguous() or rowv.numel() != act.shape[0]):
        raise RuntimeError("softplus_adjoint: rowv must be a contiguous [M] tensor")
    M = act.shape[0]
    ws = None
    if cs_out is not None:
        _need(cs_out, "cs_out", ndim=1)
        if not cs_out.is_contiguous() or cs_out.numel() < N:
            raise RuntimeError("softplus_adjoint: cs_out must be a contiguous [N] tensor")
        lib = _lib.load()
        ws = torch.empty(lib.cn_softplus_adjoint_workspace_bytes(M, N) // 4 + 1, device=act.device, dtype=torch.float32)
    _lib.call("cn_softplus_adjoint", M, N, _ptr(D), _ld(D), _ptr(act), _ld(act), float(act_beta),
              _ptr(rowv), _ptr(colv), _ptr(aux1), _ld(aux1), _ptr(aux2), _ld(aux2), float(aux2_scale), _ptr(out),
              _ld(out), int(out.dtype == torch.bfloat16), in_bf16, _ptr(cs_out),
              _ptr(rs_out if cs_out is not None else None), float(cs_div), _ptr(ws),
              0 if ws is None else ws.numel() * 4, _stream())
    return out


def colsum(X, K, out, *, w=None, wdiv=1.0, accumulate=False):
    _need(X, "X")
    M = X.shape[0]
    lib = _lib.load()
    ws = torch.empty(lib.cn_colsum_workspace_bytes(M, K) // 4 + 1, device=X.device, dtype=torch.float32)
    _lib.call("cn_colsum", M, K, _ptr(w), _ptr(X), _ld(X), wdiv, _ptr(out), 1 if accumulate else 0, _ptr(ws),
              ws.numel() * 4, _stream())
    return out


def sdf_embed(x, multires, scale, U0, U4e=None, u4div=1.0):
    """U0 = the encoding of x; U4e = its first columns / u4div; each fp32 or a bfloat16 operand image."""
    _need(x, "x")
    _need(U0, "U0")
    _need(U4e, "U4e")
    flags = int(U4e is not None and U4e.dtype == torch.bfloat16) | (2 if U0.dtype == torch.bfloat16 else 0)
    _lib.call("cn_sdf_embed", x.shape[0], _ptr(x), _ld(x), multires, scale, U0.shape[1], _ptr(U0), _ld(U0),
              _ptr(U4e), _ld(U4e), u4div, flags, _stream())
    return U0


def sdf_mlp(u0b, tail, Ws, biases, head_w, head_b, sdf, *, multires, skip_layer, skip_div, beta, threshold,
            idx=None, debug=None):
    """The sampler's SDF query in one launch (cn_sdf_mlp): sdf[idx[m] or m] from the embedding u0b [M, 64] and
    the skip tail [M, >= E] through lin0 .. lin7 and the head row -- bf16 mode: bf16 images of both and bf16 weight
    images [256][K]; bf16x6 mode (ABI v15, 3-D weight images [K/16, 256, 48]): fp32 inputs, bitwise the
    layer-by-layer bf16x6 query.  Raises if the library does not support the network's shape."""
    x6 = Ws[0].dim() == 3
    for t, n in ((u0b, "u0b"), (tail, "tail")):
        _need(t, n)
        if t.dtype != (torch.float32 if x6 else torch.bfloat16):
            raise RuntimeError(f"sdf_mlp: {n} must be {'fp32' if x6 else 'a bfloat16 image'} in this mode")
    if len(Ws) != 8 or len(biases) != 8:
        raise RuntimeError("sdf_mlp: 8 hidden layers")
    d = _lib.SdfMlpDesc()
    d.u0, d.tail, d.ld_u0, d.ld_t = _ptr(u0b), _ptr(tail), _ld(u0b), _ld(tail)
    d.M, d.n_layers = u0b.shape[0], 8
    d.hidden, d.kpad0 = (Ws[1].shape[1], 16 * Ws[0].shape[0]) if x6 else (Ws[1].shape[0], Ws[0].shape[1])
    d.multires, d.skip_layer = multires, skip_layer
    d.format = FORMATS["bf16x6"] if x6 else 0
    for i, (W, b) in enumerate(zip(Ws, biases)):
        _need(W, f"W{i}", ndim=3 if x6 else 2)
        rows = W.shape[1] if x6 else W.shape[0]
        if W.dtype != torch.bfloat16 or rows != 256 or not b.is_contiguous() or b.dtype != torch.float32 or \
                (x6 and (W.dim() != 3 or W.shape[2] != 48 or not W.is_contiguous())):
            raise RuntimeError(f"sdf_mlp: layer {i} needs a bf16 [256][K] weight image (bf16x6: a [K/16, 256, 48] "
                               f"term image) and an fp32 bias")
        d.W[i], d.ldw[i], d.bias[i] = W.data_ptr(), (256 if x6 else W.stride(0)), b.data_ptr()
    if not (head_w.is_contiguous() and head_w.numel() >= 256 and head_b.numel() >= 1):
        raise RuntimeError("sdf_mlp: head_w [256], head_b [1]")
    if not sdf.is_contiguous() or (idx is None and sdf.numel() < u0b.shape[0]):
        raise RuntimeError("sdf_mlp: sdf must be contiguous with M entries (or idx)")
    if idx is not None and (idx.dtype != torch.int32 or idx.numel() < u0b.shape[0]):
        raise RuntimeError("sdf_mlp: idx must be int32 with M entries")
    d.head_w, d.head_b, d.sdf, d.idx = head_w.data_ptr(), head_b.data_ptr(), sdf.data_ptr(), _ptr(idx)
    d.skip_div, d.beta, d.threshold = skip_div, beta, threshold
    d.debug = _ptr(debug)  # tests: [8][M][256] (bf16; fp32 in the bf16x6 mode), every layer's input
    if _timer is not None:
        e0 = _timer.start()
        _lib.check(_lib.load().cn_sdf_mlp(d, _stream()), "cn_sdf_mlp")
        M = u0b.shape[0]
        ka = [16 * W.shape[0] if x6 else W.shape[1] for W in Ws]
        fl = sum(2.0 * M * 256 * k for k in ka)
        key = ("sdf_mlp",) + (("x6",) if x6 else ())
        _timer.symbols[key] = ("void cn::sdf_mlp_x6_kernel<false>(cn::SdfMlpX6Args)" if x6 else
                               "cn::sdf_mlp_kernel(cn::SdfMlpArgs)")
        _timer.stop(key, e0, fl, u0b.element_size() * M * (64 + tail.shape[1]) + 4.0 * M)
    else:
        _lib.check(_lib.load().cn_sdf_mlp(d, _stream()), "cn_sdf_mlp")
    return sdf


def sdf_net(lay, pk, layered=False):
    """cn_sdf_net of a packed SDF network (fields.SDFLayout + fields.pack_sdf's images), and the tensors
    it points into (hold them while the descriptor is used).  layered: never the fused cn_sdf_mlp query."""
    if lay.n_lin > _lib.SDF_MAX_LIN:
        raise RuntimeError(f"sdf_net: {lay.n_lin} Linear layers (at most {_lib.SDF_MAX_LIN})")
    n, keep = _lib.SdfNet(), []
    n.n_lin, n.skip, n.multires = lay.n_lin, lay.skip, lay.multires
    n.scale, n.beta, n.threshold = lay.scale, lay.beta, lay.threshold
    for l in range(lay.n_lin):
        n.in_dim[l], n.out_dim[l] = lay.in_dim[l], lay.out_dim[l]
    B0 = pk.Bf[0]
    x6 = B0.dim() == 3
    n.mfma_dtype = 2 if x6 else (1 if B0.dtype == torch.bfloat16 else 0)
    n.flags = 1 if layered else 0

    def aligned(t):
        t = t.contiguous()
        if t.data_ptr() % 16:
            t = t.clone()
        keep.append(t)
        return t.data_ptr()

    for l in range(lay.n_lin - 1):
        B = pk.Bf[l]
        if not B.is_contiguous():
            raise RuntimeError(f"sdf_net: layer {l} image must be contiguous")
        keep.append(B)
        n.W[l] = B.data_ptr()
        n.w_rows[l], n.w_cols[l] = (B.shape[1], 16 * B.shape[0]) if x6 else (B.shape[0], B.shape[1])
        n.bias[l] = aligned(pk.b[l])
    n.head_w = aligned(pk.w80.reshape(-1))
    n.head_b = aligned(pk.b80.reshape(-1))
    for l in range(lay.n_lin - 1):  # the transposed images (cn_render_fwd's ∇ pass)
        B = pk.Bt[l]
        if not B.is_contiguous():
            raise RuntimeError(f"sdf_net: layer {l} transposed image must be contiguous")
        keep.append(B)
        n.Wt[l] = B.data_ptr()
        n.wt_rows[l], n.wt_cols[l] = (B.shape[1], 16 * B.shape[0]) if x6 else (B.shape[0], B.shape[1])
    n.head_wp = aligned(pk.w80p)
    return n, keep


def color_net(lay, pk):
    """cn_color_net of a packed RenderingNetwork (fields.ColorLayout + fields.pack_color's images, lin0 folded
    or not), and the tensors it points into."""
    n, keep = _lib.ColorNet(), []
    n.n_lin, n.d_feature, n.multires_view = lay.n_lin, lay.F, lay.multires_view
    for l in range(lay.n_lin):
        n.in_dim[l], n.out_dim[l] = lay.in_dim[l], lay.out_dim[l]
    B0 = pk.Bf[0]
    x6 = B0.dim() == 3
    n.mfma_dtype = 2 if x6 else (1 if B0.dtype == torch.bfloat16 else 0)

    def aligned(t):
        t = t.contiguous()
        if t.data_ptr() % 16:
            t = t.clone()
        keep.append(t)
        return t.data_ptr()

    for l in range(lay.n_lin - 1):
        B = pk.Bf[l]
        keep.append(B)
        n.W[l] = B.data_ptr()
        n.w_rows[l], n.w_cols[l] = (B.shape[1], 16 * B.shape[0]) if x6 else (B.shape[0], B.shape[1])
        n.bias[l] = aligned(pk.b[l])
    n.head_w = aligned(pk.W3)
    n.head_b = aligned(pk.b3)

    def image(B):  # (pointer, rows, columns) of a GEMM image as cn_linear reads it
        keep.append(B)
        return (B.data_ptr(),) + ((B.shape[1], 16 * B.shape[0]) if x6 else (B.shape[0], B.shape[1]))

    for l in range(1, lay.n_lin - 1):  # the backward's transposed images (cn_render_bwd)
        n.Wt[l], n.wt_rows[l], n.wt_cols[l] = image(pk.Bt[l])
    n.Wtf, n.wtf_rows, n.wtf_cols = image(pk.Btf)
    n.Wxt, n.wxt_rows, n.wxt_cols = image(pk.Bxt)
    n.Wg = aligned(pk.Wg)
    n.wg_ld = pk.Wg.stride(0)
    return n, keep


_SIZES = {}


def _sized(fn, desc, *extra):
    """lib.<fn>(desc, *extra) memoised on the descriptor's shape key (_lib.shape_key): the composed entry
    points' planners run once per shape, not once more per call (the entry point itself re-plans into the
    caller's buffer and refuses a plan larger than it, so a stale size fails loudly, never silently)."""
    key = (fn, _lib.shape_key(desc), extra)
    n = _SIZES.get(key)
    if n is None:
        if len(_SIZES) > 4096:
            _SIZES.clear()
        n = _SIZES[key] = int(getattr(_lib.load(), fn)(ctypes.byref(desc), *extra))
    return n


def _check_render_inputs(fn, R, rays_o, rays_d, near, far, time_step, inv_s, car, t_rand=None, n_samples=None,
                         z=None):
    """The shapes and types the C side assumes (it takes R from rays_o and S from z): anything else would be
    read out of bounds on the device, so it is refused here with a RuntimeError, as ops.sample does."""
    for t, nm in ((rays_o, "rays_o"), (rays_d, "rays_d"), (near, "near"), (far, "far"), (time_step, "time_step"),
                  (inv_s, "inv_s"), (car, "cos_anneal_ratio"), (t_rand, "t_rand"), (z, "z")):
        if t is not None and (t.dtype != torch.float32 or not t.is_contiguous() or not t.is_cuda):
            raise RuntimeError(f"{fn}: {nm} must be a contiguous fp32 device tensor")
    if rays_o.shape != (R, 3) or rays_d.shape != (R, 3):
        raise RuntimeError(f"{fn}: rays_o and rays_d must be [R, 3] (got {tuple(rays_o.shape)}, {tuple(rays_d.shape)})")
    if near.numel() != R or far.numel() != R:
        raise RuntimeError(f"{fn}: near and far must hold R = {R} entries (got {near.numel()}, {far.numel()})")
    if time_step.numel() < 1 or inv_s.numel() < 1 or car.numel() < 1:
        raise RuntimeError(f"{fn}: time_step, inv_s and cos_anneal_ratio need one element each")
    if t_rand is not None and t_rand.shape != (R, n_samples):
        raise RuntimeError(f"{fn}: t_rand must be [R, n_samples] = [{R}, {n_samples}] (got {tuple(t_rand.shape)})")
    if z is not None and (z.dim() != 2 or z.shape[0] != R):
        raise RuntimeError(f"{fn}: z must be [R, S] with R = {R} rows (got {tuple(z.shape)})")


def render_fwd(sdf_net_, color_net_, rays_o, rays_d, near, far, time_step, inv_s, car, n_samples, n_importance,
               up_sample_steps, t_rand=None, z_in=None, philox=None):
    """NeuSRenderer.forward without gradient in one call (cn_render_fwd): returns z, pts, sdf, grad, rgb, color,
    depth, weights, cdf."""
    R, dev = rays_o.shape[0], rays_o.device
    _check_render_inputs("render_fwd", R, rays_o, rays_d, near, far, time_step, inv_s, car, t_rand=t_rand,
                         n_samples=n_samples, z=z_in)
    if z_in is not None:
        S = z_in.shape[1]
    else:
        k = n_importance // up_sample_steps if n_importance > 0 else 0
        S = n_samples + up_sample_steps * k
    f = lambda *s: torch.empty(*s, device=dev)  # noqa: E731
    out = dict(z=f(R, S), pts=f(R * S, 4), sdf=f(R * S), grad=f(R * S, 4), rgb=f(R * S, 3), color=f(R, 3),
               depth=f(R), weights=f(R, S), cdf=f(R, S))
    d = _lib.RenderDesc()
    d.R, d.n_samples, d.n_importance, d.up_sample_steps = R, n_samples, n_importance, up_sample_steps
    d.S_in = S if z_in is not None else 0
    d.rays_o, d.rays_d, d.near, d.far = _ptr(rays_o), _ptr(rays_d), _ptr(near), _ptr(far)
    d.t_rand, d.time_step, d.z_in = _ptr(t_rand), _ptr(time_step), _ptr(z_in)
    d.inv_s, d.cos_anneal_ratio = _ptr(inv_s), _ptr(car)
    d.sdf_net, d.color_net = ctypes.pointer(sdf_net_), ctypes.pointer(color_net_)
    _check_philox(philox)
    d.philox = _ptr(philox)
    for k, v in out.items():
        setattr(d, k, v.data_ptr())
    lib = _lib.load()
    ws = torch.empty(max(_sized("cn_render_fwd_workspace_bytes", d), 1), dtype=torch.uint8, device=dev)
    _lib.check(lib.cn_render_fwd(ctypes.byref(d), _ptr(ws), ws.numel(), _stream()), "cn_render_fwd")
    return out


def render_train_fwd(sdf_net_, color_net_, rays_o, rays_d, near, far, time_step, inv_s, car, n_coarse, z):
    """render_core at the samples z [R, S] keeping its backward's state -- cn_render_train_fwd: returns the outputs
    (pts [M, 4], sdf [M, 1], grad [M, 4], color [R, 3], depth [R, 1], weights, cdf [R, S]), the state buffer and the
    descriptor render_bwd takes (the inputs must stay alive and unchanged until then)."""
    R, S = z.shape
    M, dev = R * S, z.device
    _check_render_inputs("render_train_fwd", rays_o.shape[0], rays_o, rays_d, near, far, time_step, inv_s, car, z=z)
    f = lambda *s: torch.empty(*s, device=dev)  # noqa: E731
    out = dict(pts=f(M, 4), sdf=f(M, 1), grad=f(M, 4), color=f(R, 3), depth=f(R, 1), weights=f(R, S), cdf=f(R, S))
    d = _lib.RenderDesc()
    d.R, d.n_samples, d.S_in = R, n_coarse, S
    d.rays_o, d.rays_d, d.near, d.far = _ptr(rays_o), _ptr(rays_d), _ptr(near), _ptr(far)
    d.time_step, d.z_in, d.inv_s, d.cos_anneal_ratio = _ptr(time_step), _ptr(z), _ptr(inv_s), _ptr(car)
    d.sdf_net, d.color_net = ctypes.pointer(sdf_net_), ctypes.pointer(color_net_)
    for k, v in out.items():
        setattr(d, k, v.data_ptr())
    lib = _lib.load()
    state = torch.empty(max(_sized("cn_render_state_bytes", d), 1), dtype=torch.uint8, device=dev)
    _lib.check(lib.cn_render_train_fwd(ctypes.byref(d), _ptr(state), state.numel(), _stream()), "cn_render_train_fwd")
    return out, state, d


def render_bwd(d, state, *, dcolor=None, ddepth=None, dweights=None, dcdf=None, dsdf=None, dgrad=None, dpts=None,
               sdf_dWs, sdf_dbs, col_dWs, col_dbs, dinv_s, drays_o=None, drays_d=None):
    """The backward of render_train_fwd -- cn_render_bwd (upstream gradients contiguous float32 or None)."""
    for t in (dcolor, ddepth, dweights, dcdf, dsdf, dgrad, dpts):
        if t is not None and (not t.is_contiguous() or t.dtype != torch.float32):
            raise RuntimeError("render_bwd: upstream gradients must be contiguous float32")
    g = _lib.RenderGrads()
    g.dcolor, g.ddepth, g.dweights, g.dcdf = _ptr(dcolor), _ptr(ddepth), _ptr(dweights), _ptr(dcdf)
    g.dsdf, g.dgrad, g.dpts = _ptr(dsdf), _ptr(dgrad), _ptr(dpts)
    for l, (w, b) in enumerate(zip(sdf_dWs, sdf_dbs)):
        g.sdf_dW[l], g.sdf_db[l] = _ptr(w), _ptr(b)
    for l, (w, b) in enumerate(zip(col_dWs, col_dbs)):
        g.col_dW[l], g.col_db[l] = _ptr(w), _ptr(b)
    g.dinv_s, g.drays_o, g.drays_d = _ptr(dinv_s), _ptr(drays_o), _ptr(drays_d)
    lib = _lib.load()
    nb = _sized("cn_render_bwd_workspace_bytes", d, 1 if drays_o is not None else 0)
    ws = torch.empty(max(nb, 1), dtype=torch.uint8, device=state.device)
    _lib.check(lib.cn_render_bwd(ctypes.byref(d), ctypes.byref(g), _ptr(state), state.numel(), _ptr(ws), ws.numel(),
                                 _stream()), "cn_render_bwd")


def sdf_query(net, x, sdf, idx=None):
    """sdf[idx[m] or m] = SDFNetwork.sdf(x[m]) -- cn_sdf_query (net: sdf_net's descriptor)."""
    _need(x, "x")
    M = x.shape[0]
    if idx is not None and (idx.dtype != torch.int32 or idx.numel() < M or not idx.is_contiguous()):
        raise RuntimeError("sdf_query: idx must be contiguous int32 with M entries")
    if not sdf.is_contiguous() or (idx is None and sdf.numel() < M):
        raise RuntimeError("sdf_query: sdf must be contiguous with M entries (or idx)")
    lib = _lib.load()
    ws = torch.empty(max(int(lib.cn_sdf_query_workspace_bytes(ctypes.byref(net), M)), 1), dtype=torch.uint8,
                     device=x.device)
    _lib.check(lib.cn_sdf_query(ctypes.byref(net), M, _ptr(x), _ld(x), _ptr(sdf), _ptr(idx), _ptr(ws), ws.numel(),
                                _stream()), "cn_sdf_query")
    return sdf


def _mlp_desc(net, M, x=None, sdf=None, dsdf=None, dWs=None, dbs=None, dx=None):
    d = _lib.MlpDesc()
    d.M, d.x, d.net, d.sdf, d.dsdf, d.dx = M, _ptr(x), ctypes.pointer(net), _ptr(sdf), _ptr(dsdf), _ptr(dx)
    for l, (w, b) in enumerate(zip(dWs or [], dbs or [])):
        d.dW[l], d.db[l] = _ptr(w), _ptr(b)
    return d


def mlp_fwd(net, x, sdf):
    """sdf[m] = SDFNetwork.sdf(x[m]) keeping the activations the backward reads -- cn_mlp_fwd; returns the
    state buffer mlp_bwd takes (net: sdf_net's descriptor, with its transposed images)."""
    _need(x, "x")
    M = x.shape[0]
    if x.dim() != 2 or x.shape[1] != 4 or x.stride(0) != 4 or x.dtype != torch.float32:
        raise RuntimeError("mlp_fwd: x must be a contiguous float32 [M, 4]")
    if not sdf.is_contiguous() or sdf.numel() < M:
        raise RuntimeError("mlp_fwd: sdf must be contiguous with M entries")
    lib = _lib.load()
    d = _mlp_desc(net, M, x=x, sdf=sdf)
    state = torch.empty(max(_sized("cn_mlp_state_bytes", d), 1), dtype=torch.uint8, device=x.device)
    _lib.check(lib.cn_mlp_fwd(ctypes.byref(d), _ptr(state), state.numel(), _stream()), "cn_mlp_fwd")
    return state


def mlp_bwd(net, M, state, dsdf, dWs=None, dbs=None, dx=None):
    """The gradients of SDFNetwork.sdf from dsdf [M] -- cn_mlp_bwd: dWs[l] [out_dim, in_dim] / dbs[l]
    (every Linear, or None: dx only) and dx [M, 4] (or None)."""
    _need(dsdf, "dsdf", ndim=1)
    if not dsdf.is_contiguous() or dsdf.numel() < M:
        raise RuntimeError("mlp_bwd: dsdf must be contiguous with M entries")
    for t in list(dWs or []) + list(dbs or []) + [dx]:
        if t is not None and (not t.is_contiguous() or t.dtype != torch.float32):
            raise RuntimeError("mlp_bwd: gradients must be contiguous float32")
    lib = _lib.load()
    d = _mlp_desc(net, M, dsdf=dsdf, dWs=dWs, dbs=dbs, dx=dx)
    ws = torch.empty(max(_sized("cn_mlp_bwd_workspace_bytes", d), 1), dtype=torch.uint8,
                     device=dsdf.device)
    _lib.check(lib.cn_mlp_bwd(ctypes.byref(d), _ptr(state), state.numel(), _ptr(ws), ws.numel(), _stream()),
               "cn_mlp_bwd")


def sample(net, rays_o, rays_d, near, far, t_rand, time_step, n_samples, n_importance, up_sample_steps, z,
           philox=None):
    """z [R, n_samples + up_sample_steps * (n_importance // up_sample_steps)] -- cn_sample: coarse z and the
    up-sampling rounds with their SDF queries in one call (net: sdf_net's descriptor).  philox (with t_rand
    None): a device uint64 [2] (seed, offset) -- the jitter drawn on the device (cn_uniform_philox)."""
    _check_philox(philox)
    for t, nm in ((rays_o, "rays_o"), (rays_d, "rays_d"), (near, "near"), (far, "far"), (t_rand, "t_rand"),
                  (time_step, "time_step"), (z, "z")):
        if t is not None and (t.dtype != torch.float32 or not t.is_contiguous()):
            raise RuntimeError(f"sample: {nm} must be a contiguous fp32 tensor")
    R = z.shape[0]
    k = n_importance // up_sample_steps if n_importance > 0 else 0
    if z.shape[1] != n_samples + up_sample_steps * k or (t_rand is not None and t_rand.shape != (R, n_samples)):
        raise RuntimeError("sample: z [R, n_samples + up_sample_steps * k] and t_rand [R, n_samples]")
    d = _lib.SampleDesc()
    d.R, d.n_samples, d.n_importance, d.up_sample_steps = R, n_samples, n_importance, up_sample_steps
    d.rays_o, d.rays_d, d.near, d.far = _ptr(rays_o), _ptr(rays_d), _ptr(near), _ptr(far)
    d.t_rand, d.time_step, d.z = _ptr(t_rand), _ptr(time_step), _ptr(z)
    d.net, d.philox = ctypes.pointer(net), _ptr(philox)
    lib = _lib.load()
    ws = torch.empty(max(_sized("cn_sample_workspace_bytes", d), 1), dtype=torch.uint8, device=z.device)
    _lib.check(lib.cn_sample(ctypes.byref(d), _ptr(ws), ws.numel(), _stream()), "cn_sample")
    return z


def sdf_grad_assemble(multires, scale, U0, Q0, QE, G):
    _lib.call("cn_sdf_grad_assemble", U0.shape[0], multires, scale, _ptr(U0), _ld(U0), _ptr(Q0), _ld(Q0),
              _ptr(QE), _ld(QE), _ptr(G), _ld(G), _stream())
    return G


def sdf_tangent_prep(multires, scale, U0, v, T0, T4e=None, t4div=1.0):
    """T0 = the tangent of the encoding along v; T4e (fp32, or a bfloat16 image) = its first columns / t4div."""
    _need(v, "v")
    _need(T4e, "T4e")
    _lib.call("cn_sdf_tangent_prep", U0.shape[0], multires, scale, T0.shape[1], _ptr(U0), _ld(U0), _ptr(v),
              _ld(v), _ptr(T0), _ld(T0), _ptr(T4e), _ld(T4e), t4div, int(T4e is not None and T4e.dtype == torch.bfloat16),
              _stream())
    return T0


def color_extras(G, pts, dirs, dir_div, multires_view, ext):
    for t, n in ((G, "G"), (pts, "pts"), (dirs, "dirs"), (ext, "ext")):
        _need(t, n)
    _lib.call("cn_color_extras", G.shape[0], _ptr(G), _ld(G), _ptr(pts), _ld(pts), _ptr(dirs), _ld(dirs),
              dir_div, multires_view, ext.shape[1], _ptr(ext), _ld(ext), _stream())
    return ext


def rgb_head_bwd(drgb, rgb, H3, K, W3, dZ2, dW3, db3):
    M = rgb.shape[0]
    lib = _lib.load()
    ws = torch.empty(lib.cn_rgb_head_bwd_workspace_bytes(M, K) // 4 + 1, device=rgb.device, dtype=torch.float32)
    _lib.call("cn_rgb_head_bwd", M, K, _ptr(drgb), _ptr(rgb), _ptr(H3), _ld(H3), _ptr(W3), _ptr(dZ2), _ld(dZ2),
              1 if dZ2.dtype == torch.bfloat16 else 0, _ptr(dW3), _ptr(db3), _ptr(ws), ws.numel() * 4, _stream())


def patch_indices(h, w, ps, n_patches, key, out=None):
    """Flat pixel ids [n_patches * ps * ps] (int64) of distinct random patches -- cn_patch_indices;
    key: int32 [4] device tensor."""
    _need(key, "key", ndim=1)
    if key.dtype != torch.int32 or key.numel() < 4:
        raise RuntimeError("patch_indices: key must be an int32 tensor of 4 values")
    if out is None:
        out = torch.empty(n_patches * ps * ps, dtype=torch.int64, device=key.device)
    _lib.call("cn_patch_indices", h, w, ps, n_patches, _ptr(key), _ptr(out), _stream())
    return out


def _check_philox(so):
    if so is not None and (so.dtype != torch.uint64 or so.numel() < 2 or not so.is_contiguous() or not so.is_cuda):
        raise RuntimeError("philox: a contiguous device uint64 tensor [2] = (seed, offset)")


def uniform_philox(n, seed_offset, out=None):
    """out[i] in [0, 1) from Philox4x32-10 (counter (i // 4, offset), key seed) -- cn_uniform_philox; seed_offset
    is a device uint64 [2] read by the kernel (a replayed graph draws with its current value)."""
    _check_philox(seed_offset)
    out = torch.empty(n, device=seed_offset.device) if out is None else out
    _lib.call("cn_uniform_philox", n, _ptr(seed_offset), _ptr(out), _stream())
    return out


def coarse_z(near, far, n, t_rand, z):
    _lib.call("cn_coarse_z", z.shape[0], n, _ptr(near), _ptr(far), _ptr(t_rand), _ptr(z), _stream())
    return z


def points(rays_o, rays_d, z, t, pts, *, mid=False, near=None, far=None, n_coarse=0):
    R, n = z.shape
    _lib.call("cn_points", R, n, _ptr(rays_o), _ptr(rays_d), _ptr(z), _ptr(t), 1 if mid else 0, _ptr(near),
              _ptr(far), n_coarse, _ptr(pts), _stream())
    return pts


def up_sample_merge(z, sdf, n_imp, inv_s, z_out, z_new, sdf_out=None, new_dst=None):
    R, n = z.shape
    _lib.call("cn_up_sample_merge", R, n, n_imp, float(inv_s), _ptr(z), _ptr(sdf), _ptr(z_out), _ptr(z_new),
              _ptr(sdf_out), _ptr(new_dst), _stream())


def device_scalar(x, device) -> torch.Tensor:
    """A float / 0-d tensor as a 1-element fp32 device tensor (the kernels read schedule
    values such as cos_anneal_ratio from device memory, so a replayed graph sees updates)."""
    if isinstance(x, torch.Tensor):
        t = x.reshape(-1)[:1]
        if t.device != device or t.dtype != torch.float32:
            t = t.to(device=device, dtype=torch.float32)
        return t.contiguous()
    return torch.full((1,), float(x), device=device, dtype=torch.float32)


def composite_fwd(z, sdf, G, rgb, rays_d, inv_s, near, far, n_coarse, car, color, depth, weights, cdf):
    """car: cos_anneal_ratio as a 1-element device tensor (device_scalar)."""
    R, S = z.shape
    _lib.call("cn_composite_fwd", R, S, _ptr(z), _ptr(sdf), _ptr(G), G.stride(0), _ptr(rgb), _ptr(rays_d),
              _ptr(inv_s), _ptr(near), _ptr(far), n_coarse, _ptr(car), _ptr(color), _ptr(depth), _ptr(weights),
              _ptr(cdf), _stream())


def composite_bwd(z, sdf, G, rgb, rays_d, inv_s, near, far, n_coarse, car, dcolor, ddepth, dweights, dcdf,
                  dsdf, dG, drgb, dinv_part, drays_d=None):
    R, S = z.shape
    _lib.call("cn_composite_bwd", R, S, _ptr(z), _ptr(sdf), _ptr(G), G.stride(0), _ptr(rgb), _ptr(rays_d),
              _ptr(inv_s), _ptr(near), _ptr(far), n_coarse, _ptr(car), _ptr(dcolor), _ptr(ddepth),
              _ptr(dweights), _ptr(dcdf), _ptr(dsdf), _ptr(dG), _ptr(drgb), _ptr(dinv_part), _ptr(drays_d),
              _stream())


def points_bwd(z, dP, drays_o, drays_d, *, mid=False, near=None, far=None, n_coarse=0):
    """drays_o = sum_i dP_i, drays_d = sum_i dP_i * zz_i per ray -- cn_points_bwd."""
    _need(dP, "dP")
    R, n = z.shape
    _lib.call("cn_points_bwd", R, n, _ptr(z), 1 if mid else 0, _ptr(near), _ptr(far), n_coarse, _ptr(dP), _ld(dP),
              _ptr(drays_o), _ptr(drays_d), _stream())


def color_extras_bwd(d_ext, dirs, dir_div, multires_view, ddirs, accumulate=False):
    """ddirs [R,3] (+)= view-encoding gradient of d_ext -- cn_color_extras_bwd."""
    _need(d_ext, "d_ext")
    _need(dirs, "dirs")
    _lib.call("cn_color_extras_bwd", dirs.shape[0], dir_div, _ptr(d_ext), _ld(d_ext), _ptr(dirs), _ld(dirs),
              multires_view, _ptr(ddirs), 1 if accumulate else 0, _stream())
    return ddirs


def train_loss(color, gt, depth, normals, *, w_rgb=1.0, w_eik=0.1, w_edge=1.0, w_smooth=1e-4, patch=4, gamma=0.1,
               weights=None, nonfinite=None):
    """(loss [], dcolor [R,3], ddepth [R,1], dnormals [M,3]) -- cn_train_loss: the colour
    L1, eikonal, edge-aware and plain smoothness terms and their input gradients.
    normals may be any [M,3] row view (e.g. the first three columns of ∇ₓSDF).
    weights: optional device tensor [4] (w_rgb, w_eik, w_edge, w_smooth) read by the
    kernels (overrides the floats); nonfinite: optional device int32 [1] flag set when
    the loss is not finite."""
    for t, n in ((color, "color"), (gt, "gt"), (normals, "normals")):
        _need(t, n)
    _need(depth.reshape(-1, 1), "depth")
    R, M, dev = color.shape[0], normals.shape[0], color.device
    if not (color.is_contiguous() and gt.is_contiguous() and depth.is_contiguous()):
        raise RuntimeError("train_loss: color, gt and depth must be contiguous")
    lib = _lib.load()
    if weights is None:
        weights = torch.tensor([w_rgb, w_eik, w_edge, w_smooth], dtype=torch.float32).to(dev, non_blocking=True)
    elif weights.dtype != torch.float32 or weights.numel() != 4 or not weights.is_contiguous() or weights.device != dev:
        raise RuntimeError("train_loss: weights must be a contiguous fp32 [4] tensor on the loss device")
    if nonfinite is not None and (nonfinite.dtype != torch.int32 or nonfinite.device != dev):
        raise RuntimeError("train_loss: nonfinite must be an int32 tensor on the loss device")
    ws = torch.empty(lib.cn_train_loss_workspace_bytes(R, patch) // 8 + 1, device=dev, dtype=torch.float64)
    loss = torch.empty((), device=dev)
    dcolor = torch.empty_like(color)
    ddepth = torch.empty(R, 1, device=dev)
    dn = torch.empty(M, 3, device=dev)
    _lib.call("cn_train_loss", R, patch, M, _ptr(color), _ptr(gt), _ptr(depth), _ptr(normals), _ld(normals),
              _ptr(weights), float(gamma), _ptr(loss), _ptr(dcolor), _ptr(ddepth), _ptr(dn), 3, _ptr(nonfinite),
              _ptr(ws), ws.numel() * 8, _stream())
    return loss, dcolor, ddepth, dn
