"""SDF / colour / variance fields backed by the HIP kernels.

API mirror of the reference modules (same constructor arguments, attribute
names, parameter initialisation order and state-dict keys, so reference
checkpoints and `pretrained_sdf/model.pt` load unchanged):

  SDFNetwork            model/neus_fields.py:205-303
  RenderingNetwork      model/neus_fields.py:307-374
  SingleVarianceNetwork model/neus_fields.py:459-465
  NeRF                  model/neus_fields.py:378-456  (constructed by train.py:39;
                        the n_outside > 0 branch that calls it is out of scope)

The forward passes do not run the torch layers: the effective (weight-normed)
weights are packed once per call and the whole MLP -- encoding, 9 Linear +
Softplus layers, the sdf head, the ∇ₓSDF pass and its create_graph double
backward -- runs in cn_linear / cn_wgrad launches (see sdf_forward /
sdf_backward below and DESIGN.md §3).
"""
from __future__ import annotations

import dataclasses
import math
from typing import List, Optional

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

from . import ops
from .embedder import embed_dim
from .ops import (EPI_BWD_RELU, EPI_BWD_SOFTPLUS, EPI_MUL, EPI_RELU, EPI_SOFTPLUS, EPI_SOFTPLUS_HEAD, EPI_STORE,
                  EPI_TANGENT, SQRT2, rup)


def effective_weight(lin: nn.Linear) -> torch.Tensor:
    """W = g * v / ||v|| (torch.nn.utils.weight_norm, dim 0), or the plain weight."""
    if hasattr(lin, "weight_v"):
        return torch._weight_norm(lin.weight_v, lin.weight_g, 0)
    return lin.weight


def release_weight_norm_graphs(module: nn.Module) -> nn.Module:
    """nn.utils.weight_norm keeps the last weight it computed (g v / |v|, at construction and in
    every forward pre-hook) as a plain attribute that carries its autograd graph, i.e. the
    AccumulateGrad nodes of weight_g / weight_v, alive for the module's lifetime.  Autograd
    then reuses those nodes in every later step, bound to the stream of construction, which
    a HIP-graph capture on another stream reports as a stream mismatch (and may synchronise
    on).  This build computes the effective weights itself (effective_weight(s)), so the
    attribute is replaced by a detached copy: same values, no graph.  Not part of the state
    dict either way."""
    for m in module.modules():
        w = m.__dict__.get("weight")
        if hasattr(m, "weight_v") and torch.is_tensor(w) and w.grad_fn is not None:
            m.weight = w.detach()
    return module


class _WeightNormFn(torch.autograd.Function):
    """W_l = g_l v_l / |v_l| for every weight-normed Linear of a network in one launch
    forward and one backward (cn_weight_norm) instead of one torch launch per layer each way."""

    @staticmethod
    def forward(ctx, n, *vg):
        vs, gs = vg[:n], vg[n:]
        ctx.save_for_backward(*vs, *gs)
        ctx.n = n
        return tuple(ops.weight_norm_batch(list(vs), list(gs)))

    @staticmethod
    def backward(ctx, *dWs):
        n = ctx.n
        saved = ctx.saved_tensors
        vs, gs = list(saved[:n]), list(saved[n:])
        dws = [d if d is not None else torch.zeros_like(v) for d, v in zip(dWs, vs)]
        dvs, dgs = ops.weight_norm_batch(vs, gs, dws=dws)
        return (None,) + tuple(dvs) + tuple(dg.view_as(g) for dg, g in zip(dgs, gs))


def effective_weights(lins) -> List[torch.Tensor]:
    """effective_weight of every layer; the weight-normed ones on a HIP device in one batched launch."""
    wn = [i for i, lin in enumerate(lins) if hasattr(lin, "weight_v") and lin.weight_v.is_cuda]
    out = [None] * len(lins)
    if wn:
        vs = [lins[i].weight_v for i in wn]
        gs = [lins[i].weight_g for i in wn]
        for i, w in zip(wn, _WeightNormFn.apply(len(wn), *vs, *gs)):
            out[i] = w
    return [w if w is not None else effective_weight(lin) for w, lin in zip(out, lins)]


def _empty(M, n, dev):
    return torch.empty(M, n, device=dev, dtype=torch.float32)


# ---------------------------------------------------------------------------
# SDF network
@dataclasses.dataclass
class SDFLayout:
    n_lin: int               # number of Linear layers (9)
    in_dim: List[int]
    out_dim: List[int]
    E: int                   # encoding width (52)
    KE: int                  # padded encoding width (64)
    HL: int                  # leading dimension of hidden buffers (>= widths, multiple of 128)
    skip: int                # index of the layer whose input is cat([x, emb]) / sqrt(2), or -1
    multires: int
    scale: float
    beta: float = 100.0
    threshold: float = 20.0

    @property
    def H_feat(self):
        return self.out_dim[-1] - 1


@dataclasses.dataclass
class SDFPack:
    Bf: list      # forward weights [Npad][Kpad], hidden layers
    Bt: list      # transposed weights [in_pad][out_pad]
    b: list       # hidden biases
    w80: torch.Tensor   # [1, in8] sdf row / scale
    b80: torch.Tensor   # [1] sdf bias / scale
    w80p: torch.Tensor  # [HL] sdf row / scale, zero padded
    Bf8: torch.Tensor   # feature rows of the last layer
    Bt8: torch.Tensor
    bf8: torch.Tensor


MFMA_DTYPES = ("fp32", "bf16", "bf16x6")


def _kq(mfma_dtype: str) -> int:
    """K padding multiple of the B images for an MFMA mode (bf16 MFMA steps are 64 deep)."""
    if mfma_dtype not in MFMA_DTYPES:
        raise ValueError(f"mfma_dtype must be one of {MFMA_DTYPES} (got {mfma_dtype!r})")
    return 64 if mfma_dtype == "bf16" else 32


def _wgrad_mode(pk) -> str:
    """The weight gradients run in the pack's MFMA mode."""
    if pk.Bf[0].dtype != torch.bfloat16:
        return "fp32"
    return "bf16x6" if pk.Bf[0].dim() == 3 else "bf16"


def pack_sdf(lay: SDFLayout, Ws, bs, mfma_dtype: str = "fp32") -> SDFPack:
    """Zero-padded GEMM images of the effective weights, built in one
    cn_pack_weights launch.  mfma_dtype "bf16": bfloat16 images with K padded
    to 64 (cn_linear's bf16 MFMA path); "bf16x6": chunk-major bf16 term images [K/16, N, 48]
    (fp32 GEMMs on the bf16 MFMA)."""
    kq = _kq(mfma_dtype)
    pk = ops.ImagePacker(mfma_dtype)
    with torch.no_grad():
        dev = Ws[0].device
        Bf, Bt, b = [], [], []
        for l in range(lay.n_lin - 1):
            W = Ws[l].detach().contiguous()
            o, i = W.shape
            kp = lay.KE if l == 0 else rup(i, kq)
            Bf.append(pk.put(pk.image(rup(o, 128), kp, dev), W))
            Bt.append(pk.put(pk.image(rup(i, 128), rup(o, kq), dev), W, transpose=True))
            b.append(bs[l].detach().contiguous())
        W8, b8 = Ws[-1].detach().contiguous(), bs[-1].detach()
        s = float(lay.scale)
        w80 = (W8[0] / s) if s != 1.0 else W8[0]
        b80 = (b8[:1] / s) if s != 1.0 else b8[:1]
        w80p = F.pad(w80, (0, lay.HL - w80.shape[0])).contiguous()
        Wf = W8[1:]
        o, i = Wf.shape
        Bf8 = pk.put(pk.image(rup(o, 128), rup(i, kq), dev), Wf)
        Bt8 = pk.put(pk.image(rup(i, 128), rup(o, kq), dev), Wf, transpose=True)
        pk.run()
        return SDFPack(Bf, Bt, b, w80.contiguous()[None], b80.contiguous(), w80p, Bf8, Bt8, b8[1:].contiguous())


def _fuse_head(lay: SDFLayout, pk: SDFPack) -> bool:
    """The last hidden layer computes the sdf head in its epilogue (EPI_SOFTPLUS_HEAD)
    when one GEMM tile spans its whole output row: N <= 128 in every mode, N <= 256
    with the 256-wide bf16x6 and bf16 tiles."""
    L8 = lay.n_lin - 1
    N = lay.out_dim[L8 - 1]
    if lay.in_dim[L8] != N or N % 4 or L8 == lay.skip or L8 - 1 == 0:
        return False
    B = pk.Bf[L8 - 1]
    x6 = B.dim() == 3
    bf = B.dtype == torch.bfloat16 and not x6
    return N <= 128 or (x6 and N <= 256 and B.shape[1] >= 256 and rup(lay.in_dim[L8 - 1], 32) % 64 == 0) or \
        (bf and N <= 256 and B.shape[0] >= 256)


def sig_beta(lay: SDFLayout, l: int) -> float:
    """aux_beta of softplus' σ_l read from the stored activation U[l+1] = a_l / c
    (c = √2 for the layer feeding the skip concat, neus_fields.py:276-277):
    σ_l = 1 - exp(-β c U[l+1])."""
    return lay.beta * (SQRT2 if (l + 1) == lay.skip else 1.0)


# Attribution switches of the bf16 mode's quality study (tools/quality_sweep.py), honoured by
# the layer-by-layer composition only (renderer.RENDER_NATIVE / MLP_NATIVE off):
#   BF16_IMAGES = False  no operand images: the bf16 GEMMs round fp32 operands while staging (the same
#                        products), σ and the second-order term's s, u̇ from fp32 values;
#   SIGMA_FP32 = True    the images stay the GEMMs' operands, but MUL / TANGENT / BWD_SOFTPLUS recover σ from
#                        an fp32 copy of the activation (the second-order term's s, u̇ keep their image values).
BF16_IMAGES = True
SIGMA_FP32 = False


def _img_mode(pk, lay) -> bool:
    """bf16 MFMA mode (config C3): activations whose consumers are GEMM operands are stored as bf16
    operand images -- the bits the GEMM staging would round them to -- beside (or instead of) the fp32
    values the epilogues read.  Only with 256-padded hidden buffers: image operands of a
    weight gradient need the 256x256 stage ring (cn_wgrad's bf16 images); narrower networks keep fp32
    operands, rounded on load."""
    B = pk.Bf[0]
    return BF16_IMAGES and B.dtype == torch.bfloat16 and B.dim() == 2 and lay.HL % 256 == 0


def _empty_b(M, n, dev):
    return torch.empty(M, n, device=dev, dtype=torch.bfloat16)


def _act(U, Ub, l):
    """The stored activation U_l an epilogue recovers σ_{l-1} from: fp32, or (bf16 mode, hidden layers
    1..7) its bf16 image -- the only copy kept there."""
    return U[l] if U[l] is not None else Ub[l]


# The no-grad SDF query (the sampler's, neus_renderer.py:492-525) in one launch in the bf16 mode
# (cn_sdf_mlp: activations on chip, bitwise equal to the layer-by-layer path); False: layer by layer
FUSED_SDF_QUERY = True


def _x6_pack(pk) -> bool:
    """The pack holds bf16x6 term images (chunk-major [K/16, rows, 48])."""
    return pk.Bf[0].dim() == 3


def _fused_query_ok(lay: SDFLayout, pk: SDFPack) -> bool:
    """cn_sdf_mlp's shape: 8 hidden layers of 256 (the skip layer 256 - E), K0 = 64, bf16 images -- or, ABI v15,
    the bf16x6 mode's term images of 256 rows."""
    x6 = _x6_pack(pk)
    if not (FUSED_SDF_QUERY and (_img_mode(pk, lay) or x6) and lay.n_lin == 9 and lay.HL == 256 and lay.KE == 64):
        return False
    sk = lay.skip
    if not (2 <= sk <= 7 and lay.E + lay.out_dim[sk - 1] == 256):
        return False
    rows = (lambda B: B.shape[1]) if x6 else (lambda B: B.shape[0])
    return all(lay.out_dim[l] == 256 for l in range(8) if l != sk - 1) and lay.out_dim[8] >= 1 and \
        all(rows(pk.Bf[l]) == 256 for l in range(8)) and lay.in_dim[8] == 256


def sdf_query_fused(lay: SDFLayout, pk: SDFPack, x: torch.Tensor, sdf_out: Optional[torch.Tensor] = None,
                    dst: Optional[torch.Tensor] = None) -> torch.Tensor:
    """SDFNetwork.sdf(x) with no gradient (neus_fields.py:268-283) in two launches: cn_sdf_embed writes the
    embedding's bf16 images (lin0's input, the skip concat's tail / sqrt 2) -- fp32 rows in the bf16x6 mode --,
    cn_sdf_mlp runs lin0 .. lin7 and the sdf head with the activations on chip."""
    M, dev = x.shape[0], x.device
    mk = _empty if _x6_pack(pk) else _empty_b
    u0b = mk(M, lay.KE, dev)
    tail = mk(M, 64, dev)
    ops.sdf_embed(x, lay.multires, lay.scale, u0b, tail[:, :lay.E], SQRT2)
    sdf = sdf_out if sdf_out is not None else _empty(M, 1, dev)
    ops.sdf_mlp(u0b, tail[:, :lay.E], pk.Bf[:8], pk.b[:8], pk.w80[0], pk.b80, sdf, multires=lay.multires,
                skip_layer=lay.skip - 1, skip_div=SQRT2, beta=lay.beta, threshold=lay.threshold, idx=dst)
    return sdf


def sdf_forward(lay: SDFLayout, pk: SDFPack, x: torch.Tensor, *, want_feat: bool, want_grad: bool, keep: bool,
                sdf_out: Optional[torch.Tensor] = None, dst: Optional[torch.Tensor] = None):
    """Forward of SDFNetwork (neus_fields.py:268-283) and, with want_grad, the
    ∇ₓSDF pass of SDFNetwork.gradient (neus_fields.py:291-303).

    Returns a dict of device buffers; with keep=True everything the backward
    needs (layer inputs U_l and the ∇ pass adjoints S_l) is retained.  softplus'
    σ_l is never stored: its consumers recover it from U[l+1] (sig_beta).
    want_feat="hidden": no feature head -- the caller consumes the last hidden
    activation U[L8] directly (the renderer folds the feature head into the
    colour network's first layer, NeuSRenderer._folded_color_pack).
    bf16 mode (_img_mode): Ub / Sb hold the bf16 operand images of the hidden activations and ∇-pass
    adjoints, which the next GEMMs, the weight gradients and (s) the adjoint's second-order term read;
    fp32 is kept only where it is needed: the encoding U_0, the last hidden activation U_8 (the
    elementwise last adjoint, the colour network's fold), s_0 and s_7 for the fp32 first-layer weight
    gradient / the elementwise last adjoint.  The hidden activations U_1..U_7 are images only: the GEMMs
    read them as A, the weight gradients as X, and MUL / TANGENT / BWD_SOFTPLUS recover σ from them.
    """
    M, dev = x.shape[0], x.device
    if want_feat is False and not want_grad and not keep and _fused_query_ok(lay, pk):
        return {"U": None, "Ub": None, "S": None, "Sb": None, "sdf": sdf_query_fused(lay, pk, x, sdf_out, dst),
                "feat": None, "G": None}
    nl, sk, HL, KE = lay.n_lin, lay.skip, lay.HL, lay.KE
    keep_u = keep or want_grad
    img = _img_mode(pk, lay)
    L8 = nl - 1
    U, Ub = [None] * nl, [None] * nl
    U[0] = _empty(M, KE, dev)
    Usk, Usk_b, e_view = None, None, None
    if sk >= 0:
        o = lay.out_dim[sk - 1]
        if img and 1 <= sk < L8:
            Usk_b = _empty_b(M, HL, dev)  # the skip input's operand image, its tail written by the embedding
            e_view = Usk_b[:, o:o + lay.E]
            if SIGMA_FP32 and keep_u:  # (attribution) σ's fp32 source; its embedding tail is never read
                Usk = torch.zeros(M, HL, device=dev)
        else:
            Usk = _empty(M, HL, dev)
            e_view = Usk[:, o:o + lay.E]
    ops.sdf_embed(x, lay.multires, lay.scale, U[0], e_view, SQRT2)
    sdf = sdf_out if sdf_out is not None else _empty(M, 1, dev)
    fuse = _fuse_head(lay, pk)
    S7, S7b = None, None
    for l in range(nl - 1):
        into = (l + 1) == sk
        K = KE if l == 0 else rup(lay.in_dim[l], 32)
        A = Ub[l] if Ub[l] is not None else U[l]
        if l == L8 - 1 and fuse:
            # the sdf head (and the ∇-pass seed s_7 = w80 ⊙ softplus'_7) in the layer's epilogue;
            # the activation itself is stored only when a consumer needs it (not on the sampler path)
            out = _empty(M, HL, dev) if (keep_u or want_feat is not False) else None
            # bf16 mode with the folded feature head: s_7's consumers (the next ∇ GEMM, a weight
            # gradient, the elementwise last adjoint's second-order term) all read its image
            S7 = _empty(M, HL, dev) if (want_grad and not (img and want_feat is not True)) else None
            S7b = _empty_b(M, HL, dev) if (want_grad and img) else None
            ops.linear(A, pk.Bf[l], lay.out_dim[l], K, out, EPI_SOFTPLUS_HEAD, bias=pk.b[l], nzero=HL, beta=lay.beta,
                       threshold=lay.threshold, kalg=lay.in_dim[l], out1=S7, colv=pk.w80p if want_grad else None,
                       aux_beta=sig_beta(lay, l) if want_grad else 0.0, head_w=pk.w80[0], head_b=pk.b80, head_out=sdf,
                       head_idx=dst, M=M, out1_b=S7b)
            U[l + 1] = out
        else:
            ob = None
            if img and l + 1 < L8:  # the next layer's operand image, the activation's only copy
                ob = Usk_b if into else _empty_b(M, HL, dev)
                out = None
                if SIGMA_FP32 and keep_u:  # (attribution) + an fp32 copy that σ is recovered from
                    out = Usk if into else _empty(M, HL, dev)
            else:
                out = Usk if into else _empty(M, HL, dev)
            ops.linear(A, pk.Bf[l], lay.out_dim[l], K, out, EPI_SOFTPLUS, bias=pk.b[l],
                       nzero=lay.out_dim[l] if into else HL, odiv=SQRT2 if into else 1.0, beta=lay.beta,
                       threshold=lay.threshold, kalg=lay.in_dim[l], out0_b=ob)
            U[l + 1], Ub[l + 1] = out, ob
        if not keep_u and l >= 1 and (l != sk):
            U[l] = Ub[l] = None  # free as we go on the no-grad sampler path
    if not fuse:
        ops.row_head(U[L8], lay.in_dim[L8], pk.w80, pk.b80, 1, 0, sdf, dst_index=dst)
    feat = None
    if want_feat is True:
        feat = _empty(M, rup(lay.H_feat, 128), dev)
        ops.linear(U[L8], pk.Bf8, lay.H_feat, rup(lay.in_dim[L8], 32), feat, EPI_STORE, bias=pk.bf8,
                   nzero=feat.shape[1])
    G, S, Sb = None, None, None
    if want_grad:
        S, Sb = [None] * (nl - 1), [None] * (nl - 1)
        S[L8 - 1], Sb[L8 - 1] = S7, S7b
        if S7 is None and S7b is None:
            S[L8 - 1] = _empty(M, HL, dev)
            ops.scale_cols(U[L8], HL, pk.w80p, S[L8 - 1], act_beta=sig_beta(lay, L8 - 1))
        QE = _empty(M, KE, dev) if sk >= 0 else None
        for l in range(L8 - 1, 0, -1):
            Kl = rup(lay.out_dim[l], 32)
            # bf16 mode: s_l is read by the next ∇ GEMM, a weight gradient and the second-order term
            # of the adjoint (all from its image); s_0 also by the first layer's fp32 weight gradient
            Sb[l - 1] = _empty_b(M, HL, dev) if img else None
            S[l - 1] = _empty(M, HL, dev) if (not img or l - 1 == 0) else None
            A = Sb[l] if Sb[l] is not None else S[l]
            if l == sk:
                ops.linear(A, pk.Bt[l], lay.in_dim[l], Kl, S[l - 1], EPI_MUL, aux0=_act(U, Ub, l),
                           aux_beta=sig_beta(lay, l - 1), nsplit=lay.out_dim[l - 1], out_split=QE, nzero=HL,
                           adiv=SQRT2, kalg=lay.out_dim[l], out0_b=Sb[l - 1])
            else:
                ops.linear(A, pk.Bt[l], lay.out_dim[l - 1], Kl, S[l - 1], EPI_MUL, aux0=_act(U, Ub, l),
                           aux_beta=sig_beta(lay, l - 1), nzero=HL, kalg=lay.out_dim[l], out0_b=Sb[l - 1])
        Q0 = _empty(M, KE, dev)
        ops.linear(Sb[0] if Sb[0] is not None else S[0], pk.Bt[0], lay.E, rup(lay.out_dim[0], 32), Q0, EPI_STORE,
                   nzero=KE, kalg=lay.out_dim[0])
        G = _empty(M, 4, dev)
        ops.sdf_grad_assemble(lay.multires, lay.scale, U[0], Q0, QE, G)
    return {"U": U, "Ub": Ub, "S": S, "Sb": Sb, "sdf": sdf, "feat": feat, "G": G}


def sdf_input_grad(lay: SDFLayout, pk: SDFPack, st, dsdf, dfeat, dh=None):
    """dL/dx of the sdf / feature outputs (the non-detached SDF forward of
    neus_renderer.py:352; the ∇ₓSDF pass runs on detached points,
    neus_renderer.py:356, so it contributes nothing here).  Primal adjoint chain
    P_{l-1} = (W_lᵀ P_l) ⊙ σ_{l-1} from P_7 = (W_8fᵀ dfeat + dsdf w80) ⊙ σ_7, then
    dx = scale · J_emb(x)ᵀ (W_0ᵀ P_0 + skip-embedding part)."""
    U = st["U"]
    Ub = st.get("Ub") or [None] * lay.n_lin
    M, dev = U[0].shape[0], U[0].device
    nl, sk, HL, KE = lay.n_lin, lay.skip, lay.HL, lay.KE
    L8 = nl - 1
    dx = _empty(M, 4, dev)
    if dsdf is None and dfeat is None and dh is None:
        return dx.zero_()
    dsdf_flat = None if dsdf is None else dsdf.reshape(M, 1).contiguous()
    P = _empty(M, HL, dev)
    if dh is not None:  # gradient of the last hidden activation given (folded feature head): no GEMM
        ops.softplus_adjoint(U[L8], HL, P, act_beta=sig_beta(lay, L8 - 1), D=dh, rowv=dsdf_flat,
                             colv=pk.w80p if dsdf_flat is not None else None)
    elif dfeat is None:  # sdf only: P_7 = dsdf[m] w80[n] σ_7 -- elementwise, no GEMM over a zero operand
        ops.scale_cols(U[L8], HL, pk.w80p, P, act_beta=sig_beta(lay, L8 - 1), rowv=dsdf_flat)
    else:
        ops.linear(dfeat, pk.Bt8, lay.out_dim[L8 - 1], rup(lay.H_feat, 32), P, EPI_BWD_SOFTPLUS,
                   rowv=dsdf_flat, colv=pk.w80p if dsdf_flat is not None else None, aux0=U[L8],
                   aux_beta=sig_beta(lay, L8 - 1), nzero=HL)
    PE = _empty(M, KE, dev) if sk >= 0 else None
    for l in range(L8 - 1, 0, -1):
        Kl = rup(lay.out_dim[l], 32)
        Pn = _empty(M, HL, dev)
        if l == sk:
            ops.linear(P, pk.Bt[l], lay.in_dim[l], Kl, Pn, EPI_MUL, aux0=_act(U, Ub, l),
                       aux_beta=sig_beta(lay, l - 1), nsplit=lay.out_dim[l - 1], out_split=PE, nzero=HL, adiv=SQRT2,
                       kalg=lay.out_dim[l])
        else:
            ops.linear(P, pk.Bt[l], lay.out_dim[l - 1], Kl, Pn, EPI_MUL, aux0=_act(U, Ub, l),
                       aux_beta=sig_beta(lay, l - 1), nzero=HL, kalg=lay.out_dim[l])
        P = Pn
    P0 = _empty(M, KE, dev)
    ops.linear(P, pk.Bt[0], lay.E, rup(lay.out_dim[0], 32), P0, EPI_STORE, nzero=KE, kalg=lay.out_dim[0])
    ops.sdf_grad_assemble(lay.multires, lay.scale, U[0], P0, PE, dx)
    return dx


def sdf_backward(lay: SDFLayout, pk: SDFPack, st, dsdf, dfeat, dG, dh=None, want_dx=False):
    """Parameter gradients of SDFNetwork for upstream (dL/dsdf, dL/dfeature,
    dL/d∇ₓSDF); with want_dx also dL/dx, returned third.  First order (dG None) the
    parameter adjoint chain Z_l is the input adjoint chain P_l of sdf_input_grad
    (same seed, same recurrence), so dx comes from the same GEMMs: the skip layer's
    adjoint also writes its embedding columns, then W_0ᵀ Z_0 and the assembly (the
    consistency re-query of train.py:504 with pose gradients: 7 GEMM passes fewer).  The ∇ₓSDF term (the create_graph double backward of
    neus_fields.py:296) is computed forward-over-reverse:

      tangent   u̇_0 = J_emb(x)·v,  ż_l = W_l u̇_l,  u̇_{l+1} = σ_l ⊙ ż_l
      adjoint   Z_l = (W_{l+1}ᵀ Z_{l+1}) ⊙ σ_l + β s_l ⊙ (1-σ_l) ⊙ ż_l
      weights   dW_l = Σ_m Z_l u_lᵀ + s_l u̇_lᵀ,   db_l = Σ_m Z_l

    where s_l are the ∇ pass adjoints kept from the forward; dh (instead of
    dfeat): the gradient of the last hidden activation itself (folded feature
    head), so Z_7 is elementwise and the feature rows of lin8 get no gradient
    here (autograd routes theirs through the fold).  Six GEMMs per
    layer instead of autograd's nine.  σ_l is recovered from
    U[l+1] inside every epilogue (sig_beta), and the second-order term is rebuilt
    by the adjoint's epilogue from s_l and u̇_{l+1} (ż_l = u̇_{l+1} c / σ_l), so the
    tangent pass writes one buffer per layer, not two.
    """
    wmode = _wgrad_mode(pk)
    U, S = st["U"], st["S"]
    M, dev = U[0].shape[0], U[0].device
    nl, sk, HL, KE = lay.n_lin, lay.skip, lay.HL, lay.KE
    L8 = nl - 1
    img = _img_mode(pk, lay)
    Ub = st.get("Ub") or [None] * nl
    Sb = st.get("Sb") or [None] * (nl - 1)
    second = dG is not None
    if second and S is None:
        raise RuntimeError("SDF double backward needs the ∇ pass buffers (want_grad=True in forward)")

    def s_fp32(l):
        """s_l in fp32.  The bf16-mode forward with the folded head keeps s_7 as an image only; the paths
        that read it in fp32 (a second-order term without dh, a weight-gradient pair whose Y is fp32)
        rebuild it from the stored activation: s_7 = w80 ⊙ σ_7."""
        if S[l] is None:
            if l != L8 - 1:
                raise RuntimeError(f"sdf_backward: s_{l} was not kept in fp32")
            S[l] = _empty(M, HL, dev)
            ops.scale_cols(U[L8], HL, pk.w80p, S[l], act_beta=sig_beta(lay, L8 - 1))
        return S[l]
    i8 = lay.in_dim[L8]
    # dW8[0] = Σ_m dsdf U8 (+ Ud8) / scale: fused into the adjoint kernel on the folded-head path
    # (also on the sdf-only first-order path, e.g. the consistency re-query: Z_7 = dsdf w80 σ_7)
    sdf_only = dh is None and dfeat is None and not second and dsdf is not None
    fused_cs = i8 == HL and ((dh is not None and (dsdf is not None or second)) or sdf_only)
    # bf16 mode: the top tangent u̇_8 and s_7 reach the elementwise last adjoint (and its fused column
    # sums) as images
    top_img = img and second and dh is not None and fused_cs and Sb[L8 - 1] is not None
    Ud, Udb = None, [None] * nl
    if second:
        Ud = [None] * nl
        Ud[0] = _empty(M, KE, dev)
        Usk_d, Usk_db, e_view = None, None, None
        if sk >= 0:
            o = lay.out_dim[sk - 1]
            if img and 1 <= sk < L8:  # the tangent's skip input as an operand image (tail from the prep)
                Usk_db = _empty_b(M, HL, dev)
                e_view = Usk_db[:, o:o + lay.E]
            else:
                Usk_d = _empty(M, HL, dev)
                e_view = Usk_d[:, o:o + lay.E]
        ops.sdf_tangent_prep(lay.multires, lay.scale, U[0], dG, Ud[0], e_view, SQRT2)
        for l in range(nl - 1):
            into = (l + 1) == sk
            # bf16 mode: u̇_{l+1} is read by the next tangent GEMM, a weight gradient and the adjoint's
            # second-order term (all from its image); u̇_8 by the elementwise last adjoint (an image with
            # top_img, else fp32)
            if img and (l + 1 < L8 or top_img):
                out, ob = None, (Usk_db if into else _empty_b(M, HL, dev))
            else:
                out, ob = (Usk_d if into else _empty(M, HL, dev)), None
            K = KE if l == 0 else rup(lay.in_dim[l], 32)
            A = Udb[l] if Udb[l] is not None else Ud[l]
            ops.linear(A, pk.Bf[l], lay.out_dim[l], K, out, EPI_TANGENT, aux0=_act(U, Ub, l + 1),
                       aux_beta=sig_beta(lay, l),
                       nzero=lay.out_dim[l] if into else HL, odiv=SQRT2 if into else 1.0, beta=lay.beta,
                       kalg=lay.in_dim[l], out0_b=ob)
            Ud[l + 1], Udb[l + 1] = out, ob

    def z_img(l):
        """Z_l as a bf16 operand image only (its consumers: the next adjoint GEMM and the weight
        gradient, whose second pair's Y is S_l: that must have an image too)."""
        return img and 1 <= l < L8 and (not second or Sb[l] is not None) and Ub[l] is not None

    o8 = lay.out_dim[L8]
    dW8 = torch.empty(o8, i8, device=dev)
    db8 = torch.empty(o8, device=dev)
    if dfeat is not None and dh is None:
        ops.wgrad(dfeat, U[L8], lay.H_feat, i8, dW8[1:], db=db8[1:], mode=wmode)
    else:
        dW8[1:].zero_()
        db8[1:].zero_()
    dsdf_flat = None
    if dsdf is not None:
        dsdf = dsdf.reshape(M, 1).contiguous()
        dsdf_flat = dsdf
        if not fused_cs:
            ops.colsum(U[L8], i8, dW8[0], w=dsdf, wdiv=lay.scale)
            ops.colsum(dsdf, 1, db8[0:1], wdiv=lay.scale)
    else:
        if not fused_cs:
            dW8[0].zero_()
        db8[0].zero_()
    if second and not fused_cs:
        ops.colsum(Ud[L8], i8, dW8[0], wdiv=lay.scale, accumulate=True)

    def second_order(l):  # BWD_SOFTPLUS inputs of β s_l (1-σ_l) ż_l, ż_l = u̇_{l+1} c_l / σ_l
        if not second:
            return {}
        # (bf16 mode: the images; the top layer's only on the elementwise path, top_img)
        img2 = (l < L8 - 1 or top_img) and Sb[l] is not None and Udb[l + 1] is not None
        a1, a2 = (Sb[l], Udb[l + 1]) if img2 else (s_fp32(l), Ud[l + 1])
        if img2 and SIGMA_FP32:  # (attribution) the image values in fp32, the dtype of σ's fp32 source
            a1, a2 = a1.float(), a2.float()
        return dict(aux1=a1, aux2=a2, aux2_scale=lay.beta * (SQRT2 if (l + 1) == sk else 1.0))

    Z = _empty_b(M, HL, dev) if (z_img(L8 - 1) and (dh is not None or (sdf_only and fused_cs))) else _empty(M, HL, dev)
    if dh is not None:  # Z_7 = (dh + dsdf w80) σ_7 + the second-order term: elementwise
        so = second_order(L8 - 1)
        ops.softplus_adjoint(U[L8], HL, Z, act_beta=sig_beta(lay, L8 - 1), D=dh, rowv=dsdf_flat,
                             colv=pk.w80p if dsdf_flat is not None else None, aux1=so.get("aux1"),
                             aux2=so.get("aux2"), aux2_scale=so.get("aux2_scale", 0.0),
                             cs_out=dW8[0] if fused_cs else None,
                             rs_out=db8[0:1] if (fused_cs and dsdf_flat is not None) else None, cs_div=lay.scale)
    elif sdf_only:
        # sdf only, first order (e.g. SDFNetwork.sdf at train.py:504): Z_7 = dsdf[m] w80[n] σ_7,
        # elementwise -- no GEMM over a zero feature gradient; lin8's sdf row / bias gradients
        # from the same pass when fused_cs
        if fused_cs:
            ops.softplus_adjoint(U[L8], HL, Z, act_beta=sig_beta(lay, L8 - 1), rowv=dsdf_flat, colv=pk.w80p,
                                 cs_out=dW8[0], rs_out=db8[0:1], cs_div=lay.scale)
        else:
            ops.scale_cols(U[L8], HL, pk.w80p, Z, act_beta=sig_beta(lay, L8 - 1), rowv=dsdf_flat)
    else:
        phi = dfeat if dfeat is not None else torch.zeros(M, lay.H_feat, device=dev)
        ops.linear(phi, pk.Bt8, lay.out_dim[L8 - 1], rup(lay.H_feat, 32), Z, EPI_BWD_SOFTPLUS,
                   rowv=dsdf_flat, colv=pk.w80p if dsdf_flat is not None else None, aux0=U[L8],
                   aux_beta=sig_beta(lay, L8 - 1), nzero=HL, **second_order(L8 - 1))
    dWs, dbs = [None] * nl, [None] * nl
    dWs[L8], dbs[L8] = dW8, db8
    share = want_dx and not second  # Z_l == P_l: dx from the parameter adjoint chain
    PE = _empty(M, KE, dev) if (share and sk >= 0) else None
    wq = ops.WgradQueue()  # the hidden layers' weight gradients: one launch after the chain
    for l in range(L8 - 1, -1, -1):
        Zl = Z
        if l > 0:
            zb = z_img(l - 1)  # Z_{l-1} as an operand image only
            Z = _empty_b(M, HL, dev) if zb else _empty(M, HL, dev)
            zo = dict(out0_b=Z) if zb else {}
            if share and l == sk:  # + the embedding columns of the skip input (sdf_input_grad's PE)
                ops.linear(Zl, pk.Bt[l], lay.in_dim[l], rup(lay.out_dim[l], 32), None if zb else Z, EPI_MUL,
                           aux0=_act(U, Ub, l), aux_beta=sig_beta(lay, l - 1), nsplit=lay.out_dim[l - 1], out_split=PE,
                           nzero=HL, adiv=SQRT2, kalg=lay.out_dim[l], **zo)
            else:
                # first order only (no second-order term): Z = (W̃ᵀZ)σ is the MUL epilogue, which runs on
                # the 256x256 tile (BWD_SOFTPLUS would add an all-zero term on the 128x128 tile)
                ops.linear(Zl, pk.Bt[l], lay.out_dim[l - 1], rup(lay.out_dim[l], 32), None if zb else Z,
                           EPI_BWD_SOFTPLUS if second else EPI_MUL,
                           aux0=_act(U, Ub, l), aux_beta=sig_beta(lay, l - 1), nzero=HL,
                           adiv=SQRT2 if l == sk else 1.0,
                           kalg=lay.out_dim[l], **second_order(l - 1), **zo)
        dW = torch.empty(lay.out_dim[l], lay.in_dim[l], device=dev)
        db = torch.empty(lay.out_dim[l], device=dev)
        # the operands in one format per side: the images where Z_l is one (Y) / where U_l has one (X)
        yb = Zl.dtype == torch.bfloat16
        xb = Ub[l] is not None and (not second or Udb[l] is not None)
        wq.add(Zl, Ub[l] if xb else U[l], lay.out_dim[l], lay.in_dim[l], dW, db=db,
               Y1=(Sb[l] if yb else s_fp32(l)) if second else None, X1=(Udb[l] if xb else Ud[l]) if second else None,
               mode=wmode)
        dWs[l], dbs[l] = dW, db
    wq.flush()
    if not want_dx:
        return dWs, dbs
    if not share:
        dx = sdf_input_grad(lay, pk, st, dsdf, dfeat, dh=dh)
        return dWs, dbs, dx
    P0 = _empty(M, KE, dev)  # Zl is Z_0 here
    ops.linear(Zl, pk.Bt[0], lay.E, rup(lay.out_dim[0], 32), P0, EPI_STORE, nzero=KE, kalg=lay.out_dim[0])
    dx = _empty(M, 4, dev)
    ops.sdf_grad_assemble(lay.multires, lay.scale, U[0], P0, PE, dx)
    return dWs, dbs, dx


# SDFNetwork.sdf under autograd (the stage-1 consistency re-query, train.py:502-505) through the composed
# entry points cn_mlp_fwd / cn_mlp_bwd (bitwise the layer-by-layer composition below); the per-kernel
# timer (ops.set_timer) sees the launches only when they are made one by one, so it keeps the composition
MLP_NATIVE = True


class _SDFFieldFn(torch.autograd.Function):
    """(x [M,4], weights...) -> (sdf [M,1], feature [M,H], ∇ₓSDF [M,4])."""

    @staticmethod
    def forward(ctx, x, lay, pk, want_feat, want_grad, *params):
        ctx.set_materialize_grads(False)
        keep = any(ctx.needs_input_grad[5:]) or ctx.needs_input_grad[0]
        ctx.nparams = len(params)
        if keep and want_feat is False and not want_grad and MLP_NATIVE and ops._timer is None:
            net, refs = ops.sdf_net(lay, pk)
            sdf = _empty(x.shape[0], 1, x.device)
            state = ops.mlp_fwd(net, x, sdf.view(-1))
            ctx.lay, ctx.hidden, ctx.st = lay, False, None
            ctx.native = (net, refs, state)
            feat, G = x.new_empty(0), x.new_empty(0)
            ctx.mark_non_differentiable(feat, G)
            return sdf, feat, G
        ctx.native = None
        st = sdf_forward(lay, pk, x, want_feat=want_feat, want_grad=want_grad, keep=keep)
        ctx.lay, ctx.pk, ctx.st = lay, pk, (st if keep else None)
        ctx.hidden = want_feat == "hidden"
        empty = x.new_empty(0)
        if ctx.hidden:  # the last hidden activation in place of the feature (folded feature head)
            feat = st["U"][lay.n_lin - 1][:, :lay.in_dim[lay.n_lin - 1]]
        else:
            feat = st["feat"][:, :lay.H_feat] if want_feat else empty
        G = st["G"] if want_grad else x.new_empty(0)
        if not want_feat:
            ctx.mark_non_differentiable(feat)
        if not want_grad:
            ctx.mark_non_differentiable(G)
        return st["sdf"], feat, G

    @staticmethod
    def backward(ctx, dsdf, dfeat, dG):
        none4 = (None,) * 4
        if ctx.native is not None:
            return _SDFFieldFn._native_backward(ctx, dsdf)
        if ctx.st is None:
            return (None,) + none4 + (None,) * ctx.nparams
        if dfeat is not None and dfeat.stride(1) != 1:
            dfeat = dfeat.contiguous()
        if dG is not None:
            dG = dG.contiguous()
        dh = None
        if ctx.hidden:
            dh, dfeat = dfeat, None
        want_dx = ctx.needs_input_grad[0]
        dx = None
        grads = [None] * ctx.nparams
        if any(ctx.needs_input_grad[5:]):
            res = sdf_backward(ctx.lay, ctx.pk, ctx.st, dsdf, dfeat, dG, dh=dh, want_dx=want_dx)
            dWs, dbs = res[0], res[1]
            if want_dx:
                dx = res[2]
            grads = []
            for w, b in zip(dWs, dbs):
                grads += [w, b]
        elif want_dx:
            dx = sdf_input_grad(ctx.lay, ctx.pk, ctx.st, dsdf, dfeat, dh=dh)
        ctx.st = None
        return (dx,) + none4 + tuple(grads)

    @staticmethod
    def _native_backward(ctx, dsdf):
        """cn_mlp_bwd: sdf_backward (sdf only, first order, want_dx) or sdf_input_grad in one call."""
        net, refs, state = ctx.native
        ctx.native = None
        lay = ctx.lay
        none4 = (None,) * 4
        want_dx, params = ctx.needs_input_grad[0], any(ctx.needs_input_grad[5:])
        if dsdf is None or not (want_dx or params):
            return (None,) + none4 + (None,) * ctx.nparams
        dev = dsdf.device
        M = dsdf.shape[0]
        dWs = [torch.empty(lay.out_dim[l], lay.in_dim[l], device=dev) for l in range(lay.n_lin)] if params else None
        dbs = [torch.empty(lay.out_dim[l], device=dev) for l in range(lay.n_lin)] if params else None
        dx = _empty(M, 4, dev) if want_dx else None
        ops.mlp_bwd(net, M, state, dsdf.reshape(M).contiguous(), dWs, dbs, dx)
        del refs, state
        grads = [None] * ctx.nparams
        if params:
            grads = []
            for w, b in zip(dWs, dbs):
                grads += [w, b]
        return (dx,) + none4 + tuple(grads)


def _init_geometric(lin: nn.Linear, l: int, dims, out_dim, skip_in, multires, n_lin, bias, inside_outside,
                    d_pos: int):
    """Geometric (sphere) initialisation of IDR / NeuS (neus_fields.py:241-259),
    in the same RNG order as the reference so seeded builds give equal weights."""
    if l == n_lin - 1:
        mean = np.sqrt(np.pi) / np.sqrt(dims[l])
        torch.nn.init.normal_(lin.weight, mean=-mean if inside_outside else mean, std=0.0001)
        torch.nn.init.constant_(lin.bias, bias if inside_outside else -bias)
    elif multires > 0 and l == 0:
        torch.nn.init.constant_(lin.bias, 0.0)
        torch.nn.init.constant_(lin.weight[:, d_pos:], 0.0)
        torch.nn.init.normal_(lin.weight[:, :d_pos], 0.0, np.sqrt(2) / np.sqrt(out_dim))
    elif multires > 0 and l in skip_in:
        torch.nn.init.constant_(lin.bias, 0.0)
        torch.nn.init.normal_(lin.weight, 0.0, np.sqrt(2) / np.sqrt(out_dim))
        torch.nn.init.constant_(lin.weight[:, -(dims[0] - d_pos):], 0.0)
    else:
        torch.nn.init.constant_(lin.bias, 0.0)
        torch.nn.init.normal_(lin.weight, 0.0, np.sqrt(2) / np.sqrt(out_dim))


class SDFNetwork(nn.Module):
    """Reference: model/neus_fields.py:205-303 (IDR SDF MLP, Softplus(beta=100))."""

    def __init__(self, d_in, d_out, d_hidden, n_layers, skip_in=(4,), multires=0, bias=0.5, scale=1,
                 geometric_init=True, weight_norm=True, inside_outside=False):
        super().__init__()
        dims = [d_in] + [d_hidden for _ in range(n_layers)] + [d_out]
        if multires > 0:
            dims[0] = embed_dim(multires, d_in)
        self.d_in = d_in
        self.multires = multires
        self.num_layers = len(dims)
        self.skip_in = list(skip_in)
        self.scale = scale
        self.dims = dims
        n_lin = self.num_layers - 1
        for l in range(n_lin):
            out_dim = dims[l + 1] - dims[0] if (l + 1) in self.skip_in else dims[l + 1]
            lin = nn.Linear(dims[l], out_dim)
            if geometric_init:
                _init_geometric(lin, l, dims, out_dim, self.skip_in, multires, n_lin, bias, inside_outside, 4)
            if weight_norm:
                lin = nn.utils.weight_norm(lin)
            setattr(self, "lin" + str(l), lin)
        self.activation = nn.Softplus(beta=100)
        self._layout = None
        self.mfma_dtype = "fp32"  # "bf16": bf16-operand MFMA GEMMs (config C3); not part of the state dict
        release_weight_norm_graphs(self)

    # -- kernel plumbing ---------------------------------------------------
    def layout(self) -> SDFLayout:
        if self._layout is None:
            if self.d_in != 4:
                raise NotImplementedError("copenerf SDF kernels take (x, y, z, t) inputs (d_in = 4)")
            if len(self.skip_in) > 1 or any(s <= 0 for s in self.skip_in):
                raise NotImplementedError("copenerf SDF kernels support one skip connection")
            n_lin = self.num_layers - 1
            in_dim, out_dim = [], []
            for l in range(n_lin):
                lin = getattr(self, "lin" + str(l))
                w = lin.weight_v if hasattr(lin, "weight_v") else lin.weight
                out_dim.append(w.shape[0])
                in_dim.append(w.shape[1])
            E = self.dims[0]
            hl = rup(max(max(in_dim[1:]), max(out_dim[:-1])), 128)  # hidden buffers (feature has its own)
            self._layout = SDFLayout(n_lin=n_lin, in_dim=in_dim, out_dim=out_dim, E=E, KE=rup(E, 64), HL=hl,
                                     skip=self.skip_in[0] if self.skip_in else -1, multires=self.multires,
                                     scale=float(self.scale), beta=float(self.activation.beta),
                                     threshold=float(self.activation.threshold))
        return self._layout

    def params_and_pack(self):
        """Effective weights (autograd-tracked) and their padded kernel images."""
        lay = self.layout()
        lins = [getattr(self, "lin" + str(l)) for l in range(lay.n_lin)]
        Ws = effective_weights(lins)
        bs = [lin.bias for lin in lins]
        return Ws, bs, pack_sdf(lay, Ws, bs, self.mfma_dtype)

    def field(self, x, *, want_feat=True, want_grad=True, packed=None):
        """Fused (sdf, feature, ∇ₓsdf) of the points x [M, 4] in one launch sequence
        (want_feat="hidden": the last hidden activation instead of the feature)."""
        Ws, bs, pk = packed if packed is not None else self.params_and_pack()
        params = []
        for w, b in zip(Ws, bs):
            params += [w, b]
        x = x.contiguous()
        return _SDFFieldFn.apply(x, self.layout(), pk, want_feat, want_grad, *params)

    # -- reference API -------------------------------------------------------
    def forward(self, inputs):
        sdf, feat, _ = self.field(inputs, want_feat=True, want_grad=False)
        return torch.cat([sdf, feat], dim=-1)

    def sdf(self, x):
        sdf, _, _ = self.field(x, want_feat=False, want_grad=False)
        return sdf

    def sdf_hidden_appearance(self, x):
        return self.forward(x)

    def gradient(self, x):
        _, _, g = self.field(x.detach(), want_feat=False, want_grad=True)
        return g.unsqueeze(1)


# ---------------------------------------------------------------------------
# Colour network (mode 'idr')
@dataclasses.dataclass
class ColorLayout:
    F: int          # feature width (256)
    P: int          # point width (4: pts_time)
    V: int          # encoded view-dir width (27)
    Gd: int         # gradient width (4)
    KX: int         # padded extras width (64)
    HL: int
    n_lin: int
    in_dim: List[int]
    out_dim: List[int]
    multires_view: int


@dataclasses.dataclass
class ColorPack:
    Bf: list
    Bt: list
    b: list
    W3: torch.Tensor   # [3][H]
    b3: torch.Tensor
    Btf: torch.Tensor  # feature columns of lin0, transposed
    Wg: torch.Tensor   # [4][H]: gradient columns of lin0, transposed
    Bxt: torch.Tensor  # [64][Hpad]: extras columns [g | pts | emb(dirs)] of lin0, transposed (ray gradients)


def pack_color(lay: ColorLayout, Ws, bs, mfma_dtype: str = "fp32") -> ColorPack:
    """GEMM images of the colour network in one cn_pack_weights launch.  lin0's
    columns [pts | emb(dirs) | gradient | feature] (neus_fields.py:352-356) are
    permuted to [feature | gradient | pts | emb | 0] to match the operands
    (feature, extras) of the first GEMM."""
    kq = _kq(mfma_dtype)
    pk = ops.ImagePacker(mfma_dtype)
    with torch.no_grad():
        dev = Ws[0].device
        P, V, Gd, Fd = lay.P, lay.V, lay.Gd, lay.F
        W0 = Ws[0].detach().contiguous()
        o = W0.shape[0]
        pts, emb, g, feat = (W0[:, 0:P], W0[:, P:P + V], W0[:, P + V:P + V + Gd], W0[:, P + V + Gd:])
        B0 = pk.image(rup(o, 128), Fd + lay.KX, dev)
        pk.put(B0, feat, c0=0, c1=Fd)
        pk.put(B0, g, c0=Fd, c1=Fd + Gd)
        pk.put(B0, pts, c0=Fd + Gd, c1=Fd + Gd + P)
        pk.put(B0, emb, c0=Fd + Gd + P, c1=Fd + lay.KX)
        Bf, Bt = [B0], [None]
        b = [bs[0].detach().contiguous()]
        for l in range(1, lay.n_lin - 1):
            W = Ws[l].detach().contiguous()
            oo, ii = W.shape
            Bf.append(pk.put(pk.image(rup(oo, 128), rup(ii, kq), dev), W))
            Bt.append(pk.put(pk.image(rup(ii, 128), rup(oo, kq), dev), W, transpose=True))
            b.append(bs[l].detach().contiguous())
        Btf = pk.put(pk.image(rup(Fd, 128), rup(o, kq), dev), feat, transpose=True)
        Wg = pk.put(pk.image(Gd, o, dev, fmt="fp32"), g, transpose=True, fmt="fp32")
        # extras columns [g | pts | emb] of lin0, transposed, rows padded to 64
        Bxt = pk.image(64, rup(o, kq), dev)
        pk.put(Bxt, g, transpose=True, r0=0, r1=Gd)
        pk.put(Bxt, pts, transpose=True, r0=Gd, r1=Gd + P)
        pk.put(Bxt, emb, transpose=True, r0=Gd + P, r1=64)
        pk.run()
        return ColorPack(Bf, Bt, b, Ws[-1].detach().contiguous(), bs[-1].detach().contiguous(), Btf, Wg, Bxt)


class _ColorFieldFn(torch.autograd.Function):
    """(pts_time [M,4], dirs, ∇ₓSDF [M,4], feature [M,F], weights...) -> rgb [M,3]."""

    @staticmethod
    def forward(ctx, pts, dirs, dir_div, G, feat, lay, pk, *params):
        ctx.set_materialize_grads(False)
        M, dev = pts.shape[0], pts.device
        ext = _empty(M, lay.KX, dev)
        ops.color_extras(G, pts, dirs, dir_div, lay.multires_view, ext)
        H = []
        img = _img_mode(pk, lay)
        A, A2, K1, K = feat, ext, lay.F, lay.F + lay.KX
        for l in range(lay.n_lin - 1):
            # bf16 mode: the hidden activations but the last are read only as GEMM operands (the next
            # layer, the weight gradient) and for ReLU's sign (BWD_RELU): bf16 operand images only
            if img and l < lay.n_lin - 2:
                out = _empty_b(M, lay.HL, dev)
                ops.linear(A, pk.Bf[l], lay.out_dim[l], K, None, EPI_RELU, bias=pk.b[l], A2=A2, K1=K1, nzero=lay.HL,
                           kalg=lay.in_dim[l], out0_b=out)
            else:
                out = _empty(M, lay.HL, dev)
                ops.linear(A, pk.Bf[l], lay.out_dim[l], K, out, EPI_RELU, bias=pk.b[l], A2=A2, K1=K1, nzero=lay.HL,
                           kalg=lay.in_dim[l])
            H.append(out)
            A, A2, K1, K = out, None, None, rup(lay.out_dim[l], 32)
        rgb = _empty(M, 3, dev)
        ops.row_head(H[-1], lay.in_dim[-1], pk.W3, pk.b3, 3, 1, rgb)
        ctx.lay, ctx.pk = lay, pk
        ctx.bufs = (feat, ext, H, rgb)
        ctx.dirs, ctx.dir_div = (dirs, dir_div) if ctx.needs_input_grad[1] else (None, 1)
        return rgb

    @staticmethod
    def backward(ctx, drgb):
        lay, pk = ctx.lay, ctx.pk
        wmode = _wgrad_mode(pk)
        feat, ext, H, rgb = ctx.bufs
        ctx.bufs = None
        nparams = 2 * lay.n_lin
        if drgb is None:
            return (None,) * (7 + nparams)
        M, dev = rgb.shape[0], rgb.device
        drgb = drgb.contiguous()
        n = lay.n_lin
        dWs, dbs = [None] * n, [None] * n
        dWs[n - 1] = torch.empty(3, lay.in_dim[n - 1], device=dev)
        dbs[n - 1] = torch.empty(3, device=dev)
        # bf16 mode: the last hidden layer's adjoint as an operand image (read by the next adjoint GEMM
        # and a weight gradient only)
        dZ = _empty_b(M, lay.HL, dev) if (_img_mode(pk, lay) and n - 2 >= 1) else _empty(M, lay.HL, dev)
        ops.rgb_head_bwd(drgb, rgb, H[-1], lay.in_dim[n - 1], pk.W3, dZ, dWs[n - 1], dbs[n - 1])
        wq = ops.WgradQueue()  # the 256x256 weight gradients: one launch after the chain
        for l in range(n - 2, 0, -1):
            dW = torch.empty(lay.out_dim[l], lay.in_dim[l], device=dev)
            db = torch.empty(lay.out_dim[l], device=dev)
            wq.add(dZ, H[l - 1], lay.out_dim[l], lay.in_dim[l], dW, db=db, mode=wmode)
            dWs[l], dbs[l] = dW, db
            if _img_mode(pk, lay) and l - 1 >= 1:  # dZ_{l-1}: read by the next adjoint GEMM and a weight gradient only
                dZp = _empty_b(M, lay.HL, dev)
                ops.linear(dZ, pk.Bt[l], lay.out_dim[l - 1], rup(lay.out_dim[l], 32), None, EPI_BWD_RELU,
                           aux0=H[l - 1], nzero=lay.HL, out0_b=dZp)
            else:
                dZp = _empty(M, lay.HL, dev)
                ops.linear(dZ, pk.Bt[l], lay.out_dim[l - 1], rup(lay.out_dim[l], 32), dZp, EPI_BWD_RELU,
                           aux0=H[l - 1], nzero=lay.HL)
            dZ = dZp
        o0 = lay.out_dim[0]
        dWf = torch.empty(o0, lay.F, device=dev)
        db0 = torch.empty(o0, device=dev)
        dWx = torch.empty(o0, lay.KX, device=dev)
        wq.add(dZ, feat, o0, lay.F, dWf, db=db0, mode=wmode)
        ops.wgrad(dZ, ext, o0, lay.KX, dWx, mode=wmode)
        wq.flush()
        P, V, Gd = lay.P, lay.V, lay.Gd
        dfeat = None
        if ctx.needs_input_grad[4]:
            dfeat = _empty(M, lay.F, dev)
            ops.linear(dZ, pk.Btf, lay.F, rup(o0, 32), dfeat, EPI_STORE, nzero=lay.F)
        dG = dpts = ddirs = None
        if ctx.needs_input_grad[0] or ctx.needs_input_grad[1]:
            # ray / pose gradients: d ext = dZ0 W0[:, ext] in one GEMM, ext = [g | pts | emb(dirs)]
            d_ext = _empty(M, 64, dev)
            ops.linear(dZ, pk.Bxt, rup(Gd + P + V, 4), rup(o0, 32), d_ext, EPI_STORE, nzero=64, kalg=o0)
            if ctx.needs_input_grad[3]:
                dG = d_ext[:, 0:Gd]
            if ctx.needs_input_grad[0]:
                dpts = d_ext[:, Gd:Gd + P]
            if ctx.needs_input_grad[1]:
                dirs = ctx.dirs
                ddirs = torch.empty(dirs.shape[0], 3, device=dev)
                ops.color_extras_bwd(d_ext, dirs, ctx.dir_div, lay.multires_view, ddirs)
        elif ctx.needs_input_grad[3]:
            dG = _empty(M, Gd, dev)
            ops.row_head(dZ, o0, pk.Wg, None, Gd, 0, dG)
        # back to the reference column order [pts | emb(dirs) | gradients | feature]
        dWs[0] = torch.cat([dWx[:, Gd:Gd + P], dWx[:, Gd + P:Gd + P + V], dWx[:, 0:Gd], dWf], 1)
        dbs[0] = db0
        grads = []
        for w, b in zip(dWs, dbs):
            grads += [w, b]
        return (dpts, ddirs, None, dG, dfeat, None, None) + tuple(grads)


class RenderingNetwork(nn.Module):
    """Reference: model/neus_fields.py:307-374."""

    def __init__(self, d_feature, mode, d_in, d_out, d_hidden, n_layers, weight_norm=True, multires_view=0,
                 squeeze_out=True, use_negative_ray_vector=False):
        super().__init__()
        self.mode = mode
        self.squeeze_out = squeeze_out
        self.use_negative_ray_vector = use_negative_ray_vector
        dims = [d_in + d_feature] + [d_hidden for _ in range(n_layers)] + [d_out]
        self.multires_view = multires_view
        if multires_view > 0:
            dims[0] += embed_dim(multires_view, 3) - 3
        self.num_layers = len(dims)
        self.d_feature = d_feature
        self.d_in = d_in
        for l in range(0, self.num_layers - 1):
            lin = nn.Linear(dims[l], dims[l + 1])
            if weight_norm:
                lin = nn.utils.weight_norm(lin)
            setattr(self, "lin" + str(l), lin)
        self.relu = nn.ReLU()
        self._layout = None
        self.mfma_dtype = "fp32"  # see SDFNetwork.mfma_dtype
        release_weight_norm_graphs(self)

    def layout(self) -> ColorLayout:
        if self._layout is None:
            if self.mode != "idr" or not self.squeeze_out or self.use_negative_ray_vector:
                raise NotImplementedError("copenerf colour kernels implement mode='idr', squeeze_out=True, "
                                          "use_negative_ray_vector=False (every shipped config)")
            n = self.num_layers - 1
            in_dim, out_dim = [], []
            for l in range(n):
                lin = getattr(self, "lin" + str(l))
                w = lin.weight_v if hasattr(lin, "weight_v") else lin.weight
                out_dim.append(w.shape[0])
                in_dim.append(w.shape[1])
            V = embed_dim(self.multires_view, 3)
            P, Gd = 4, 4
            if self.d_in != P + 3 + Gd or out_dim[-1] != 3 or self.d_feature % 32 != 0:
                raise NotImplementedError("copenerf colour kernels expect d_in = 11 (pts_time, dirs, gradients), "
                                          "d_out = 3, d_feature % 32 == 0")
            hl = rup(max(out_dim[:-1]), 128)
            self._layout = ColorLayout(F=self.d_feature, P=P, V=V, Gd=Gd, KX=rup(P + V + Gd, 64), HL=hl, n_lin=n,
                                       in_dim=in_dim, out_dim=out_dim, multires_view=self.multires_view)
        return self._layout

    def params_and_pack(self, fold_feature=None):
        """Effective weights and their kernel images.  fold_feature=(W8, b8), the SDF's
        last Linear (row 0 sdf, rows 1: the feature head): lin0's feature columns W0f are
        replaced by W0f @ W8[1:] and its bias by b0 + W0f @ b8[1:], so the first layer
        reads the SDF's last hidden activation h directly:
            W0f (W8[1:] h + b8[1:]) + b0  =  (W0f W8[1:]) h + (b0 + W0f b8[1:]).
        The products are torch ops on the effective weights: autograd takes the
        gradient of the folded weight back to both networks' parameters."""
        lay = self.layout()
        lins = [getattr(self, "lin" + str(l)) for l in range(lay.n_lin)]
        Ws = effective_weights(lins)
        bs = [lin.bias for lin in lins]
        if fold_feature is not None:
            W8, b8 = fold_feature
            c = lay.P + lay.V + lay.Gd
            W0f = Ws[0][:, c:]
            # in float64: exact to fp32 rounding, and faster than hipBLASLt's fp32 kernel for 256^3
            Ws[0] = torch.cat([Ws[0][:, :c], (W0f.double() @ W8[1:].double()).float()], 1)
            bs[0] = bs[0] + (W0f.double() @ b8[1:].double()).float()
        return Ws, bs, pack_color(lay, Ws, bs, self.mfma_dtype)

    def color(self, points, normals, dirs, dir_div, feature_vectors, packed=None):
        """rgb [M,3]; dirs is [M/dir_div, 3] (one row per ray when dir_div = S)."""
        Ws, bs, pk = packed if packed is not None else self.params_and_pack()
        params = []
        for w, b in zip(Ws, bs):
            params += [w, b]
        if feature_vectors.stride(1) != 1:
            feature_vectors = feature_vectors.contiguous()
        return _ColorFieldFn.apply(points.contiguous(), dirs.contiguous(), int(dir_div), normals.contiguous(),
                                   feature_vectors, self.layout(), pk, *params)

    def forward(self, points, normals, view_dirs, feature_vectors):
        return self.color(points, normals, view_dirs, 1, feature_vectors)


class SingleVarianceNetwork(nn.Module):
    """Reference: model/neus_fields.py:459-465."""

    def __init__(self, init_val):
        super().__init__()
        self.register_parameter("variance", nn.Parameter(torch.tensor(init_val)))

    def forward(self, x):
        return torch.ones([len(x), 1], device=self.variance.device) * torch.exp(self.variance * 10.0)


class NeRF(nn.Module):
    """Reference: model/neus_fields.py:378-456.  Background (NeRF++) density MLP;
    constructed by train.py:39 so checkpoints keep their keys, but rendered only
    when n_outside > 0, which no shipped config sets -- out of scope here."""

    def __init__(self, D=8, W=256, d_in=3, d_in_view=3, multires=0, multires_view=0, output_ch=4, skips=[4],
                 use_viewdirs=False):
        super().__init__()
        self.D, self.W, self.d_in, self.d_in_view = D, W, d_in, d_in_view
        self.input_ch = embed_dim(multires, d_in) if multires > 0 else 3
        self.input_ch_view = embed_dim(multires_view, d_in_view) if multires_view > 0 else 3
        self.skips = skips
        self.use_viewdirs = use_viewdirs
        self.pts_linears = nn.ModuleList(
            [nn.Linear(self.input_ch, W)] +
            [nn.Linear(W, W) if i not in self.skips else nn.Linear(W + self.input_ch, W) for i in range(D - 1)])
        self.views_linears = nn.ModuleList([nn.Linear(self.input_ch_view + W, W // 2)])
        if use_viewdirs:
            self.feature_linear = nn.Linear(W, W)
            self.alpha_linear = nn.Linear(W, 1)
            self.rgb_linear = nn.Linear(W // 2, 3)
        else:
            self.output_linear = nn.Linear(W, output_ch)

    def forward(self, input_pts, input_views):
        raise NotImplementedError("NeRF++ background branch (n_outside > 0) is out of scope (SURVEY.md §2)")
