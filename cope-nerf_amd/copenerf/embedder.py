"""Positional encoding (reference: model/neus_embedder.py:6-51).

Only the dimension bookkeeping lives here: on the hot path the encoding is
computed by the HIP kernels cn_sdf_embed / cn_color_extras (csrc/cn_fields.hip),
which write the first layers' operand rows (in bf16 mode the skip input's
embedding tail straight into its operand image) for the first Linear to read;
the round-3 fusion into that Linear's operand staging was measured no faster
and removed in round 4.  `get_embedder` keeps the reference's call signature
(multires, input_dims) -> (fn, out_dim) for API compatibility; its fn is a
torch expression usable on any device, used by tests and by the out-of-scope
NeRF branch only.
"""
from __future__ import annotations

import torch


def embed_dim(multires: int, input_dims: int = 3) -> int:
    """include_input + [sin, cos] x multires bands (neus_embedder.py:13-27)."""
    return input_dims * (1 + 2 * multires) if multires > 0 else input_dims


def embed(x: torch.Tensor, multires: int) -> torch.Tensor:
    """[x, sin(2^0 x), cos(2^0 x), ..., sin(2^(L-1) x), cos(2^(L-1) x)] (neus_embedder.py:29-36)."""
    if multires <= 0:
        return x
    outs = [x]
    for k in range(multires):
        f = float(2 ** k)
        outs.append(torch.sin(x * f))
        outs.append(torch.cos(x * f))
    return torch.cat(outs, -1)


class Embedder:
    def __init__(self, multires: int, input_dims: int = 3):
        self.multires = multires
        self.input_dims = input_dims
        self.out_dim = embed_dim(multires, input_dims)

    def embed(self, inputs):
        return embed(inputs, self.multires)


def get_embedder(multires, input_dims=3):
    e = Embedder(multires, input_dims)
    return e.embed, e.out_dim
