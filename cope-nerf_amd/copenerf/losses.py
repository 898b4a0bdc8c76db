"""Losses on the hot path.

  SmoothnessLoss / EdgePreservingSmoothnessLoss   model/losses.py:7-38
  rgb L1 + mse, weighted sum, NaN guard           model/training.py:490-549
  eikonal                                         train.py:526
The classes and functions below are the reference's own torch expressions, so
train.py's loss code runs unchanged on the HIP renderer's outputs.  Those
expressions launch ~150 small kernels per step (forward + autograd);
`train_losses` computes the same weighted sum and its input gradients with one
HIP call (cn_train_loss: three launches) and is what the training step uses.
"""
from __future__ import annotations

import torch
from torch import nn

from . import ops


def _l1mean(x):
    return torch.mean(torch.abs(x))


class SmoothnessLoss(nn.Module):
    def __init__(self, patch_size):
        super().__init__()
        self.patch_size = patch_size

    def forward(self, d):
        return (_l1mean(d[:, :, :-1] - d[:, :, 1:]) + _l1mean(d[:, :-1, :] - d[:, 1:, :]) +
                _l1mean(d[:, :-1, :-1] - d[:, 1:, 1:]) + _l1mean(d[:, 1:, :-1] - d[:, :-1, 1:])) / 4


class EdgePreservingSmoothnessLoss(nn.Module):
    def __init__(self, patch_size, bilateral_gamma=0.1):
        super().__init__()
        self.patch_size = patch_size
        self.gamma = bilateral_gamma

    def _bw(self, x):
        return torch.exp(-torch.abs(x).sum(-1) / self.gamma).unsqueeze(-1)

    def forward(self, d, img):
        pairs = (((slice(None), slice(None), slice(None, -1)), (slice(None), slice(None), slice(1, None))),
                 ((slice(None), slice(None, -1), slice(None)), (slice(None), slice(1, None), slice(None))),
                 ((slice(None), slice(None, -1), slice(None, -1)), (slice(None), slice(1, None), slice(1, None))),
                 ((slice(None), slice(1, None), slice(None, -1)), (slice(None), slice(None, -1), slice(1, None))))
        tot = 0.0
        for a, b in pairs:
            tot = tot + _l1mean(self._bw(img[a] - img[b]) * (d[a] - d[b]))
        return tot / 4


def eikonal_loss(normals):
    return torch.mean((torch.linalg.norm(normals.reshape(-1, 3), ord=2, dim=-1) - 1.0) ** 2)


def rgb_l1(rgb, gt):
    return torch.sum(torch.abs(rgb - gt)) / float(rgb.shape[0])


class _TrainLossFn(torch.autograd.Function):
    """(color, gt, depth, normals) -> weighted loss; the input gradients come out of
    the same cn_train_loss call and are scaled by the upstream gradient."""

    @staticmethod
    def forward(ctx, color, gt, depth, normals, weights, patch, gamma, nonfinite):
        shape = normals.shape
        loss, dc, dd, dn = ops.train_loss(color.contiguous(), gt.contiguous(), depth.contiguous(),
                                          normals.reshape(-1, 3), weights=weights, patch=patch, gamma=gamma,
                                          nonfinite=nonfinite)
        ctx.save_for_backward(dc, dd.view(depth.shape), dn.view(shape))
        return loss

    @staticmethod
    def backward(ctx, g):
        dc, dd, dn = ctx.saved_tensors
        dc, dd, dn = torch._foreach_mul([dc, dd, dn], g)
        return dc, None, dd, dn, None, None, None, None


def loss_weight_vector(w_rgb=1.0, w_eik=0.1, w_edge=1.0, w_smooth=1e-4, device=None):
    """The device weight vector cn_train_loss reads: (w_rgb, w_eik, w_edge, w_smooth)."""
    return torch.tensor([w_rgb, w_eik, w_edge, w_smooth], dtype=torch.float32, device=device)


def train_losses(color, gt, depth, normals, *, w_rgb=1.0, w_eik=0.1, w_edge=1.0, w_smooth=1e-4, patch=4,
                 gamma=0.1, weights=None, nonfinite=None):
    """w_rgb rgb_l1 + w_eik eikonal + w_edge EdgePreservingSmoothnessLoss + w_smooth
    SmoothnessLoss on patch x patch ray patches, on the device in one call
    (color [R,3], gt [R,3], depth [R,1], normals [..., 3] sample normals).
    weights: optional device [4] tensor replacing the floats (updated in place by a
    schedule, read by the kernels at run time: graph-replay safe); nonfinite: optional
    device int32 [1] sticky flag, the device form of model/training.py:532-533's
    `assert not torch.isnan(loss)`."""
    if weights is None:
        weights = torch.tensor([w_rgb, w_eik, w_edge, w_smooth], dtype=torch.float32).to(color.device,
                                                                                         non_blocking=True)
    return _TrainLossFn.apply(color, gt, depth, normals, weights, int(patch), float(gamma), nonfinite)
