"""Losses on the hot path.

  SmoothnessLoss / EdgePreservingSmoothnessLoss   model/losses.py:7-38
  rgb L1 + mse, weighted sum, NaN guard           model/training.py:490-549
  eikonal                                         train.py:526
They act on [R,3] / [R/16,4,4] / [M,3] tensors -- a few µs of elementwise work
on the device next to the ~10^2 ms of MLP work -- and stay torch expressions so
train.py's loss code runs unchanged on the HIP renderer's outputs.
"""
from __future__ import annotations

import torch
from torch import nn


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
