"""copenerf — MI355X-native (gfx950) kernels for cope-nerf's NeuS rendering hot path.

Drop-in host API mirroring the reference's `model` package (model/__init__.py:1-14):
NeuSRenderer, SDFNetwork, RenderingNetwork, SingleVarianceNetwork, NeRF,
MotionNetwork, PoseRetriever, Trainer, CheckpointIO and the smoothness losses.
The compute runs in libcopenerf.so (include/copenerf.h); there is no CPU path.
"""
from .fields import NeRF, RenderingNetwork, SDFNetwork, SingleVarianceNetwork  # noqa: F401
from .renderer import NeuSRenderer  # noqa: F401
from .losses import EdgePreservingSmoothnessLoss, SmoothnessLoss  # noqa: F401
from .rays import PoseRetriever  # noqa: F401
from .motion import MotionNetwork  # noqa: F401
from .trainer import Trainer  # noqa: F401
from .checkpoints import CheckpointIO  # noqa: F401
from . import _lib  # noqa: F401

__all__ = ["NeuSRenderer", "SDFNetwork", "RenderingNetwork", "SingleVarianceNetwork", "NeRF",
           "EdgePreservingSmoothnessLoss", "SmoothnessLoss", "PoseRetriever", "MotionNetwork", "Trainer",
           "CheckpointIO"]
