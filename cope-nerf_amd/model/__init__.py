"""Drop-in replacement for the reference's `model` package (model/__init__.py:1-14).

Put `cope-nerf_amd/` on sys.path ahead of the reference checkout and
`from model import NeuSRenderer, SDFNetwork, ...` resolves to the HIP-backed
classes.  Names outside the rendering hot path (Trainer, CheckpointIO,
MotionNetwork) are out of scope for this build and are not exported.
"""
from copenerf import (EdgePreservingSmoothnessLoss, NeRF, NeuSRenderer, PoseRetriever,  # noqa: F401
                      RenderingNetwork, SDFNetwork, SingleVarianceNetwork, SmoothnessLoss)
