"""Drop-in replacement for the reference's `model` package (model/__init__.py:1-14).

Put `cope-nerf_amd/` on sys.path ahead of the reference checkout and
`from model import NeuSRenderer, SDFNetwork, ...` resolves to the HIP-backed
classes.  Trainer and CheckpointIO (outside the rendering hot path) are not
exported; MotionNetwork is the stage-1 motion model of copenerf/motion.py.
"""
from copenerf import (EdgePreservingSmoothnessLoss, MotionNetwork, NeRF, NeuSRenderer,  # noqa: F401
                      PoseRetriever, RenderingNetwork, SDFNetwork, SingleVarianceNetwork, SmoothnessLoss)
