"""Drop-in replacement for the reference's `model` package (model/__init__.py:1-14).

Put `cope-nerf_amd/` on sys.path ahead of the reference checkout and
`from model import NeuSRenderer, SDFNetwork, ..., Trainer, CheckpointIO`
resolves to the HIP-backed classes, so train.py's `mdl.Trainer(...)`,
`mdl.CheckpointIO(...)` and the per-iteration calls (train.py:102, 433-438,
528-532) run against this build.
"""
from copenerf import (CheckpointIO, EdgePreservingSmoothnessLoss, MotionNetwork, NeRF, NeuSRenderer,  # noqa: F401
                      PoseRetriever, RenderingNetwork, SDFNetwork, SingleVarianceNetwork, SmoothnessLoss, Trainer)
