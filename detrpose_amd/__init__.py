"""MI355X-native DETRPose inference forward (HIP kernels for gfx950 behind a C ABI).

Public API mirrors the reference's src/models module API:
    DETRPose, HGNetv2, HybridEncoder, Transformer, PostProcess, build_model
"""
from .configs import GFLOP_PER_IMAGE, get_config
from .detrpose import DETRPose, build_model
from .hgnetv2 import HGNetv2
from .hybrid_encoder import HybridEncoder
from .postprocesses import PostProcess
from .transformer import Transformer

__all__ = ["DETRPose", "HGNetv2", "HybridEncoder", "Transformer", "PostProcess", "build_model", "get_config",
           "GFLOP_PER_IMAGE"]
