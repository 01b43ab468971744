"""spe — MI355X-native keypoint-set inference + PnP pose path (host package).

Mirrors the reference's call surface (build_model / PostProcess / build_solver / SpeedEval /
evaluate) over libspe.so's C ABI (include/spe.h).  Light modules (config, synthetic, misc)
import without the native library; models/solver/speed_eval/engine/pipeline require it.
"""
from .config import SpeConfig, Camera, world_points  # noqa: F401

__all__ = ["SpeConfig", "Camera", "world_points"]
