"""Model / camera configuration for the keypoint-set pose path.

Mirrors the argparse fields the reference's `build_model(args)` reads
(REV/main.py:90-187) and the camera constants of REV/utils/utils.py:30-46.
"""
from __future__ import annotations

import json
import os
from dataclasses import dataclass, asdict

import numpy as np

_DATA = os.path.join(os.path.dirname(__file__), "data")


@dataclass(frozen=True)
class SpeConfig:
    input_size: int = 416          # --input_size (REV/main.py:99)
    num_queries: int = 11          # --num_queries (REV/main.py:137)
    enc_layers: int = 6            # --enc_layers (REV/main.py:122)
    dec_layers: int = 6            # --dec_layers (REV/main.py:124)
    hidden_dim: int = 256          # --hidden_dim (REV/main.py:130)
    nheads: int = 8                # --nheads (REV/main.py:135)
    dim_feedforward: int = 2048    # --dim_feedforward (REV/main.py:127)
    num_classes: int = 11          # REV/models/detr_speed.py:305 (+1 no-object)
    sigma_head: bool = False       # UNC sigma head (UNC/src/zoo/rtdetr/rtdetr_decoder.py:295-297)

    @property
    def feat_size(self) -> int:
        # ResNet-50 stride-8 feature map (REV/models/backbone.py:140-142)
        return self.input_size // 8

    @property
    def tokens(self) -> int:
        return self.feat_size * self.feat_size

    @classmethod
    def from_args(cls, args) -> "SpeConfig":
        """Build from a reference-style argparse.Namespace (REV/main.py:90-187)."""
        return cls(input_size=int(getattr(args, "input_size", 416)),
                   num_queries=int(getattr(args, "num_queries", 11)),
                   enc_layers=int(getattr(args, "enc_layers", 6)),
                   dec_layers=int(getattr(args, "dec_layers", 6)),
                   hidden_dim=int(getattr(args, "hidden_dim", 256)),
                   nheads=int(getattr(args, "nheads", 8)),
                   dim_feedforward=int(getattr(args, "dim_feedforward", 2048)),
                   sigma_head=bool(getattr(args, "sigma_head", False)))

    def to_dict(self):
        return asdict(self)


class Camera:
    """SPEED camera (REV/utils/utils.py:30-46): fx = 0.0176 m / 5.86e-6 m/px."""
    fx = 0.0176
    fy = 0.0176
    nu = 1920
    nv = 1200
    ppx = 5.86e-6
    ppy = ppx
    fpx = fx / ppx
    fpy = fy / ppy
    K = np.array([[fpx, 0, nu / 2], [0, fpy, nv / 2], [0, 0, 1]], dtype=np.float64)
    dist = np.zeros(5)


def world_points() -> np.ndarray:
    """The 11 satellite landmarks (REV/all_result.json 'pt', REV/utils/speed_eval.py:33-39)."""
    with open(os.path.join(_DATA, "world_points.json")) as f:
        return np.asarray(json.load(f)["points"], dtype=np.float64)


def quat_to_matrix(q) -> np.ndarray:
    """Rotation matrix of a (w, x, y, z) quaternion, `mathutils.Quaternion(q).to_matrix()`
    convention (used by REV/utils/utils.py:49-53 to project landmarks)."""
    q = np.asarray(q, dtype=np.float64)
    w, x, y, z = q / np.linalg.norm(q)
    return np.array([
        [1 - 2 * (y * y + z * z), 2 * (x * y - w * z), 2 * (x * z + w * y)],
        [2 * (x * y + w * z), 1 - 2 * (x * x + z * z), 2 * (y * z - w * x)],
        [2 * (x * z - w * y), 2 * (y * z + w * x), 1 - 2 * (x * x + y * y)]])


def project(pts, q, t, K=None) -> np.ndarray:
    """Pinhole projection K [R|t] X (REV/utils/utils.py:56-69)."""
    K = Camera.K if K is None else K
    R = quat_to_matrix(q)
    pc = np.asarray(pts, np.float64) @ R.T + np.asarray(t, np.float64).reshape(1, 3)
    uv = pc @ K.T
    return uv[:, :2] / uv[:, 2:3]
