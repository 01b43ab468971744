"""Validation input pipeline on the device (REV/datasets/speed.py).

The reference's SpeedTrain(train=False).__getitem__ (REV/datasets/speed.py:209-233) runs per
image in DataLoader worker processes: Image.open().convert('RGB'), generate_clip_bbox_val
(:246-258), img.crop(bbox_clip), A.Resize(S, S, cv2.INTER_CUBIC) (make_transforms(train=False),
:295-299), F.to_tensor and Normalize (:25-41).  `SpeedValTransform` does everything after the
decode for a whole batch of frames already in HBM with one HIP launch (spe_preprocess,
csrc/preprocess.hip) and returns the model input and the clip boxes PostProcess needs.
JPEG decode stays on the host (no rocJPEG in this image); the reference's validation-time
img_trunc(p=0.2) augmentation (:232) is a defect and is not reproduced.
"""
from __future__ import annotations

import numpy as np
import torch

from . import _lib
from .config import Camera

IMAGENET_MEAN = (0.485, 0.456, 0.406)      # REV/datasets/speed.py:196-197 (Normalize args)
IMAGENET_STD = (0.229, 0.224, 0.225)


def generate_clip_bbox_val(bbox, image_size=(Camera.nu, Camera.nv)):
    """REV/datasets/speed.py:246-258 on the host (fp64): 1.2 x max-side square about the box
    centre, each coordinate clipped to the image.  image_size = (width, height)."""
    x1, y1, x2, y2 = (float(v) for v in bbox)
    scale = max(x2 - x1, y2 - y1) * 1.2
    xc, yc, h = (x1 + x2) / 2, (y1 + y2) / 2, scale / 2
    c = np.asarray([xc - h, yc - h, xc + h, yc + h], dtype=np.float64)
    c[0::2] = c[0::2].clip(0, image_size[0])
    c[1::2] = c[1::2].clip(0, image_size[1])
    return c


class SpeedValTransform:
    """frames (device uint8 [B,H,W] grayscale or [B,H,W,3]) + detector boxes [B,4] (x1,y1,x2,y2)
    -> images fp32 [B,3,S,S] (ImageNet-normalised, the model input), clip_bbox fp32 [B,4],
    status int32 [B] (1 = empty crop: the reference would raise; zeros are written)."""

    def __init__(self, size: int = 416):
        self.size = int(size)

    def __call__(self, frames: torch.Tensor, bbox_xxyy, out=None, stream=None):
        if frames.dtype != torch.uint8 or frames.dim() not in (3, 4) or not frames.is_cuda:
            raise ValueError("frames must be a device uint8 tensor [B,H,W] or [B,H,W,3]")
        frames = frames.contiguous()
        B, H, W = frames.shape[:3]
        C = 1 if frames.dim() == 3 else frames.shape[3]
        dev = frames.device
        bb = torch.as_tensor(bbox_xxyy, dtype=torch.float64).to(dev).contiguous().view(B, 4)
        S = self.size
        if out is None:
            out = {"images": torch.empty(B, 3, S, S, device=dev),
                   "clip_bbox": torch.empty(B, 4, device=dev),
                   "status": torch.empty(B, dtype=torch.int32, device=dev)}
        _lib.check(_lib.lib().spe_preprocess(_lib.stream_ptr(stream), _lib.ptr(frames), B, H, W, C, _lib.ptr(bb), S,
                                             _lib.ptr(out["images"]), _lib.ptr(out["clip_bbox"]),
                                             _lib.ptr(out["status"])), "spe_preprocess")
        return out
