"""Validation input pipeline on the device (REV/datasets/speed.py).

The reference's SpeedTrain(train=False).__getitem__ (REV/datasets/speed.py:209-233) runs per
image in DataLoader worker processes: Image.open().convert('RGB'), generate_clip_bbox_val
(:246-258), img.crop(bbox_clip), A.Resize(S, S, cv2.INTER_CUBIC) (make_transforms(train=False),
:295-299), F.to_tensor and Normalize (:25-41).  `SpeedValTransform` does everything after the
decode for a whole batch of frames already in HBM with one HIP launch (spe_preprocess,
csrc/preprocess.hip) and returns the model input and the clip boxes PostProcess needs.
`JpegDecoder` does the decode before it on the device too (spe_jpeg_decode, csrc/jpeg.hip:
Huffman, dequantisation and libjpeg's islow IDCT, bit-exact with Pillow), so a batch can start
from the JPEG files' bytes in HBM.  The reference's validation-time img_trunc(p=0.2)
augmentation (:232) is a defect and is not reproduced.
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


class JpegDecoder:
    """Image.open(path).convert('RGB') of SpeedTrain.__getitem__ (REV/datasets/speed.py:209-210)
    for a batch of SPEED frames on the device: baseline 8-bit grayscale JPEG files (the dataset's
    format) -> uint8 [B,H,W] frames, the 1-channel input SpeedValTransform replicates to RGB.
    Files are packed into one device byte buffer (pack); status [B]: 0 ok, 1 unsupported coding,
    2 corrupt stream, 3 wrong frame size, 4 file larger than max_bytes (zero frame written)."""

    def __init__(self, height: int = Camera.nv, width: int = Camera.nu, max_bytes: int = 4 << 20):
        self.height, self.width, self.max_bytes = int(height), int(width), int(max_bytes)
        self._ws = {}

    @staticmethod
    def pack(files, device="cuda"):
        """list of JPEG file contents (bytes) -> (data uint8, offsets int64, sizes int64) on device."""
        sizes = np.asarray([len(f) for f in files], np.int64)
        offs = np.zeros(len(files), np.int64)
        if len(files) > 1:
            offs[1:] = np.cumsum(sizes)[:-1]
        buf = np.frombuffer(b"".join(files) + bytes(16), np.uint8)
        dev = torch.device(device)
        return torch.from_numpy(buf.copy()).to(dev), torch.from_numpy(offs).to(dev), torch.from_numpy(sizes).to(dev)

    def workspace(self, B, device):
        key = (torch.device(device).index, B)
        if key not in self._ws:
            n = _lib.lib().spe_jpeg_workspace_bytes(B, self.height, self.width, self.max_bytes)
            self._ws[key] = torch.empty(int(n), dtype=torch.uint8, device=device)
        return self._ws[key]

    def __call__(self, data: torch.Tensor, offsets: torch.Tensor, sizes: torch.Tensor, out=None, stream=None):
        if not (data.is_cuda and data.dtype == torch.uint8):
            raise ValueError("data must be a device uint8 tensor")
        B = offsets.numel()
        dev = data.device
        if out is None:
            out = {"frames": torch.empty(B, self.height, self.width, dtype=torch.uint8, device=dev),
                   "status": torch.empty(B, dtype=torch.int32, device=dev)}
        ws = self.workspace(B, dev)
        _lib.check(_lib.lib().spe_jpeg_decode(_lib.stream_ptr(stream), _lib.ptr(data),
                                              _lib.ptr(offsets.to(torch.int64).contiguous()),
                                              _lib.ptr(sizes.to(torch.int64).contiguous()), B, self.height, self.width,
                                              self.max_bytes, _lib.ptr(out["frames"]), _lib.ptr(out["status"]),
                                              _lib.ptr(ws), ws.numel()), "spe_jpeg_decode")
        return out
