"""ORACLE (test infrastructure only — never imported by the product path).

numpy restatement of the reference's validation-path input pipeline:

  REV/datasets/speed.py:209-233   SpeedTrain.__getitem__ (train=False): Image.open().convert('RGB'),
                                  generate_clip_bbox_val, img.crop(bbox_clip), transforms,
                                  F.to_tensor, Normalize
  REV/datasets/speed.py:246-258   generate_clip_bbox_val: 1.2 x max side square about the box
                                  centre, each coordinate clipped to the image (fp64)
  REV/datasets/speed.py:295-299   make_transforms(train=False) = A.Resize(S, S, cv2.INTER_CUBIC)
  REV/datasets/speed.py:25-41     Normalize: F.normalize(mean=(0.485, 0.456, 0.406),
                                  std=(0.229, 0.224, 0.225)) after to_tensor's u8 / 255

Third-party arithmetic restated (absent here, so bit-parity against them is partly unpinned):
  * Pillow Image.crop (Pillow is importable here: tests/test_preprocess.py pins `pil_crop`
    against it): box = map(int, map(round, box)) -- Python round, half to even.
  * OpenCV 4.4 (opencv-python==4.4.0.44, REV/requirements.txt:6) cv::resize INTER_CUBIC on
    8-bit images, generic path (imgproc/src/resize.cpp: resizeGeneric_ with HResizeCubic /
    VResizeCubic and FixedPtCast<int, uchar, 22>): scale = 1 / (dsize / ssize) in double,
    fx = (float)((dx + 0.5) * scale - 0.5), sx = floor(fx), fx -= sx, interpolateCubic(fx)
    with A = -0.75 in float, coefficients rounded to short at scale 2048, taps clamped to the
    image (replicated border), int horizontal then vertical sums, (v + 2^21) >> 22, saturated
    to [0, 255].  UNPINNED: no cv2 here, and OpenCV's x86 SIMD vertical pass evaluates the same
    sum in fp32 with round-half-even, which may differ by 1 at exact ties.
  * The reference's img_trunc(p=0.2) random augmentation in the validation path
    (REV/datasets/speed.py:232) is a defect and is not reproduced.
"""
from __future__ import annotations

import numpy as np

MEAN = np.array([0.485, 0.456, 0.406], np.float32)
STD = np.array([0.229, 0.224, 0.225], np.float32)
COEF_SCALE = 2048          # INTER_RESIZE_COEF_SCALE
CAST_BITS = 22             # 2 * INTER_RESIZE_COEF_BITS


def generate_clip_bbox_val(bbox, width, height):
    """REV/datasets/speed.py:246-258 (fp64)."""
    x1, y1, x2, y2 = (float(v) for v in bbox)
    scale = max(x2 - x1, y2 - y1) * 1.2
    xc, yc = (x1 + x2) / 2, (y1 + y2) / 2
    h = scale / 2
    c = np.asarray([xc - h, yc - h, xc + h, yc + h], np.float64)
    c[0::2] = c[0::2].clip(0, width)
    c[1::2] = c[1::2].clip(0, height)
    return c


def crop_box(clip):
    """Pillow Image.crop's integer box (Image._crop): Python round, half to even."""
    return tuple(int(round(float(v))) for v in clip)


def pil_crop(img, clip):
    """img: uint8 [H, W, C] -> the crop Pillow returns (zero fill outside the image)."""
    x0, y0, x1, y1 = crop_box(clip)
    H, W = img.shape[:2]
    out = np.zeros((max(y1 - y0, 0), max(x1 - x0, 0)) + img.shape[2:], img.dtype)
    sx0, sy0, sx1, sy1 = max(x0, 0), max(y0, 0), min(x1, W), min(y1, H)
    if sx1 > sx0 and sy1 > sy0:
        out[sy0 - y0:sy1 - y0, sx0 - x0:sx1 - x0] = img[sy0:sy1, sx0:sx1]
    return out


def _cubic_coeffs(x):
    """interpolateCubic (OpenCV imgproc/src/resize.cpp), float32, in its operation order."""
    f = np.float32
    A = f(-0.75)
    t = x + f(1)
    c0 = ((A * t - f(5) * A) * t + f(8) * A) * t - f(4) * A
    c1 = ((A + f(2)) * x - (A + f(3))) * x * x + f(1)
    u = f(1) - x
    c2 = ((A + f(2)) * u - (A + f(3))) * u * u + f(1)
    c3 = f(1) - c0 - c1 - c2
    return np.stack([c0, c1, c2, c3], -1)


def _axis(dst, src):
    """Per destination index: first tap and the 4 fixed-point coefficients."""
    scale = 1.0 / (float(dst) / float(src))
    fx = ((np.arange(dst, dtype=np.float64) + 0.5) * scale - 0.5).astype(np.float32)
    sx = np.floor(fx).astype(np.int64)
    fx = (fx - sx.astype(np.float32)).astype(np.float32)
    coef = np.rint(_cubic_coeffs(fx) * np.float32(COEF_SCALE)).astype(np.int64)
    idx = np.clip(sx[:, None] - 1 + np.arange(4)[None, :], 0, src - 1)
    return idx, coef


def resize_cubic_u8(img, size):
    """cv2.resize(img, (size, size), interpolation=cv2.INTER_CUBIC) for uint8 [h, w] or [h, w, C]."""
    h, w = img.shape[:2]
    if (h, w) == (size, size):
        return img.copy()                      # cv::resize copies when dsize == ssize
    xi, xc = _axis(size, w)
    yi, yc = _axis(size, h)
    a = img.astype(np.int64)
    if a.ndim == 2:
        a = a[..., None]
    hs = (a[:, xi, :] * xc[None, :, :, None]).sum(2)              # [h, S, C]
    v = (hs[yi, :, :] * yc[:, :, None, None]).sum(1)              # [S, S, C]
    out = np.clip((v + (1 << (CAST_BITS - 1))) >> CAST_BITS, 0, 255).astype(np.uint8)
    return out if img.ndim == 3 else out[..., 0]


def to_tensor_normalize(u8):
    """F.to_tensor (u8 / 255, CHW) + F.normalize, fp32 in torchvision's operation order."""
    if u8.ndim == 2:
        u8 = np.repeat(u8[..., None], 3, -1)   # Image.convert('RGB') of a grayscale frame
    x = u8.transpose(2, 0, 1).astype(np.float32) / np.float32(255)
    return ((x - MEAN[:, None, None]) / STD[:, None, None]).astype(np.float32)


def preprocess(frames, bboxes, size):
    """frames uint8 [B, H, W] (grayscale, as SPEED ships) or [B, H, W, 3]; bboxes [B, 4]
    detector boxes (x1, y1, x2, y2).  Returns images fp32 [B, 3, S, S], clip_bbox fp64 [B, 4],
    crops (list of the resized uint8 crops) and status [B] (1: empty crop -> zeros)."""
    B, H, W = frames.shape[:3]
    imgs = np.zeros((B, 3, size, size), np.float32)
    clips = np.zeros((B, 4), np.float64)
    status = np.zeros(B, np.int32)
    crops = []
    for i in range(B):
        clips[i] = generate_clip_bbox_val(bboxes[i], W, H)
        c = pil_crop(frames[i], clips[i])
        if c.shape[0] == 0 or c.shape[1] == 0:
            status[i] = 1
            crops.append(None)
            continue
        r = resize_cubic_u8(c, size)
        crops.append(r)
        imgs[i] = to_tensor_normalize(r)
    return {"images": imgs, "clip_bbox": clips, "crops": crops, "status": status}
