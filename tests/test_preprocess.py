"""Validation input pipeline (REV/datasets/speed.py:209-233).

CPU: the numpy restatement (oracle/preprocess_ref.py) pinned where a checker exists here --
Pillow's own Image.crop (box rounding, including exact .5 ties) -- plus known-answer properties
of OpenCV's cubic resize that hold whatever its build (dsize == ssize copies, constant images
stay constant, the fixed-point result is the bicubic value within 1 LSB).  cv2 itself is absent,
so bit-parity of the resize against OpenCV is UNPINNED (see the oracle's header).
GPU: csrc/preprocess.hip against the restatement, bit-exact (uint8 crops and therefore the
fp32 normalised images), on synthetic 1920x1200 frames, grayscale and RGB, border-clipped
(non-square) boxes, up- and down-scaling, and the empty-crop status.
"""
import numpy as np
import pytest
import torch
from PIL import Image

import preprocess_ref as pr
from spe.synthetic import synthetic_frames


def test_crop_matches_pillow():
    rng = np.random.Generator(np.random.PCG64(3))
    img = rng.integers(0, 256, (60, 90, 3), dtype=np.uint8)
    pil = Image.fromarray(img)
    boxes = [(10.5, 3.5, 40.5, 33.5), (11.5, 4.5, 41.5, 34.5), (0.0, 0.0, 90.0, 60.0), (2.49, 7.51, 88.5, 59.5)]
    for _ in range(40):
        x = np.sort(rng.uniform(0, 90, 2)) if rng.random() < 0.5 else np.sort(rng.integers(0, 180, 2) / 2.0)
        y = np.sort(rng.uniform(0, 60, 2)) if rng.random() < 0.5 else np.sort(rng.integers(0, 120, 2) / 2.0)
        boxes.append((x[0], y[0], x[1], y[1]))
    for b in boxes:
        ref = np.asarray(pil.crop(np.asarray(b, np.float64)))
        got = pr.pil_crop(img, np.asarray(b, np.float64))
        assert got.shape == ref.shape and (got == ref).all(), b


def test_clip_bbox_val_rule():
    c = pr.generate_clip_bbox_val([100.0, 200.0, 300.0, 250.0], 1920, 1200)
    assert np.allclose(c, [80.0, 105.0, 320.0, 345.0])            # 1.2 x 200 square about (200, 225)
    c = pr.generate_clip_bbox_val([-50.0, 1100.0, 60.0, 1250.0], 1920, 1200)
    assert c[0] == 0.0 and c[3] == 1200.0                         # clipped per coordinate (non-square)


def test_resize_known_answers():
    rng = np.random.Generator(np.random.PCG64(5))
    a = rng.integers(0, 256, (37, 37), dtype=np.uint8)
    assert (pr.resize_cubic_u8(a, 37) == a).all()                 # dsize == ssize: copy
    for v in (0, 1, 77, 254, 255):
        for (h, w, s) in ((50, 70, 416), (900, 640, 416), (33, 33, 640)):
            c = np.full((h, w), v, np.uint8)
            assert (pr.resize_cubic_u8(c, s) == v).all()          # interpolation of a constant
    # the fixed-point pipeline computes separable bicubic (A = -0.75, half-pixel centres,
    # replicated border) to within one LSB of the real-valued result
    b = rng.integers(0, 256, (41, 29), dtype=np.uint8)
    got = pr.resize_cubic_u8(b, 64).astype(np.float64)

    def w(t):
        t = abs(t)
        A = -0.75
        return ((A + 2) * t - (A + 3)) * t * t + 1 if t <= 1 else (((t - 5) * t + 8) * t - 4) * A if t < 2 else 0.0

    def taps(n_src, n_dst):
        M = np.zeros((n_dst, n_src))
        for d in range(n_dst):
            f = (d + 0.5) * n_src / n_dst - 0.5
            s = int(np.floor(f))
            for k in range(-1, 3):
                M[d, min(max(s + k, 0), n_src - 1)] += w(f - (s + k))
        return M
    ref = taps(41, 64) @ b.astype(np.float64) @ taps(29, 64).T
    assert np.abs(got - np.clip(ref, 0, 255)).max() <= 1.0 + 1e-9


@pytest.mark.gpu
@pytest.mark.parametrize("channels,S,B", [(1, 416, 5), (3, 416, 3), (1, 640, 2), (1, 128, 4)])
def test_preprocess_hip_matches_oracle(gpu_device, channels, S, B):
    from spe.datasets import SpeedValTransform
    d = synthetic_frames(B, seed=11 + S + channels, channels=channels)
    bb = d["bbox_xxyy"].copy()
    bb[0] = [1800.0, 1150.0, 1930.0, 1260.0]                      # clipped at the frame corner
    if B > 2:
        bb[1] = [900.0, 500.0, 920.0, 512.0]                      # tiny box: 24 px -> upscaling
        bb[2] = [100.5, 80.5, 1500.5, 1000.5]                     # .5 coordinates, downscaling
    frames = torch.from_numpy(d["frames"]).to(gpu_device)
    o = SpeedValTransform(S)(frames, bb)
    torch.cuda.synchronize()
    ref = pr.preprocess(d["frames"], bb, S)
    assert (o["status"].cpu().numpy() == ref["status"]).all()
    assert np.array_equal(o["clip_bbox"].cpu().numpy(), ref["clip_bbox"].astype(np.float32))
    got = o["images"].cpu().numpy()
    if not np.array_equal(got, ref["images"]):
        # report in uint8 units for a readable failure
        u = np.rint((got * pr.STD[None, :, None, None] + pr.MEAN[None, :, None, None]) * 255)
        r = np.rint((ref["images"] * pr.STD[None, :, None, None] + pr.MEAN[None, :, None, None]) * 255)
        raise AssertionError(f"{int((u != r).sum())} of {u.size} values differ, max {np.abs(u - r).max()} LSB")


@pytest.mark.gpu
def test_preprocess_empty_crop_status(gpu_device):
    from spe.datasets import SpeedValTransform
    frames = torch.zeros(2, 100, 120, dtype=torch.uint8, device=gpu_device)
    bb = np.array([[10.0, 10.0, 50.0, 40.0], [130.0, 110.0, 140.0, 120.0]])   # 2nd entirely off-frame
    o = SpeedValTransform(64)(frames, bb)
    torch.cuda.synchronize()
    ref = pr.preprocess(frames.cpu().numpy(), bb, 64)
    assert o["status"].cpu().tolist() == ref["status"].tolist() == [0, 1]
    assert (o["images"][1] == 0).all()
