"""On-device baseline-JPEG decode (csrc/jpeg.hip) against Pillow itself -- the
decoder the reference calls (Image.open(path).convert('RGB'), REV/datasets/speed.py:209-210).

Bit-exact: every decoded pixel equals Pillow's (libjpeg-turbo, islow IDCT) on files Pillow
encodes: SPEED-sized synthetic frames at several qualities, optimised Huffman tables, restart
markers every block / every two rows, sizes that are not multiples of 8, a batch mixing them.
Unsupported codings (progressive, colour) and a wrong frame size give a status and a zero frame.
"""
import io

import numpy as np
import pytest
import torch
from PIL import Image

from spe import _lib


def _encode(a, **kw):
    b = io.BytesIO()
    Image.fromarray(a).save(b, "JPEG", **kw)
    return b.getvalue()


def _pillow(data):
    return np.asarray(Image.open(io.BytesIO(data)).convert("L"))


def _frames(n, h, w, seed):
    from spe.synthetic import synthetic_frames
    if (h, w) == (1200, 1920):
        return synthetic_frames(n, seed=seed)["frames"]
    rng = np.random.default_rng(seed)
    yy, xx = np.mgrid[0:h, 0:w]
    out = []
    for _ in range(n):
        g = 60 + 40 * np.sin(xx / rng.uniform(3, 20)) * np.cos(yy / rng.uniform(3, 20)) + rng.normal(0, 12, (h, w))
        out.append(np.clip(np.round(g), 0, 255).astype(np.uint8))
    return np.stack(out)


def test_jpeg_workspace_plan():
    L = _lib.lib()
    a = L.spe_jpeg_workspace_bytes(4, 1200, 1920, 1 << 20)
    b = L.spe_jpeg_workspace_bytes(8, 1200, 1920, 1 << 20)
    assert 0 < a < b
    assert L.spe_jpeg_workspace_bytes(4, 0, 1920, 1 << 20) == -1


CASES = [
    ("q75", 1200, 1920, dict(quality=75)),
    ("q95", 1200, 1920, dict(quality=95)),
    ("q30_opt", 1200, 1920, dict(quality=30, optimize=True)),
    ("rst_blocks", 1200, 1920, dict(quality=75, restart_marker_blocks=1)),
    ("rst_rows", 1200, 1920, dict(quality=85, restart_marker_rows=2)),
    ("odd", 37, 53, dict(quality=90)),
    ("odd_rst", 101, 67, dict(quality=60, restart_marker_blocks=7)),
]


@pytest.mark.gpu
@pytest.mark.parametrize("tag,h,w,kw", CASES, ids=[c[0] for c in CASES])
def test_jpeg_decode_matches_pillow(gpu_device, tag, h, w, kw):
    from spe.datasets import JpegDecoder
    fr = _frames(3, h, w, seed=len(tag) * 7 + h)
    files = [_encode(f, **kw) for f in fr]
    dec = JpegDecoder(h, w, max_bytes=max(len(f) for f in files))
    o = dec(*JpegDecoder.pack(files, gpu_device))
    torch.cuda.synchronize()
    np.testing.assert_array_equal(o["status"].cpu().numpy(), 0)
    got = o["frames"].cpu().numpy()
    for i, f in enumerate(files):
        ref = _pillow(f)
        assert np.array_equal(got[i], ref), (tag, i, int((got[i] != ref).sum()))


@pytest.mark.gpu
def test_jpeg_batch_mixed_and_unsupported(gpu_device):
    """One batch: good files of different encodings next to a progressive file, an RGB file and
    a file of another size; the good ones decode exactly, the others get their status and a
    zero frame, and nothing spills into the neighbours."""
    from spe.datasets import JpegDecoder
    h, w = 96, 128
    fr = _frames(6, h, w, seed=3)
    rgb = np.repeat(fr[3][..., None], 3, -1)
    files = [_encode(fr[0], quality=75), _encode(fr[1], quality=75, progressive=True),
             _encode(rgb, quality=75), _encode(fr[4][:64, :64].copy(), quality=75),
             _encode(fr[5], quality=92, optimize=True), _encode(fr[2], quality=50, restart_marker_blocks=3)]
    dec = JpegDecoder(h, w, max_bytes=max(len(f) for f in files))
    o = dec(*JpegDecoder.pack(files, gpu_device))
    torch.cuda.synchronize()
    st = o["status"].cpu().numpy()
    got = o["frames"].cpu().numpy()
    np.testing.assert_array_equal(st, [0, 1, 1, 3, 0, 0])
    for i in (0, 4, 5):
        np.testing.assert_array_equal(got[i], _pillow(files[i]))
    for i in (1, 2, 3):
        assert (got[i] == 0).all()


def _truncated_files(fr):
    """A file cut at 60 % (no EOI: Pillow raises "image file is truncated"), the same cut with an EOI
    appended, and a file whose third restart interval lost two thirds of its bytes."""
    f = _encode(fr[0], quality=75)
    cut = f[:int(len(f) * 0.6)]
    g = _encode(fr[1], quality=75, restart_marker_blocks=4)
    rst = [i for i in range(len(g) - 1) if g[i] == 0xFF and 0xD0 <= g[i + 1] <= 0xD7]
    p2, p3 = rst[2], rst[3]
    short = g[:p2 + 2] + g[p2 + 2:p2 + 2 + (p3 - p2 - 2) // 3] + g[p3:]
    return [cut, cut + b"\xff\xd9", short]


@pytest.mark.gpu
def test_jpeg_truncated_streams_are_corrupt(gpu_device):
    """Entropy-coded data that ends before the frame's blocks are complete is status 2 (corrupt) with
    a zero frame -- never a frame holding an earlier image's coefficients (the coefficient buffer is
    reused uncleared).  The neighbours in the batch decode exactly.  Pillow raises on the cut file
    without EOI (checked here); with an EOI, or with a short restart interval, libjpeg instead warns
    and paints the rest of the segment gray -- that recovery is not reproduced (status 2)."""
    from spe.datasets import JpegDecoder
    h, w = 96, 128
    fr = _frames(4, h, w, seed=11)
    bad = _truncated_files(fr)
    with pytest.raises(OSError):
        Image.open(io.BytesIO(bad[0])).load()
    good = [_encode(fr[2], quality=80), _encode(fr[3], quality=60, restart_marker_blocks=4)]
    dec = JpegDecoder(h, w, max_bytes=max(len(f) for f in good + bad))
    # decode the good files first so the workspace holds coefficients of real images
    dec(*JpegDecoder.pack(good + good[:1], gpu_device))
    files = [good[0], bad[0], bad[1], good[1], bad[2]]
    o = dec(*JpegDecoder.pack(files, gpu_device))
    torch.cuda.synchronize()
    st = o["status"].cpu().numpy()
    got = o["frames"].cpu().numpy()
    np.testing.assert_array_equal(st, [0, 2, 2, 0, 2])
    np.testing.assert_array_equal(got[0], _pillow(good[0]))
    np.testing.assert_array_equal(got[3], _pillow(good[1]))
    for i in (1, 2, 4):
        assert (got[i] == 0).all()


@pytest.mark.gpu
def test_jpeg_to_model_input_matches_pillow_path(gpu_device):
    """Decode -> spe_preprocess on the device equals Pillow's decode -> the same preprocess on
    Pillow's frames (the whole SpeedTrain.__getitem__ validation path from JPEG bytes)."""
    from spe.datasets import JpegDecoder, SpeedValTransform
    from spe.synthetic import synthetic_frames
    d = synthetic_frames(4, seed=12)
    files = [_encode(f, quality=80) for f in d["frames"]]
    dec = JpegDecoder(max_bytes=max(len(f) for f in files))
    o = dec(*JpegDecoder.pack(files, gpu_device))
    ref = torch.from_numpy(np.stack([_pillow(f) for f in files])).to(gpu_device)
    t = SpeedValTransform(416)
    bb = torch.from_numpy(d["bbox_xxyy"]).to(gpu_device)
    a = t(o["frames"], bb)
    b = t(ref, bb)
    torch.cuda.synchronize()
    assert torch.equal(a["images"], b["images"]) and torch.equal(a["clip_bbox"], b["clip_bbox"])
