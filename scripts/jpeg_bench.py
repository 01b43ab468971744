"""Device JPEG decode throughput on SPEED-sized synthetic frames (spe.datasets.JpegDecoder).

usage: python scripts/jpeg_bench.py [--batch 64] [--quality 90] [--iters 10]
Run under rocprofv3 --kernel-trace --stats for the per-kernel split."""
import argparse
import io
import os
import sys
import time

import numpy as np
import torch
from PIL import Image

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "satellite-pose-estimation_amd"))
from spe.datasets import JpegDecoder  # noqa: E402
from spe.synthetic import synthetic_frames  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--quality", type=int, default=90)
    ap.add_argument("--iters", type=int, default=10)
    a = ap.parse_args()
    d = synthetic_frames(8, seed=3)
    files = []
    for f in d["frames"]:
        b = io.BytesIO()
        Image.fromarray(f).save(b, "JPEG", quality=a.quality)
        files.append(b.getvalue())
    files = [files[i % len(files)] for i in range(a.batch)]
    dev = torch.device("cuda", 0)
    dec = JpegDecoder(max_bytes=max(map(len, files)))
    packed = JpegDecoder.pack(files, dev)
    o = dec(*packed)
    torch.cuda.synchronize()
    assert (o["status"] == 0).all()
    t0 = time.perf_counter()
    for _ in range(a.iters):
        dec(*packed, out=o)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / a.iters
    mb = sum(map(len, files)) / 1e6
    print(f"jpeg decode B={a.batch} q{a.quality}: {dt * 1e3:.3f} ms/batch, {a.batch / dt:.0f} img/s, "
          f"{mb / dt / 1e3:.2f} GB/s of JPEG, {a.batch * 1920 * 1200 / dt / 1e9:.2f} Gpx/s")


if __name__ == "__main__":
    main()
