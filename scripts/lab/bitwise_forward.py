"""GPU: dump the fp32h3 model's outputs on the bench weights / images of configs 2 (= 3), 4 and 5, or
compare two such dumps bit for bit.  Used to show that a kernel change which keeps every product and
its accumulation order (a different DMA pipeline, a different launch form) leaves the accuracy-
contract mode's results -- and so every validated bench line -- unchanged.

  python scripts/lab/bitwise_forward.py dump gpurun_out/a.npz      (SPE_LIB_PATH selects the library)
  python scripts/lab/bitwise_forward.py compare gpurun_out/a.npz gpurun_out/b.npz
"""
import argparse
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
CASES = {2: dict(size=416, queries=11, sigma=False, images=64),
         4: dict(size=416, queries=11, sigma=True, images=64),
         5: dict(size=640, queries=40, sigma=False, images=32)}


def dump(path):
    import torch
    sys.path.insert(0, REPO)
    sys.path.insert(0, os.path.join(REPO, "satellite-pose-estimation_amd"))
    import bench
    from spe.config import SpeConfig
    from spe.models import DETR
    from spe.synthetic import bench_images
    dev = torch.device("cuda:0")
    out = {}
    for c, cc in CASES.items():
        cfg = SpeConfig(input_size=cc["size"], num_queries=cc["queries"], enc_layers=6, dec_layers=6,
                        sigma_head=cc["sigma"])
        w, _, _ = bench.bench_weights_for(argparse.Namespace(weights="pose-consistent"), cfg, None, 0, 1, dev)
        data = bench_images(cfg, 0, cc["images"])
        x = torch.from_numpy(data["images"]).to(dev)
        clip = torch.from_numpy(data["clip_bbox"]).float().to(dev)
        m = DETR(cfg, dtype="fp32h3")
        m.load_state_dict(w)
        o = m(x, clip_bbox=clip)
        torch.cuda.synchronize()
        for k, v in o.items():
            if torch.is_tensor(v):
                out[f"c{c}.{k}"] = v.detach().float().cpu().numpy()
        print(f"config {c}: {sorted(k for k, v in o.items() if torch.is_tensor(v))}", flush=True)
        del m, o
    np.savez(path, **out)


def compare(a, b):
    A, B = np.load(a), np.load(b)
    same = True
    for k in sorted(A.files):
        x, y = A[k], B[k]
        eq = x.shape == y.shape and np.array_equal(x.view(np.uint32), y.view(np.uint32))
        d = float(np.abs(x - y).max()) if x.shape == y.shape and x.size else float("nan")
        print(f"{k:28s} {'identical' if eq else 'DIFFERS'}  max|d| {d:.3e}")
        same &= eq
    print("ALL BIT-IDENTICAL" if same else "OUTPUTS DIFFER")
    return 0 if same else 1


if __name__ == "__main__":
    if sys.argv[1] == "dump":
        dump(sys.argv[2])
    else:
        sys.exit(compare(sys.argv[2], sys.argv[3]))
