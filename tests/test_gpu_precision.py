"""GPU: the accuracy contract on the bench's own weights (BASELINE north_star "keypoint L2 within 1e-4
of reference").

The bench's pose-consistent weights (bench.py: label-diverse random init with a 64x-sharpened
decoder cross-attention and a point head fitted to random decoder outputs) amplify perturbations of
the decoder output hs ~20x into the keypoints.  This test measures, on the bench's timed batch
(config 2, B = 64), how far apart INDEPENDENT fp32 implementations of the same model land:

  * ours-fp32     the exact-f32 parity mode (this repo; <= 1e-4 of the reference on its goldens)
  * torch-gpu     the oracle's torch restatement (oracle/model_ref.py, pinned to the reference at
                  <= 2e-7 on the goldens) in fp32 on the GPU (hipBLASLt / MIOpen, TF32 off)
  * torch-cpu     the same restatement on the CPU for the first 4 images (the reference's own
                  execution model: REV main.py --eval on CPU, BASELINE config 1)

and where the fast parity modes land against them:

  * fp32x6        the accuracy-contract mode (GEMMs three-way split, attention fp32x3)
  * fp32x3        split-bf16 everywhere

Gates (written here): fp32x6 is within the fp32 implementation spread -- its keypoint distance to
ours-fp32 is at most 2x the distance between the two fp32 implementations ours-fp32 / torch-gpu,
plus 1e-5 -- and within 1e-4 normalised of the torch restatement on the CPU images.
"""
import json
import os
import sys

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _kpt(a, b, fg):
    return float((a - b).abs().amax(-1)[fg].max())


def test_fp32x6_within_fp32_implementation_spread(gpu_device):
    sys.path.insert(0, REPO)
    import argparse
    import bench
    import model_ref
    from spe.config import SpeConfig
    from spe.models import DETR
    from spe.synthetic import bench_weights

    dev = gpu_device
    B = 64
    cfg = SpeConfig(input_size=416, num_queries=11, enc_layers=6, dec_layers=6)

    def hs_fn(w, images):
        m = DETR(cfg, dtype="bf16")
        m.load_state_dict(w)
        n = len(images)
        x = torch.from_numpy(np.concatenate([images] * ((B + n - 1) // n))[:B]).to(dev)
        return m(x, return_hs=True)["hs"].cpu().numpy()[:n]

    w = bench_weights(cfg, 0, hs_fn)
    w, _ = bench.pose_consistent_weights(w, cfg, argparse.Namespace(dtype="bf16", attn_dtype="bf16"), B, 0, 1, dev)
    data = bench.bench_data(cfg, B, 0)
    x = torch.from_numpy(data["images"]).to(dev)

    def ours(dtype):
        m = DETR(cfg, dtype=dtype)
        m.load_state_dict(w)
        o = m(x)
        torch.cuda.synchronize()
        return o["pred_points"].clone(), o["pred_logits"].argmax(-1)

    p32, lab = ours("fp32")
    p6, lab6 = ours("fp32x6")
    p3, lab3 = ours("fp32x3")
    mm, cv = torch.backends.cuda.matmul.allow_tf32, torch.backends.cudnn.allow_tf32
    torch.backends.cuda.matmul.allow_tf32 = torch.backends.cudnn.allow_tf32 = False
    try:
        with torch.no_grad():
            tg = model_ref.forward(x, w, cfg)
            torch.cuda.synchronize()
            ptg, labtg = tg["pred_points"], tg["pred_logits"].argmax(-1)
            tc = model_ref.forward(data["images"][:4], w, cfg)
    finally:
        torch.backends.cuda.matmul.allow_tf32, torch.backends.cudnn.allow_tf32 = mm, cv
    ptc = tc["pred_points"].to(dev)
    fg = (lab < 11) & (lab6 == lab) & (lab3 == lab) & (labtg == lab)
    fg4 = fg[:4] & (tc["pred_logits"].argmax(-1).to(dev) == lab[:4])
    r = {"config": "config 2, B=64, bench pose-consistent weights", "fg_queries": int(fg.sum()),
         "ours_fp32_vs_torch_gpu": _kpt(p32, ptg, fg), "fp32x6_vs_ours_fp32": _kpt(p6, p32, fg),
         "fp32x6_vs_torch_gpu": _kpt(p6, ptg, fg), "fp32x3_vs_ours_fp32": _kpt(p3, p32, fg),
         "fp32x3_vs_torch_gpu": _kpt(p3, ptg, fg),
         "cpu_images": 4, "torch_cpu_vs_ours_fp32": _kpt(ptc, p32[:4], fg4), "torch_cpu_vs_torch_gpu": _kpt(ptc, ptg[:4], fg4),
         "fp32x6_vs_torch_cpu": _kpt(p6[:4], ptc, fg4), "fp32x3_vs_torch_cpu": _kpt(p3[:4], ptc, fg4)}
    out = os.path.join(REPO, "gpurun_out")
    if os.path.isdir(out):
        with open(os.path.join(out, "precision_floor.json"), "w") as f:
            json.dump(r, f, indent=1)
    print(json.dumps(r))
    assert fg.sum() > 300
    assert r["ours_fp32_vs_torch_gpu"] <= 1e-3
    assert r["fp32x6_vs_ours_fp32"] <= 2 * r["ours_fp32_vs_torch_gpu"] + 1e-5, r
    assert r["fp32x6_vs_torch_cpu"] <= 1e-4, r
