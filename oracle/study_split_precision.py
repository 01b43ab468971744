"""ORACLE-side precision study (test infrastructure; CPU only): how far does each split-MFMA product
scheme move the keypoints of the bench's fixture weights, with everything else exact fp32?

Every convolution / linear layer of oracle/model_ref.py (the torch-fp32 restatement of the reference
forward) is replaced by an emulation of one MFMA product scheme on the same fp32 operands:

  exact  plain fp32 (the reference)
  bf16x3 x = h + l (bf16 RNE), products h.h + h.l + l.h          (this repo's fp32x3)
  bf16x6 x = h + m + l (bf16 RNE), the six products >= 2^-16     (this repo's fp32x6)
  f16x3  x = (h + l) / s, h, l fp16 RNE of x.s, s a power of two per tensor for activations (from the
         tensor's max |x|) and per output channel for weights: products h.h + h.l + l.h
         (the candidate fp32h3 mode: fp16 MFMAs run at the bf16 rate, half of bf16x6's products)

The products of fp16 / bf16 values are exact in fp32, the sums accumulate in fp32 as the MFMAs do.
Attention stays exact here (its split error is insensitive on these weights).

    python oracle/study_split_precision.py [--images 8]
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch
import torch.nn.functional as F

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "satellite-pose-estimation_amd"))

import model_ref  # noqa: E402
from spe.config import SpeConfig  # noqa: E402
from spe.synthetic import bench_images, fixed_bench_weights  # noqa: E402

_conv, _linear = F.conv2d, F.linear


def pow2_scale(amax, target=2.0 ** 13):
    """2^k with amax * 2^k in [target/2, target) (1 for amax == 0)."""
    a = torch.as_tensor(amax, dtype=torch.float64)
    k = torch.where(a > 0, torch.floor(torch.log2(target / torch.clamp(a, min=1e-300))), torch.zeros_like(a))
    return torch.pow(2.0, k).float()


def split(x, scheme, per_channel=False):
    """-> list of (plane, scale) whose sum / scale is x's representation."""
    if scheme == "bf16x3" or scheme == "bf16x6":
        h = x.bfloat16().float()
        r = x - h
        m = r.bfloat16().float()
        if scheme == "bf16x3":
            return [h, m], 1.0
        l_ = (r - m).bfloat16().float()
        return [h, m, l_], 1.0
    if per_channel:
        amax = x.abs().reshape(x.shape[0], -1).amax(1)
        s = pow2_scale(amax).reshape((-1,) + (1,) * (x.dim() - 1))
    else:
        s = pow2_scale(x.abs().max())
    xs = x * s
    h = xs.half().float()
    l_ = (xs - h).half().float()
    return [h, l_], s


PRODUCTS = {"bf16x3": [(1, 0), (0, 1), (0, 0)], "f16x3": [(1, 0), (0, 1), (0, 0)],     # small terms first
            "bf16x6": [(2, 0), (0, 2), (1, 1), (1, 0), (0, 1), (0, 0)]}


def emulate(op, x, w, scheme, **kw):
    xa, sa = split(x, scheme)
    wb, sb = split(w, scheme, per_channel=True)
    acc = None
    for i, j in PRODUCTS[scheme]:                     # small terms first, as the kernels do
        y = op(xa[i], wb[j], None, **kw)
        acc = y if acc is None else acc + y
    if scheme == "f16x3":
        # acc / (s_a * s_b[n]) -- powers of two, exact
        sbn = sb.reshape(-1)
        shape = (1, -1, 1, 1) if op is _conv else (1,) * (acc.dim() - 1) + (-1,)
        acc = acc / (sa * sbn.reshape(shape))
    return acc


def install(scheme):
    if scheme == "exact":
        F.conv2d, F.linear = _conv, _linear
        return

    def conv(x, w, b=None, stride=1, padding=0, dilation=1, groups=1):
        y = emulate(_conv, x, w, scheme, stride=stride, padding=padding)
        return y if b is None else y + b[None, :, None, None]

    def linear(x, w, b=None):
        y = emulate(_linear, x, w, scheme)
        return y if b is None else y + b
    F.conv2d, F.linear = conv, linear


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--images", type=int, default=8)
    p.add_argument("--schemes", default="bf16x3,bf16x6,f16x3")
    a = p.parse_args()
    torch.set_num_threads(os.cpu_count() or 8)
    cfg = SpeConfig(input_size=416, num_queries=11, enc_layers=6, dec_layers=6)
    w, _ = fixed_bench_weights(cfg, 0)
    data = bench_images(cfg, 0, a.images)
    res = {}
    with torch.no_grad():
        install("exact")
        ref = model_ref.forward(data["images"], w, cfg)
        lab = ref["pred_logits"].argmax(-1)
        fg = lab < 11
        for sch in a.schemes.split(","):
            t0 = time.time()
            install(sch)
            o = model_ref.forward(data["images"], w, cfg)
            install("exact")
            same = fg & (o["pred_logits"].argmax(-1) == lab)
            dk = (o["pred_points"] - ref["pred_points"]).abs().amax(-1)[same]
            dh = ((o["hs"][-1] - ref["hs"][-1]).norm(dim=-1) / ref["hs"][-1].norm(dim=-1))
            res[sch] = {"kpt_norm_max": float(dk.max()), "kpt_norm_mean": float(dk.mean()),
                        "hs_rel_max": float(dh.max()), "label_agreement": float((o["pred_logits"].argmax(-1) == lab).float().mean()),
                        "seconds": round(time.time() - t0, 1)}
            print(sch, json.dumps(res[sch]), flush=True)
    print(json.dumps({"images": a.images, "weights": "bench fixture", "vs": "exact fp32 restatement", **res}))


if __name__ == "__main__":
    main()
