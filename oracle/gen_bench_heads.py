"""ORACLE-side fixture generator (test infrastructure; run once in the build container, CPU only).

Writes satellite-pose-estimation_amd/spe/data/bench_heads_s{S}_q{Q}_l{E}-{D}_seed{s}.npz: the class
head and the fitted point head of the bench's pose-consistent weights (spe.synthetic
.fixed_bench_weights), computed from the decoder outputs hs of the torch-fp32 CPU restatement of
the reference model (oracle/model_ref.py, <= 2e-7 of the reference on its goldens):

  1. w = sharpen_decoder(random_weights(cfg, seed))               (spe.synthetic)
  2. class head drawn in the principal subspace of hs on the 16-image calibration batch
     (diversify_class_head, the same rule the bench used in rounds 1-4)
  3. point head fitted (fit_point_head, CPU torch, fixed seeds) on the whole bench pool
     (spe.synthetic.BENCH_POOL = 256 images, the north-star global batch): each foreground query's
     target is its label's landmark projection + N(0, 2 px), 10 % uniform outliers (keypoint_targets)

Nothing here depends on a kernel of this repository, on a GPU or on a rank count, so every bench
run -- any tree, 1 or 8 GPUs, any dtype -- times the same weights.
The file holds plain float32 arrays and a JSON string (np.load without pickles).

    python oracle/gen_bench_heads.py [--size 416 --queries 11 --layers 6]
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(REPO, "satellite-pose-estimation_amd"))

import model_ref  # noqa: E402
from spe.config import SpeConfig  # noqa: E402
from spe import synthetic as syn  # noqa: E402


def hs_cpu(w, images, cfg, chunk=8):
    out = []
    with torch.no_grad():
        for i in range(0, len(images), chunk):
            out.append(model_ref.forward(images[i:i + chunk], w, cfg)["hs"][-1].numpy())
    return np.concatenate(out)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--size", type=int, default=416)
    p.add_argument("--queries", type=int, default=11)
    p.add_argument("--layers", type=int, default=6)
    p.add_argument("--seed", type=int, default=0)
    p.add_argument("--steps", type=int, default=10000)
    p.add_argument("--cache", default=None, help="npz caching the pool's hs and the class head between runs")
    a = p.parse_args()
    torch.set_num_threads(os.cpu_count() or 8)
    cfg = SpeConfig(input_size=a.size, num_queries=a.queries, enc_layers=a.layers, dec_layers=a.layers)
    t0 = time.time()
    pool = syn.bench_images(cfg, 0, syn.BENCH_POOL)
    cache = a.cache and os.path.exists(a.cache) and np.load(a.cache)
    if cache:                       # hs of an earlier run of this script (same config and seeds)
        w = syn.sharpen_decoder(syn.random_weights(cfg, a.seed), cfg)
        w["cls_embed.weight"], w["cls_embed.bias"] = cache["cls_w"], cache["cls_b"]
        hs = cache["hs"]
    else:
        w = syn.bench_weights(cfg, a.seed, lambda ww, im: hs_cpu(ww, im, cfg))
        hs = hs_cpu(w, pool["images"], cfg)
        if a.cache:
            np.savez(a.cache, hs=hs, cls_w=w["cls_embed.weight"], cls_b=w["cls_embed.bias"])
    print(f"hs of {len(hs)} pool images in {time.time() - t0:.0f}s", flush=True)
    logits = hs.astype(np.float64) @ w["cls_embed.weight"].T.astype(np.float64) + w["cls_embed.bias"]
    labels = logits.argmax(-1)
    tgt, mask = syn.keypoint_targets(pool, labels, seed=7)
    w, err = syn.fit_point_head(w, hs, tgt, mask, steps=a.steps, device="cpu")
    meta = {"generator": "oracle/gen_bench_heads.py (torch-fp32 CPU restatement oracle/model_ref.py)",
            "config": {"input_size": a.size, "num_queries": a.queries, "enc_layers": a.layers,
                       "dec_layers": a.layers}, "weight_seed": a.seed, "sharpen": 64.0,
            "calib_seed": syn.CALIB_SEED, "pool": syn.BENCH_POOL, "pool_seed": syn.BENCH_SEED,
            "targets": "keypoint_targets(seed=7, noise 2 px, 10% outliers)", "fit_steps": a.steps,
            "fg_queries": int(mask.sum()), "fit_err_max_norm": float(err.max()),
            "fit_err_mean_norm": float(err.mean()),
            "labels_per_image_mean": float(np.mean([len(set(l[l < 11])) for l in labels]))}
    path = syn.heads_fixture_path(cfg, a.seed)
    np.savez(path, meta=np.array(json.dumps(meta)), **{k: w[k].astype(np.float32) for k in syn.HEADS_KEYS})
    print(json.dumps(meta))
    print(f"wrote {path} in {time.time() - t0:.0f}s")


if __name__ == "__main__":
    main()
