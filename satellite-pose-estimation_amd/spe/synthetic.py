"""Seeded synthetic inputs for the keypoint-set pose path.

* `param_shapes(cfg)`  - the reference's state_dict key space (412 keys for the REV
  DETR, REV/models/detr_speed.py:32-56, backbone.py:105-131, transformer.py:18-49),
  plus the optional UNC-style sigma head.
* `random_weights(cfg, seed)` - deterministic random-init weights in that key space
  (there is no trained checkpoint in the reference tree), with non-trivial FrozenBN
  statistics so the BN folding path is exercised.
* `synthetic_frames(B, seed)` - full 1920x1200 8-bit frames + detector boxes, the input of
  the on-device validation transform (spe.datasets.SpeedValTransform).
* `synthetic_batch(cfg, B, seed)` - SPEED-shaped crops: GT pose, projected landmarks,
  val-rule clip box (REV/datasets/speed.py:246-260), rendered crop, ImageNet
  normalisation (REV/datasets/speed.py:25-41).
Everything is numpy PCG64 so that the same seed yields the same bytes on every box.
"""
from __future__ import annotations

import numpy as np

from .config import SpeConfig, Camera, world_points, project

IMAGENET_MEAN = np.array([0.485, 0.456, 0.406], np.float32)
IMAGENET_STD = np.array([0.229, 0.224, 0.225], np.float32)

_RESNET50_STAGES = [(64, 3, 1), (128, 4, 2), (256, 6, 2)]   # layer1..3 (layer4 never runs)


def _bn_keys(prefix, c):
    return [(f"{prefix}.{n}", (c,)) for n in ("weight", "bias", "running_mean", "running_var")]


def param_shapes(cfg: SpeConfig):
    """Ordered list of (key, shape) in the reference's state_dict naming."""
    d, ff, Q = cfg.hidden_dim, cfg.dim_feedforward, cfg.num_queries
    out = []
    for i in range(cfg.enc_layers):
        p = f"transformer.encoder.layers.{i}"
        out += [(f"{p}.self_attn.in_proj_weight", (3 * d, d)), (f"{p}.self_attn.in_proj_bias", (3 * d,)),
                (f"{p}.self_attn.out_proj.weight", (d, d)), (f"{p}.self_attn.out_proj.bias", (d,)),
                (f"{p}.linear1.weight", (ff, d)), (f"{p}.linear1.bias", (ff,)),
                (f"{p}.linear2.weight", (d, ff)), (f"{p}.linear2.bias", (d,)),
                (f"{p}.norm1.weight", (d,)), (f"{p}.norm1.bias", (d,)),
                (f"{p}.norm2.weight", (d,)), (f"{p}.norm2.bias", (d,))]
    for i in range(cfg.dec_layers):
        p = f"transformer.decoder.layers.{i}"
        for a in ("self_attn", "multihead_attn"):
            out += [(f"{p}.{a}.in_proj_weight", (3 * d, d)), (f"{p}.{a}.in_proj_bias", (3 * d,)),
                    (f"{p}.{a}.out_proj.weight", (d, d)), (f"{p}.{a}.out_proj.bias", (d,))]
        out += [(f"{p}.linear1.weight", (ff, d)), (f"{p}.linear1.bias", (ff,)),
                (f"{p}.linear2.weight", (d, ff)), (f"{p}.linear2.bias", (d,))]
        for n in ("norm1", "norm2", "norm3"):
            out += [(f"{p}.{n}.weight", (d,)), (f"{p}.{n}.bias", (d,))]
    out += [("transformer.decoder.norm.weight", (d,)), ("transformer.decoder.norm.bias", (d,)),
            ("cls_embed.weight", (cfg.num_classes + 1, d)), ("cls_embed.bias", (cfg.num_classes + 1,))]
    for j, (o, i) in enumerate([(d, d), (d, d), (2, d)]):
        out += [(f"point_embed.layers.{j}.weight", (o, i)), (f"point_embed.layers.{j}.bias", (o,))]
    out += [("query_embed.weight", (Q, d)), ("input_proj.weight", (d, 512, 1, 1)), ("input_proj.bias", (d,))]
    b = "backbone.0.body"
    out += [(f"{b}.conv1.weight", (64, 3, 7, 7))] + _bn_keys(f"{b}.bn1", 64)
    cin = 64
    for li, (w, n, s) in enumerate(_RESNET50_STAGES, start=1):
        for k in range(n):
            p = f"{b}.layer{li}.{k}"
            out += [(f"{p}.conv1.weight", (w, cin, 1, 1))] + _bn_keys(f"{p}.bn1", w)
            out += [(f"{p}.conv2.weight", (w, w, 3, 3))] + _bn_keys(f"{p}.bn2", w)
            out += [(f"{p}.conv3.weight", (4 * w, w, 1, 1))] + _bn_keys(f"{p}.bn3", 4 * w)
            if k == 0:
                out += [(f"{p}.downsample.0.weight", (4 * w, cin, 1, 1))] + _bn_keys(f"{p}.downsample.1", 4 * w)
            cin = 4 * w
    out += [("backbone.0.s8_latern.weight", (256, 512, 1, 1)),
            ("backbone.0.s16_latern.weight", (256, 1024, 3, 3)),
            ("backbone.0.output_conv.weight", (512, 512, 3, 3)),
            ("backbone.0.output_conv.bias", (512,))]
    if cfg.sigma_head:
        for j, (o, i) in enumerate([(d, d), (d, d), (1, d)]):
            out += [(f"sigma_embed.layers.{j}.weight", (o, i)), (f"sigma_embed.layers.{j}.bias", (o,))]
    return out


def random_weights(cfg: SpeConfig, seed: int = 0):
    """Deterministic random-init weights (dict key -> float32 ndarray).

    Conv weights are He-normal, linear/attention weights Xavier-uniform (the reference's
    `_reset_parameters`, REV/models/transformer.py:45-48), FrozenBN stats non-trivial and
    the residual-branch gain (bn3 weight) damped so activations stay O(1) through 13
    bottlenecks without batch statistics."""
    rng = np.random.Generator(np.random.PCG64(seed))
    w = {}
    for key, shape in param_shapes(cfg):
        if key.endswith("running_mean"):
            a = rng.normal(0.0, 0.1, shape)
        elif key.endswith("running_var"):
            a = rng.uniform(0.5, 1.5, shape)
        elif len(shape) == 4:
            fan_in = shape[1] * shape[2] * shape[3]
            a = rng.normal(0.0, np.sqrt(2.0 / fan_in), shape)
        elif len(shape) == 2:
            lim = np.sqrt(6.0 / (shape[0] + shape[1]))
            a = rng.uniform(-lim, lim, shape)
            if key == "query_embed.weight":
                a = rng.normal(0.0, 1.0, shape)
        else:  # 1-D: BN/LN affine or bias
            if ".bn" in key or "downsample.1" in key:
                if key.endswith("weight"):
                    gain = 0.25 if (".bn3" in key) else 1.0
                    a = gain * rng.uniform(0.5, 1.0, shape)
                else:
                    a = rng.normal(0.0, 0.05, shape)
            elif "norm" in key and key.endswith("weight"):
                a = 1.0 + rng.normal(0.0, 0.1, shape)
            else:
                a = rng.normal(0.0, 0.02, shape)
        w[key] = np.ascontiguousarray(a, dtype=np.float32)
    return w


def random_pose(rng, n):
    q = rng.normal(0.0, 1.0, (n, 4))
    q /= np.linalg.norm(q, axis=1, keepdims=True)
    z = rng.uniform(3.0, 30.0, n)
    t = np.stack([rng.normal(0.0, 0.3, n), rng.normal(0.0, 0.3, n), z], axis=1)
    return q, t


def clip_bbox_val(bbox, image_size=(Camera.nu, Camera.nv)):
    """1.2x max-side square around the landmark box, clipped to the image
    (REV/datasets/speed.py:246-260)."""
    x1, y1, x2, y2 = bbox
    scale = max(x2 - x1, y2 - y1) * 1.2
    xc, yc, h = (x1 + x2) / 2, (y1 + y2) / 2, scale / 2
    c = np.asarray([xc - h, yc - h, xc + h, yc + h], dtype=np.float64)
    c[0::2] = c[0::2].clip(0, image_size[0])
    c[1::2] = c[1::2].clip(0, image_size[1])
    return c


def synthetic_batch(cfg: SpeConfig, B: int, seed: int = 0, dtype=np.float32):
    """B synthetic SPEED crops. Returns dict with images [B,3,S,S] (ImageNet-normalised, fp32),
    crops_u8 [B,S,S] (the 8-bit grayscale crops `images` is the to_tensor + Normalize of, in fp32 --
    spe_forward_stages_u8's input), quat [B,4], tvec [B,3], landmarks [B,11,2] (image px),
    clip_bbox [B,4]."""
    rng = np.random.Generator(np.random.PCG64(seed))
    S = cfg.input_size
    W = world_points()
    q, t = random_pose(rng, B)
    lm = np.stack([project(W, q[i], t[i]) for i in range(B)])
    boxes = np.stack([clip_bbox_val([l[:, 0].min(), l[:, 1].min(), l[:, 0].max(), l[:, 1].max()]) for l in lm])
    ys, xs = np.meshgrid(np.arange(S, dtype=np.float32) + 0.5, np.arange(S, dtype=np.float32) + 0.5, indexing="ij")
    imgs = np.empty((B, 3, S, S), dtype=np.float32)
    crops = np.empty((B, S, S), dtype=np.uint8)
    for i in range(B):
        x1, y1, x2, y2 = boxes[i]
        sx, sy = S / max(x2 - x1, 1e-3), S / max(y2 - y1, 1e-3)
        g = rng.normal(30.0, 10.0, (S, S)).astype(np.float32)
        sig = max(4.0 * sx, 1.5)
        for (u, v) in lm[i]:
            cx, cy = (u - x1) * sx, (v - y1) * sy
            g += 200.0 * np.exp(-((xs - cx) ** 2 + (ys - cy) ** 2) / (2 * sig * sig))
        u8 = np.clip(np.round(g), 0, 255)
        crops[i] = u8.astype(np.uint8)
        g = u8 / 255.0                                   # (float32: to_tensor's u8 / 255)
        for c in range(3):
            imgs[i, c] = (g - IMAGENET_MEAN[c]) / IMAGENET_STD[c]
    return {"images": imgs.astype(dtype), "crops_u8": crops, "quat": q, "tvec": t, "landmarks": lm,
            "clip_bbox": boxes}


def synthetic_frames(B: int, seed: int = 0, height: int = Camera.nv, width: int = Camera.nu, channels: int = 1):
    """B synthetic full SPEED frames (8-bit grayscale like the dataset, or replicated RGB):
    background noise N(30, 10) plus a Gaussian blob (sigma 4 px) at every projected landmark of
    a random pose.  Returns frames uint8 [B,H,W] (or [B,H,W,3]), bbox_xxyy [B,4] (landmark
    box, the annotation field REV/datasets/speed.py:216 reads), quat, tvec, landmarks."""
    rng = np.random.Generator(np.random.PCG64(seed))
    W = world_points()
    q, t = random_pose(rng, B)
    lm = np.stack([project(W, q[i], t[i]) for i in range(B)])
    frames = np.empty((B, height, width), np.uint8)
    r = 16
    oy, ox = np.meshgrid(np.arange(-r, r + 1), np.arange(-r, r + 1), indexing="ij")
    for i in range(B):
        g = rng.normal(30.0, 10.0, (height, width)).astype(np.float32)
        for (u, v) in lm[i]:
            cx, cy = int(np.floor(u)), int(np.floor(v))
            ys, xs = cy + oy, cx + ox
            ok = (ys >= 0) & (ys < height) & (xs >= 0) & (xs < width)
            d2 = (xs - u) ** 2 + (ys - v) ** 2
            g[ys[ok], xs[ok]] += (200.0 * np.exp(-d2 / (2 * 4.0 ** 2)))[ok]
        frames[i] = np.clip(np.round(g), 0, 255).astype(np.uint8)
    bbox = np.stack([[l[:, 0].min(), l[:, 1].min(), l[:, 0].max(), l[:, 1].max()] for l in lm])
    if channels == 3:
        frames = np.repeat(frames[..., None], 3, -1)
    return {"frames": frames, "bbox_xxyy": bbox, "quat": q, "tvec": t, "landmarks": lm}


# ---------------------------------------------------------------------------- bench weights
# With plain random init every query of the DETR decoder attends almost uniformly over the
# 2704 memory tokens, so all queries carry nearly the same embedding and the class head gives
# every query the same label: the solver then sees < 4 correspondences and stops at the
# cv2.error path for every image, which would understate its cost in an end-to-end benchmark.
# The two helpers below keep the architecture and the random init but (1) sharpen the decoder
# cross-attention queries so different queries attend to different tokens, and (2) draw the
# class head inside the principal subspace of its own inputs, so queries predict distinct
# labels like a trained model and the solver runs on >= 4 correspondences.

def sharpen_decoder(w, cfg: SpeConfig, factor: float = 64.0):
    d = cfg.hidden_dim
    for l in range(cfg.dec_layers):
        k = f"transformer.decoder.layers.{l}.multihead_attn.in_proj_weight"
        w[k] = w[k].copy()
        w[k][:d] *= factor
    return w


def diversify_class_head(w, hs, seed: int = 1, k: int = 12, logit_scale: float = 6.0, head: str = "cls_embed",
                         within_image: bool = False):
    """hs: [N, d] decoder outputs (after decoder_norm) of a calibration batch; head: the class
    head's state_dict prefix (RT-DETR: decoder.dec_score_head.<last layer>).  within_image (hs
    [B, Q, d]): the head's directions come from the spread of each image's queries about their
    image mean, projected off the span of the image means' differences -- so the head ignores
    which image a query belongs to and labels by the within-image differences alone (RT-DETR's
    selected queries of one image sit close together: a head that also sees the image means gives
    all of an image's queries the same few labels)."""
    if within_image:
        h3 = np.asarray(hs, np.float64)
        means = h3.mean(axis=1)
        U, sv, _ = np.linalg.svd((means - means.mean(0)).T, full_matrices=False)
        U = U[:, sv > 1e-9 * max(sv.max(), 1e-30)]
        dev = (h3 - means[:, None, :]).reshape(-1, h3.shape[-1])
        dev = dev - (dev @ U) @ U.T
        hs = dev + means.mean(0)
    hs = np.asarray(hs, np.float64).reshape(-1, hs.shape[-1])
    mu = hs.mean(0)
    _, S, Vt = np.linalg.svd(hs - mu, full_matrices=False)
    k = min(k, len(S))
    G = np.random.Generator(np.random.PCG64(seed)).normal(size=(w[f"{head}.weight"].shape[0], k))
    W = G @ (Vt[:k] / np.maximum(S[:k, None], 1e-12)) * logit_scale * np.sqrt(hs.shape[0])
    w[f"{head}.weight"] = W.astype(np.float32)
    w[f"{head}.bias"] = (-W @ mu).astype(np.float32)
    return w


def bench_weights(cfg: SpeConfig, seed: int, hs_fn, calib_batch: int = 16):
    """Random-init weights made label-diverse (see above).  hs_fn(weights, images) -> hs [B,Q,d]
    runs a model on the calibration batch."""
    w = sharpen_decoder(random_weights(cfg, seed), cfg)
    calib = synthetic_batch(cfg, calib_batch, seed=CALIB_SEED)
    return diversify_class_head(w, hs_fn(w, calib["images"]))


# ------------------------------------------------------------------- the bench's image pool
# The bench's images are a fixed seeded pool of BENCH_POOL crops (the north-star global batch,
# BASELINE.json): image g is synthetic_batch(cfg, 1, BENCH_SEED + g), and a rank with per-GPU batch B
# times pool images [rank*B, rank*B + B) (modulo the pool).  The pool does not depend on the
# number of ranks, so the head fit below and every image's result are the same at 1 and 8 GPUs.
BENCH_POOL = 256
BENCH_SEED = 1000
CALIB_SEED = 4242
HEADS_KEYS = ["cls_embed.weight", "cls_embed.bias"] + [f"point_embed.layers.{j}.{k}" for j in range(3)
                                                      for k in ("weight", "bias")]


def bench_images(cfg: SpeConfig, first: int, count: int, pool: int = BENCH_POOL):
    """Pool images first .. first+count-1 (indices modulo `pool`), as one synthetic_batch dict."""
    parts = [synthetic_batch(cfg, 1, seed=BENCH_SEED + (g % pool)) for g in range(first, first + count)]
    return {k: np.concatenate([p[k] for p in parts]) for k in parts[0]}


def heads_fixture_path(cfg: SpeConfig, seed: int = 0):
    import os
    return os.path.join(os.path.dirname(os.path.abspath(__file__)), "data",
                        f"bench_heads_s{cfg.input_size}_q{cfg.num_queries}_l{cfg.enc_layers}-{cfg.dec_layers}"
                        f"_seed{seed}.npz")


def fixed_bench_weights(cfg: SpeConfig, seed: int = 0):
    """The bench's pose-consistent weights from the committed head fixture, or None when no
    fixture exists for this shape: random_weights(seed) with the sharpened decoder, and the class
    head + fitted point head stored by oracle/gen_bench_heads.py (computed once from the torch-fp32
    restatement of the reference model on the CPU, so they depend on no kernel of this repo, on no
    device and on no rank count).  Returns (weights, fixture metadata)."""
    import json
    import os
    path = heads_fixture_path(cfg, seed)
    if not os.path.exists(path):
        return None, None
    z = np.load(path)        # plain arrays (allow_pickle stays False)
    w = sharpen_decoder(random_weights(cfg, seed), cfg)
    for k in HEADS_KEYS:
        if z[k].shape != w[k].shape:
            raise ValueError(f"{path}: {k} has shape {z[k].shape}, the model expects {w[k].shape}")
        w[k] = np.ascontiguousarray(z[k], np.float32)
    return w, json.loads(str(z["meta"]))


def weights_checksum(w) -> str:
    """sha256 over the state dict (sorted keys, float32 bytes), first 16 hex digits."""
    import hashlib
    h = hashlib.sha256()
    for k in sorted(w):
        h.update(k.encode())
        h.update(np.ascontiguousarray(w[k], np.float32).tobytes())
    return h.hexdigest()[:16]


# ------------------------------------------------------------- pose-consistent point head
# Label-diverse weights give queries distinct labels, but their random point head puts every
# keypoint near the crop centre, so no pose explains them: RANSAC finds no consensus and the
# refinement the RANSAC configs name never runs.  A trained model's keypoints are the landmark
# projections up to a few pixels.  fit_point_head fits the point MLP (same 256-256-256-2 + sigmoid
# architecture, REV/models/detr_speed.py:52,84) on the decoder outputs of the batch the bench times,
# like a short training run, so that each foreground query predicts its label's landmark
# projection plus the SURVEY 8(d) stress-set noise: N(0, noise_px) and a fraction of uniform
# outliers inside the crop.

def keypoint_targets(batch, labels, seed: int = 0, noise_px: float = 2.0, outlier_frac: float = 0.1):
    """Crop-normalised targets [B,Q,2] for queries labelled `labels` [B,Q] (11 = no object;
    those keep target 0.5 and are masked out).  Returns (targets, mask [B,Q] bool)."""
    rng = np.random.Generator(np.random.PCG64(seed))
    lm, cb = batch["landmarks"], np.asarray(batch["clip_bbox"], np.float64)
    B, Q = labels.shape
    tgt = np.full((B, Q, 2), 0.5)
    mask = labels < lm.shape[1]
    for i in range(B):
        w, h = cb[i, 2] - cb[i, 0], cb[i, 3] - cb[i, 1]
        for q in range(Q):
            if not mask[i, q]:
                continue
            if rng.uniform() < outlier_frac:
                tgt[i, q] = rng.uniform(0.02, 0.98, 2)
                continue
            u, v = lm[i, labels[i, q]] + rng.normal(0.0, noise_px, 2)
            tgt[i, q] = ((u - cb[i, 0]) / w, (v - cb[i, 1]) / h)
    return np.clip(tgt, 1e-3, 1 - 1e-3), mask


def fit_point_head(w, hs, targets, mask, steps: int = 2000, lr: float = 1e-3, seed: int = 0, device="cpu",
                   prefix: str = "point_embed", noise_rel: float = 2.0 ** -8, offset=None):
    """Fit the 3-layer point MLP to `targets` [N,2] on decoder outputs `hs` [N,d] (rows with
    mask False ignored).  Full-batch Adam in torch on `device`; the input standardisation is
    folded into layer 0 afterwards.  Every step perturbs the inputs by Gaussian noise of
    noise_rel x |hs| (bf16's rounding scale): the hs of different images differ by only a few
    percent, and an unregularised interpolant of them amplifies any perturbation of hs (such as
    fp32 vs bf16 rounding) into tens of pixels, unlike a trained model; the noise keeps the fitted
    head smooth at that scale.  offset [N,2] (logits): the head's output is sigmoid(MLP(hs) +
    offset) -- RT-DETR's refined points, sigmoid(dec_bbox_head(hs) + inverse_sigmoid(reference))
    (UNC src/zoo/rtdetr/rtdetr_decoder.py:336-337).  Returns (weights, fit error in target units [N] on masked rows)."""
    import torch
    hs = torch.as_tensor(np.asarray(hs, np.float32).reshape(-1, np.shape(hs)[-1]), device=device)
    y = torch.as_tensor(np.asarray(targets, np.float32).reshape(-1, 2), device=device)
    m = torch.as_tensor(np.asarray(mask).reshape(-1), device=device)
    off = 0.0 if offset is None else torch.as_tensor(np.asarray(offset, np.float32).reshape(-1, 2), device=device)
    mu, sd = hs.mean(0), hs.std(0) + 1e-6
    x = (hs - mu) / sd
    d = hs.shape[1]
    g = torch.Generator(device="cpu").manual_seed(seed)
    shapes = [(d, d), (d, d), (2, d)]
    params = []
    for o, i in shapes:
        lim = (6.0 / (o + i)) ** 0.5
        params += [((torch.rand(o, i, generator=g) * 2 - 1) * lim).to(device).requires_grad_(),
                   torch.zeros(o, device=device, requires_grad=True)]

    def net(z):
        z = torch.relu(z @ params[0].t() + params[1])
        z = torch.relu(z @ params[2].t() + params[3])
        return torch.sigmoid(z @ params[4].t() + params[5] + off)

    opt = torch.optim.Adam(params, lr=lr)
    sched = torch.optim.lr_scheduler.CosineAnnealingLR(opt, steps)
    gn = torch.Generator(device=device).manual_seed(seed + 1)
    nstd = noise_rel * hs.abs() / sd
    for _ in range(steps):
        xin = x + nstd * torch.randn(x.shape, generator=gn, device=device) if noise_rel > 0 else x
        loss = ((net(xin) - y)[m] ** 2).mean()
        opt.zero_grad()
        loss.backward()
        opt.step()
        sched.step()
    with torch.no_grad():
        err = (net(x) - y)[m].abs().amax(1)
        W0 = params[0] / sd[None, :]
        b0 = params[1] - W0 @ mu
        out = dict(w)
        for j, (Wj, bj) in enumerate(((W0, b0), (params[2], params[3]), (params[4], params[5]))):
            out[f"{prefix}.layers.{j}.weight"] = Wj.detach().float().cpu().numpy().copy()
            out[f"{prefix}.layers.{j}.bias"] = bj.detach().float().cpu().numpy().copy()
    return out, err.cpu().numpy()
