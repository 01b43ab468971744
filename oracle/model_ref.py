"""ORACLE (test infrastructure only — never imported by the product path).

Plain torch-fp32 CPU restatement of the reference keypoint-set predictor, operating on a
state_dict in the reference's 412-key naming:

  backbone   REV/models/backbone.py:44-54 (FrozenBN), :105-149 (Backbone8s: ResNet-50
             stem+layer1..3, s8/s16 neck), torchvision ResNet-50 v1.5 structure
  pos-embed  REV/models/position_encoding.py:30-53 (sine, normalize=True, 128 feats)
  DETR       REV/models/detr_speed.py:59-92 (input_proj, transformer, heads)
  encoder    REV/models/transformer.py:154-167 (post-norm), decoder :218-239, :100-129
  post-proc  REV/models/detr_speed.py:266-293
  sigma head UNC/src/zoo/rtdetr/rtdetr_decoder.py:295-297,367 + exp in
             UNC/src/zoo/rtdetr/rtdetr_postprocessor.py:53

Pinned against golden vectors produced by importing the reference model code itself in
the build container (oracle/gen_golden.py -> tests/golden/model_*.npz).
"""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F


def _frozen_bn(x, sd, p):
    scale = sd[p + ".weight"] * (sd[p + ".running_var"] + 1e-5).rsqrt()
    shift = sd[p + ".bias"] - sd[p + ".running_mean"] * scale
    return x * scale[None, :, None, None] + shift[None, :, None, None]


def _bottleneck(x, sd, p, stride):
    y = F.relu(_frozen_bn(F.conv2d(x, sd[p + ".conv1.weight"]), sd, p + ".bn1"))
    y = F.relu(_frozen_bn(F.conv2d(y, sd[p + ".conv2.weight"], stride=stride, padding=1), sd, p + ".bn2"))
    y = _frozen_bn(F.conv2d(y, sd[p + ".conv3.weight"]), sd, p + ".bn3")
    if (p + ".downsample.0.weight") in sd:
        idt = _frozen_bn(F.conv2d(x, sd[p + ".downsample.0.weight"], stride=stride), sd, p + ".downsample.1")
    else:
        idt = x
    return F.relu(y + idt)


def backbone_s8(x, sd):
    """Returns (xs8 [B,512,S/8,S/8], xs16 [B,1024,S/16,S/16], neck out [B,512,S/8,S/8])."""
    b = "backbone.0.body"
    y = F.relu(_frozen_bn(F.conv2d(x, sd[b + ".conv1.weight"], stride=2, padding=3), sd, b + ".bn1"))
    y = F.max_pool2d(y, 3, 2, 1)
    feats = {}
    for li, n in ((1, 3), (2, 4), (3, 6)):
        for k in range(n):
            y = _bottleneck(y, sd, f"{b}.layer{li}.{k}", 2 if (k == 0 and li > 1) else 1)
        feats[li] = y
    xs8, xs16 = feats[2], feats[3]
    a = F.conv2d(xs8, sd["backbone.0.s8_latern.weight"])
    up = F.interpolate(xs16, scale_factor=2, mode="bilinear", align_corners=True)
    c = F.conv2d(up, sd["backbone.0.s16_latern.weight"], padding=1)
    out = F.conv2d(torch.cat([a, c], 1), sd["backbone.0.output_conv.weight"],
                   sd["backbone.0.output_conv.bias"], padding=1)
    return xs8, xs16, out


def sine_pos(h, w, d=256, dtype=torch.float32):
    """Position table for an all-valid mask, [d, h, w]."""
    npf = d // 2
    eps, scale = 1e-6, 2 * math.pi
    ye = torch.arange(1, h + 1, dtype=torch.float32)[:, None].expand(h, w)
    xe = torch.arange(1, w + 1, dtype=torch.float32)[None, :].expand(h, w)
    ye = ye / (float(h) + eps) * scale
    xe = xe / (float(w) + eps) * scale
    dim_t = torch.arange(npf, dtype=torch.float32)
    dim_t = 10000.0 ** (2 * torch.div(dim_t, 2, rounding_mode="floor") / npf)
    px = xe[..., None] / dim_t
    py = ye[..., None] / dim_t
    px = torch.stack((px[..., 0::2].sin(), px[..., 1::2].cos()), dim=3).flatten(2)
    py = torch.stack((py[..., 0::2].sin(), py[..., 1::2].cos()), dim=3).flatten(2)
    return torch.cat((py, px), dim=2).permute(2, 0, 1).to(dtype)


def _mha(q_in, k_in, v_in, sd, p, nheads):
    """nn.MultiheadAttention (batch-first here: [B, L, d]) with packed in_proj."""
    W, bvec = sd[p + ".in_proj_weight"], sd[p + ".in_proj_bias"]
    d = W.shape[1]
    hd = d // nheads
    q = F.linear(q_in, W[:d], bvec[:d])
    k = F.linear(k_in, W[d:2 * d], bvec[d:2 * d])
    v = F.linear(v_in, W[2 * d:], bvec[2 * d:])
    B, Lq, _ = q.shape
    Lk = k.shape[1]
    q = q.view(B, Lq, nheads, hd).transpose(1, 2) * (hd ** -0.5)
    k = k.view(B, Lk, nheads, hd).transpose(1, 2)
    v = v.view(B, Lk, nheads, hd).transpose(1, 2)
    a = torch.softmax(q @ k.transpose(-1, -2), dim=-1) @ v
    a = a.transpose(1, 2).reshape(B, Lq, d)
    return F.linear(a, sd[p + ".out_proj.weight"], sd[p + ".out_proj.bias"])


def _ln(x, sd, p):
    return F.layer_norm(x, (x.shape[-1],), sd[p + ".weight"], sd[p + ".bias"], 1e-5)


def _mlp3(x, sd, p):
    x = F.relu(F.linear(x, sd[p + ".layers.0.weight"], sd[p + ".layers.0.bias"]))
    x = F.relu(F.linear(x, sd[p + ".layers.1.weight"], sd[p + ".layers.1.bias"]))
    return F.linear(x, sd[p + ".layers.2.weight"], sd[p + ".layers.2.bias"])


def forward(images, sd, cfg, return_stages=False):
    """images [B,3,S,S] fp32 -> dict(pred_logits [B,Q,12], pred_points [B,Q,2], hs [L,B,Q,d],
    optional pred_sigmas [B,Q,2])."""
    images = torch.as_tensor(images, dtype=torch.float32)
    dev = images.device                                 # CPU, or a GPU for the precision-floor test
    sd = {k: torch.as_tensor(v, dtype=torch.float32).to(dev) for k, v in sd.items()}
    xs8, xs16, neck = backbone_s8(images, sd)
    B, _, h, w = neck.shape
    nh = cfg.nheads
    src = F.conv2d(neck, sd["input_proj.weight"], sd["input_proj.bias"])
    pos = sine_pos(h, w, cfg.hidden_dim).to(dev)[None].expand(B, -1, -1, -1)
    src = src.flatten(2).transpose(1, 2)               # [B, HW, d] (row-major h*W + w)
    pos = pos.flatten(2).transpose(1, 2)
    for i in range(cfg.enc_layers):
        p = f"transformer.encoder.layers.{i}"
        qk = src + pos
        src = _ln(src + _mha(qk, qk, src, sd, p + ".self_attn", nh), sd, p + ".norm1")
        ff = F.linear(F.relu(F.linear(src, sd[p + ".linear1.weight"], sd[p + ".linear1.bias"])),
                      sd[p + ".linear2.weight"], sd[p + ".linear2.bias"])
        src = _ln(src + ff, sd, p + ".norm2")
    memory = src
    qpos = sd["query_embed.weight"][None].expand(B, -1, -1)
    tgt = torch.zeros_like(qpos)
    hs = []
    for i in range(cfg.dec_layers):
        p = f"transformer.decoder.layers.{i}"
        qk = tgt + qpos
        tgt = _ln(tgt + _mha(qk, qk, tgt, sd, p + ".self_attn", nh), sd, p + ".norm1")
        tgt = _ln(tgt + _mha(tgt + qpos, memory + pos, memory, sd, p + ".multihead_attn", nh), sd, p + ".norm2")
        ff = F.linear(F.relu(F.linear(tgt, sd[p + ".linear1.weight"], sd[p + ".linear1.bias"])),
                      sd[p + ".linear2.weight"], sd[p + ".linear2.bias"])
        tgt = _ln(tgt + ff, sd, p + ".norm3")
        hs.append(_ln(tgt, sd, "transformer.decoder.norm"))
    hs = torch.stack(hs)                                # [L, B, Q, d]
    logits = F.linear(hs, sd["cls_embed.weight"], sd["cls_embed.bias"])
    points = _mlp3(hs, sd, "point_embed").sigmoid()
    out = {"pred_logits": logits[-1], "pred_points": points[-1], "hs": hs,
           "aux_logits": logits[:-1], "aux_points": points[:-1]}
    if cfg.sigma_head:
        out["pred_sigmas"] = _mlp3(hs[-1], sd, "sigma_embed").repeat(1, 1, 2)   # log-sigma
    if return_stages:
        out.update(xs8=xs8, xs16=xs16, neck=neck, memory=memory)
    return out


def postprocess(logits, points, clip_bbox, log_sigmas=None):
    """REV/models/detr_speed.py:266-293 (+ UNC sigma = exp(log-sigma))."""
    prob = torch.softmax(torch.as_tensor(logits, dtype=torch.float32), -1)
    pts = torch.as_tensor(points, dtype=torch.float32).clone()
    res = []
    for i, bb in enumerate(clip_bbox):
        bb = [float(v) for v in bb]
        wdt, hgt = bb[2] - bb[0], bb[3] - bb[1]
        pts[i, :, 0] = pts[i, :, 0] * wdt + bb[0]
        pts[i, :, 1] = pts[i, :, 1] * hgt + bb[1]
        r = {"logits": prob[i].numpy(), "points": pts[i].numpy()}
        if log_sigmas is not None:
            r["sigmas"] = torch.exp(torch.as_tensor(log_sigmas[i])).numpy()
        res.append(r)
    return res
