"""ORACLE (test infrastructure only -- never imported by the product path).

torch-fp32 functional restatement of the UNC RT-DETR keypoint model's inference forward
(SURVEY §8f.4), over a state dict in the reference's key space (spe.rtdetr_spec):

  PResNet-vd backbone      UNC/nn/backbone/presnet.py:34-124 (BasicBlock / BottleNeck, variant
                           d shortcut = AvgPool2d(2, 2, ceil_mode) + 1x1 ConvNormLayer),
                           :156-265 (3-conv stem, max-pool, stages, return_idx [1, 2, 3])
  HybridEncoder            UNC/src/zoo/rtdetr/hybrid_encoder.py:332-401: input_proj (1x1 + BN),
                           AIFI = one post-norm TransformerEncoderLayer (GELU) on the stride-32
                           level with the 2D sin-cos table of :306-330, top-down FPN (1x1
                           lateral + nearest x2 + CSPRepLayer), bottom-up PAN (bicubic x0.5 +
                           CSPRepLayer); CSPRepLayer / RepVggBlock :40-124
  RTDETRTransformer        UNC/src/zoo/rtdetr/rtdetr_decoder.py:555-710: level input_proj,
                           level-concatenated memory, enc_output + enc heads + anchors, top-k
                           query selection, 3 decoder layers (self-attention, multi-scale
                           deformable cross-attention :105-196 with the grid_sample core of
                           UNC/src/zoo/rtdetr/utils.py:15-64, FFN), per-layer refined points,
                           score and sigma heads (:298-372)
  RTDETRPostProcessor      UNC/src/zoo/rtdetr/rtdetr_postprocessor.py:44-76

Pinned against the reference itself: oracle/gen_golden_rtdetr.py imports the UNC model code
(through a small in-container shim for its `src.core.register` decorator) and records its
outputs in tests/golden/rtdetr_*.npz; tests/test_rtdetr.py checks this restatement against
them.  torch ops (conv2d, batch_norm, grid_sample, interpolate) are the reference's own
third-party arithmetic and are used as such.
"""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F


def _t(w, k):
    v = w[k]
    return v if torch.is_tensor(v) else torch.from_numpy(v)


def conv_norm(x, w, p, stride=1, act=None):
    """ConvNormLayer (UNC/nn/backbone/common.py:8-25, hybrid_encoder.py:17-37)."""
    cw = _t(w, f"{p}.conv.weight")
    k = cw.shape[-1]
    y = F.conv2d(x, cw, None, stride, (k - 1) // 2)
    y = F.batch_norm(y, _t(w, f"{p}.norm.running_mean"), _t(w, f"{p}.norm.running_var"),
                     _t(w, f"{p}.norm.weight"), _t(w, f"{p}.norm.bias"), False, 0.0, 1e-5)
    return act(y) if act is not None else y


def presnet(x, w, cfg):
    """PResNet variant d, return_idx [1, 2, 3] (presnet.py:156-265)."""
    from spe.rtdetr_spec import RESNET_CFG
    x = conv_norm(x, w, "backbone.conv1.conv1_1", 2, F.relu)
    x = conv_norm(x, w, "backbone.conv1.conv1_2", 1, F.relu)
    x = conv_norm(x, w, "backbone.conv1.conv1_3", 1, F.relu)
    x = F.max_pool2d(x, kernel_size=3, stride=2, padding=1)
    outs = []
    for i, n in enumerate(RESNET_CFG[cfg.depth]):
        for j in range(n):
            p = f"backbone.res_layers.{i}.blocks.{j}"
            stride = 2 if j == 0 and i > 0 else 1
            if cfg.depth >= 50:
                o = conv_norm(x, w, f"{p}.branch2a", 1, F.relu)
                o = conv_norm(o, w, f"{p}.branch2b", stride, F.relu)
                o = conv_norm(o, w, f"{p}.branch2c", 1)
            else:
                o = conv_norm(x, w, f"{p}.branch2a", stride, F.relu)
                o = conv_norm(o, w, f"{p}.branch2b", 1)
            if j == 0:
                if stride == 2:
                    s = conv_norm(F.avg_pool2d(x, 2, 2, 0, ceil_mode=True), w, f"{p}.short.conv", 1)
                else:
                    s = conv_norm(x, w, f"{p}.short", 1)
            else:
                s = x
            x = F.relu(o + s)
        if i >= 1:
            outs.append(x)
    return outs


def sincos_2d(w_, h_, d=256, temperature=10000.0):
    """HybridEncoder.build_2d_sincos_position_embedding (hybrid_encoder.py:306-330), [h*w, d];
    note the (w, h) meshgrid with indexing 'ij' flattened against an h*w token order."""
    gw, gh = torch.meshgrid(torch.arange(int(w_), dtype=torch.float32), torch.arange(int(h_), dtype=torch.float32),
                            indexing="ij")
    pd = d // 4
    omega = torch.arange(pd, dtype=torch.float32) / pd
    omega = 1.0 / (temperature ** omega)
    ow = gw.flatten()[..., None] @ omega[None]
    oh = gh.flatten()[..., None] @ omega[None]
    return torch.concat([ow.sin(), ow.cos(), oh.sin(), oh.cos()], dim=1)


def mha(q_in, k_in, v_in, w, p, nheads=8):
    """nn.MultiheadAttention(batch_first=True) forward in eval, [B, L, d] -> [B, Lq, d]."""
    W, bvec = _t(w, f"{p}.in_proj_weight"), _t(w, f"{p}.in_proj_bias")
    d = W.shape[1]
    q = F.linear(q_in, W[:d], bvec[:d])
    k = F.linear(k_in, W[d:2 * d], bvec[d:2 * d])
    v = F.linear(v_in, W[2 * d:], bvec[2 * d:])
    B, Lq, _ = q.shape
    Lk = k.shape[1]
    hd = d // nheads
    q = q.reshape(B, Lq, nheads, hd).transpose(1, 2) / math.sqrt(hd)
    k = k.reshape(B, Lk, nheads, hd).transpose(1, 2)
    v = v.reshape(B, Lk, nheads, hd).transpose(1, 2)
    a = torch.softmax(q @ k.transpose(-1, -2), dim=-1) @ v
    return F.linear(a.transpose(1, 2).reshape(B, Lq, d), _t(w, f"{p}.out_proj.weight"), _t(w, f"{p}.out_proj.bias"))


def layer_norm(x, w, p):
    return F.layer_norm(x, (x.shape[-1],), _t(w, f"{p}.weight"), _t(w, f"{p}.bias"), 1e-5)


def csp_rep_layer(x, w, p, cfg):
    """CSPRepLayer with one RepVggBlock (hybrid_encoder.py:40-124): conv3(rep(conv1(x)) + conv2(x))."""
    x1 = conv_norm(x, w, f"{p}.conv1", 1, F.silu)
    x2 = conv_norm(x, w, f"{p}.conv2", 1, F.silu)
    r = conv_norm(x1, w, f"{p}.bottlenecks.0.conv1", 1) + conv_norm(x1, w, f"{p}.bottlenecks.0.conv2", 1)
    y = F.silu(r) + x2
    return conv_norm(y, w, f"{p}.conv3", 1, F.silu) if cfg.csp_hidden != cfg.hidden_dim else y


def hybrid_encoder(feats, w, cfg):
    """HybridEncoder.forward (hybrid_encoder.py:332-401)."""
    d = cfg.hidden_dim
    proj = []
    for i, f in enumerate(feats):
        y = F.conv2d(f, _t(w, f"encoder.input_proj.{i}.0.weight"))
        y = F.batch_norm(y, _t(w, f"encoder.input_proj.{i}.1.running_mean"), _t(w, f"encoder.input_proj.{i}.1.running_var"),
                         _t(w, f"encoder.input_proj.{i}.1.weight"), _t(w, f"encoder.input_proj.{i}.1.bias"), False, 0.0, 1e-5)
        proj.append(y)
    # AIFI on the stride-32 level (use_encoder_idx [2]), eval_spatial_size table
    B, _, h, wd = proj[2].shape
    src = proj[2].flatten(2).permute(0, 2, 1)
    s5 = cfg.input_size // 32
    pos = sincos_2d(s5, s5, d)[None]
    p = "encoder.encoder.0.layers.0"
    qk = src + pos
    src = layer_norm(src + mha(qk, qk, src, w, f"{p}.self_attn", cfg.nheads), w, f"{p}.norm1")
    ff = F.linear(F.gelu(F.linear(src, _t(w, f"{p}.linear1.weight"), _t(w, f"{p}.linear1.bias"))),
                  _t(w, f"{p}.linear2.weight"), _t(w, f"{p}.linear2.bias"))
    src = layer_norm(src + ff, w, f"{p}.norm2")
    proj[2] = src.permute(0, 2, 1).reshape(-1, d, h, wd).contiguous()
    aifi = proj[2]
    # top-down FPN
    inner = [proj[-1]]
    for idx in range(len(feats) - 1, 0, -1):
        hi = conv_norm(inner[0], w, f"encoder.lateral_convs.{len(feats) - 1 - idx}", 1, F.silu)
        inner[0] = hi
        up = F.interpolate(hi, scale_factor=2.0, mode="nearest")
        inner.insert(0, csp_rep_layer(torch.concat([up, proj[idx - 1]], 1), w,
                                      f"encoder.fpn_blocks.{len(feats) - 1 - idx}", cfg))
    # bottom-up PAN
    outs = [inner[0]]
    for idx in range(len(feats) - 1):
        down = F.interpolate(outs[-1], scale_factor=0.5, mode="bicubic")
        outs.append(csp_rep_layer(torch.concat([down, inner[idx + 1]], 1), w, f"encoder.pan_blocks.{idx}", cfg))
    return outs, aifi


def inverse_sigmoid(x, eps=1e-5):
    """utils.py:10-12"""
    x = x.clip(min=0.0, max=1.0)
    return torch.log(x.clip(min=eps) / (1 - x).clip(min=eps))


def mlp(x, w, p, n, act=F.relu):
    for j in range(n):
        x = F.linear(x, _t(w, f"{p}.layers.{j}.weight"), _t(w, f"{p}.layers.{j}.bias"))
        if j < n - 1:
            x = act(x)
    return x


def anchors(cfg, eps=1e-2):
    """RTDETRTransformer._generate_anchors (rtdetr_decoder.py:577-611), [1, L, 2] logits."""
    out = []
    for s in cfg.level_sizes:
        gy, gx = torch.meshgrid(torch.arange(s, dtype=torch.float32), torch.arange(s, dtype=torch.float32), indexing="ij")
        gxy = (torch.stack([gx, gy], -1).unsqueeze(0) + 0.5) / torch.tensor([s, s], dtype=torch.float32)
        out.append(gxy.reshape(-1, s * s, 2))
    a = torch.concat(out, 1)
    valid = ((a > eps) * (a < 1 - eps)).all(-1, keepdim=True)
    a = torch.log(a / (1 - a))
    return torch.where(valid, a, torch.inf)


def deformable_core(value, shapes, loc, aw):
    """utils.py:15-64: value [B, L, H, c], loc [B, Lq, H, nl, np, 2], aw [B, Lq, H, nl, np]."""
    B, _, H, c = value.shape
    _, Lq, _, nl, npt, _ = loc.shape
    vals = value.split([h * w for h, w in shapes], dim=1)
    grids = 2 * loc - 1
    sampled = []
    for lv, (h, w) in enumerate(shapes):
        v = vals[lv].flatten(2).permute(0, 2, 1).reshape(B * H, c, h, w)
        g = grids[:, :, :, lv].permute(0, 2, 1, 3, 4).flatten(0, 1)
        sampled.append(F.grid_sample(v, g, mode="bilinear", padding_mode="zeros", align_corners=False))
    aw = aw.permute(0, 2, 1, 3, 4).reshape(B * H, 1, Lq, nl * npt)
    out = (torch.stack(sampled, dim=-2).flatten(-2) * aw).sum(-1).reshape(B, H * c, Lq)
    return out.permute(0, 2, 1)


def ms_deform_attn(query, ref, value_in, w, p, cfg):
    """MSDeformableAttention.forward (rtdetr_decoder.py:105-196) for 2-d reference points."""
    B, Lq, d = query.shape
    H, nl, npt = cfg.nheads, cfg.num_levels, cfg.num_points
    value = F.linear(value_in, _t(w, f"{p}.value_proj.weight"), _t(w, f"{p}.value_proj.bias")).reshape(B, -1, H, d // H)
    off = F.linear(query, _t(w, f"{p}.sampling_offsets.weight"), _t(w, f"{p}.sampling_offsets.bias")).reshape(B, Lq, H, nl, npt, 2)
    aw = F.linear(query, _t(w, f"{p}.attention_weights.weight"), _t(w, f"{p}.attention_weights.bias")).reshape(B, Lq, H, nl * npt)
    aw = F.softmax(aw, dim=-1).reshape(B, Lq, H, nl, npt)
    shapes = [[s, s] for s in cfg.level_sizes]
    # offset / (W_l, H_l) per level.  (The reference indexes the normaliser into a 10-d tensor
    # and squeezes every size-1 dimension afterwards, so its batch-1 forward fails; the
    # arithmetic for B > 1 is this broadcast.)
    norm = torch.tensor(shapes).flip([1]).reshape(1, 1, 1, nl, 1, 2)
    loc = ref[:, :, None, :, None, :] + off / norm
    out = deformable_core(value, shapes, loc, aw)
    return F.linear(out, _t(w, f"{p}.output_proj.weight"), _t(w, f"{p}.output_proj.bias"))


def rtdetr_decoder(feats, w, cfg, trace=None):
    """RTDETRTransformer.forward in eval (rtdetr_decoder.py:505-710)."""
    d, Q = cfg.hidden_dim, cfg.num_queries
    flat = []
    for i, f in enumerate(feats):
        y = conv_norm(f, w, f"decoder.input_proj.{i}", 1)
        flat.append(y.flatten(2).permute(0, 2, 1))
    memory = torch.concat(flat, 1)
    out_mem = layer_norm(F.linear(memory, _t(w, "decoder.enc_output.0.weight"), _t(w, "decoder.enc_output.0.bias")),
                         w, "decoder.enc_output.1")
    enc_cls = F.linear(out_mem, _t(w, "decoder.enc_score_head.weight"), _t(w, "decoder.enc_score_head.bias"))
    enc_coord = mlp(out_mem, w, "decoder.enc_bbox_head", 3) + anchors(cfg)
    _, topk = torch.topk(enc_cls.max(-1).values, Q, dim=1)
    ref_unact = enc_coord.gather(1, topk.unsqueeze(-1).repeat(1, 1, 2))
    enc_topk_bboxes = torch.sigmoid(ref_unact)
    enc_topk_logits = enc_cls.gather(1, topk.unsqueeze(-1).repeat(1, 1, enc_cls.shape[-1]))
    tgt = out_mem.gather(1, topk.unsqueeze(-1).repeat(1, 1, d))
    if trace is not None:
        trace.update(memory=memory, topk=topk, enc_topk_logits=enc_topk_logits, enc_topk_bboxes=enc_topk_bboxes)
    ref = torch.sigmoid(ref_unact)
    logits, pts, sigmas = [], [], []
    out = tgt
    for i in range(cfg.dec_layers):
        p = f"decoder.decoder.layers.{i}"
        qpos = mlp(ref, w, "decoder.query_pos_head", 2)
        qk = out + qpos
        out = layer_norm(out + mha(qk, qk, out, w, f"{p}.self_attn", cfg.nheads), w, f"{p}.norm1")
        out = layer_norm(out + ms_deform_attn(out + qpos, ref.unsqueeze(2), memory, w, f"{p}.cross_attn", cfg), w, f"{p}.norm2")
        ff = F.linear(F.relu(F.linear(out, _t(w, f"{p}.linear1.weight"), _t(w, f"{p}.linear1.bias"))),
                      _t(w, f"{p}.linear2.weight"), _t(w, f"{p}.linear2.bias"))
        out = layer_norm(out + ff, w, f"{p}.norm3")
        new_ref = torch.sigmoid(mlp(out, w, f"decoder.dec_bbox_head.{i}", 3) + inverse_sigmoid(ref))
        logits.append(F.linear(out, _t(w, f"decoder.dec_score_head.{i}.weight"), _t(w, f"decoder.dec_score_head.{i}.bias")))
        pts.append(new_ref)
        sigmas.append(mlp(out, w, f"decoder.decoder.sigma_embed.{i}", 3).repeat(1, 1, 2))
        ref = new_ref
    return {"pred_logits": logits[-1], "pred_pts": pts[-1], "pred_sigmas": sigmas[-1],
            "aux_logits": torch.stack(logits[:-1]), "aux_pts": torch.stack(pts[:-1]), "aux_sigmas": torch.stack(sigmas[:-1]),
            "enc_topk_logits": enc_topk_logits, "enc_topk_bboxes": enc_topk_bboxes}


@torch.no_grad()
def forward(images, w, cfg, trace=None):
    """images [B, 3, S, S] fp32 (numpy or torch) -> dict of the reference's outputs."""
    x = images if torch.is_tensor(images) else torch.from_numpy(images)
    feats = presnet(x.float(), w, cfg)
    enc, aifi = hybrid_encoder(feats, w, cfg)
    if trace is not None:
        trace.update(feats=feats, enc=enc, aifi=aifi)
    return rtdetr_decoder(enc, w, cfg, trace)


def postprocess(out, clip_bbox):
    """RTDETRPostProcessor.forward (rtdetr_postprocessor.py:44-76): softmax probabilities,
    crop -> image pixels, sigma = exp(pred_sigmas)."""
    prob = torch.softmax(out["pred_logits"], -1)
    pts = out["pred_pts"].clone()
    cb = torch.as_tensor(clip_bbox, dtype=pts.dtype)
    for b in range(pts.shape[0]):
        pts[b, :, 0] = pts[b, :, 0] * (cb[b, 2] - cb[b, 0]) + cb[b, 0]
        pts[b, :, 1] = pts[b, :, 1] * (cb[b, 3] - cb[b, 1]) + cb[b, 1]
    return {"probs": prob, "points": pts, "sigmas": torch.exp(out["pred_sigmas"])}
