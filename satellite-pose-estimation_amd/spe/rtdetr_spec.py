"""Parameter space of the UNC RT-DETR keypoint model.

The reference model is `RTDETR(PResNet, HybridEncoder, RTDETRTransformer)`
(UNC/src/zoo/rtdetr/rtdetr.py:20-38, UNC/nn/backbone/presnet.py:156-265,
UNC/src/zoo/rtdetr/hybrid_encoder.py:196-401, UNC/src/zoo/rtdetr/rtdetr_decoder.py:372-555)
as the speed configs build it (UNC/configs/rtdetr_speed/rtdetr_r{18,50}vd_6x_speed_kl_*.yml:
256x256 input, 30 queries, 3 decoder layers, hybrid-encoder expansion 0.5, no denoising).

* `RtdetrConfig`                 - the config fields those YAML files set.
* `rtdetr_param_shapes(cfg)`     - (key, shape) in the reference's state_dict order
                                   (BatchNorm `num_batches_tracked` buffers omitted, like
                                   FrozenBatchNorm2d drops them, UNC/nn/backbone/common.py:46-68).
* `random_rtdetr_weights(cfg, s)`- deterministic random weights in that key space.
"""
from __future__ import annotations

from dataclasses import dataclass, asdict

import numpy as np

RESNET_CFG = {18: [2, 2, 2, 2], 34: [3, 4, 6, 3], 50: [3, 4, 6, 3], 101: [3, 4, 23, 3]}   # presnet.py:17-23


@dataclass(frozen=True)
class RtdetrConfig:
    depth: int = 50                 # PResNet.depth (r18vd / r50vd), variant "d"
    input_size: int = 256           # eval_spatial_size / dataset resize
    num_queries: int = 30           # RTDETRTransformer.num_queries
    dec_layers: int = 3             # RTDETRTransformer.num_decoder_layers
    hidden_dim: int = 256
    nheads: int = 8
    enc_ff: int = 1024              # HybridEncoder.dim_feedforward (AIFI, GELU)
    dec_ff: int = 1024              # RTDETRTransformer.dim_feedforward (ReLU)
    expansion: float = 0.5          # HybridEncoder.expansion (CSPRepLayer hidden = 256 * e)
    num_levels: int = 3
    num_points: int = 4             # num_decoder_points
    num_classes: int = 11           # + 1 no-object logit

    @property
    def backbone_channels(self):
        e = 1 if self.depth < 50 else 4
        return [128 * e, 256 * e, 512 * e]          # return_idx [1, 2, 3]: strides 8, 16, 32

    @property
    def level_sizes(self):
        return [self.input_size // s for s in (8, 16, 32)]

    @property
    def tokens(self):
        return sum(s * s for s in self.level_sizes)

    @property
    def csp_hidden(self):
        return int(self.hidden_dim * self.expansion)

    def to_dict(self):
        return asdict(self)


def _bn(p, c):
    return [(f"{p}.{n}", (c,)) for n in ("weight", "bias", "running_mean", "running_var")]


def _cnl(p, cin, cout, k):
    """ConvNormLayer: conv (no bias) + BatchNorm2d (UNC/nn/backbone/common.py:8-25)."""
    return [(f"{p}.conv.weight", (cout, cin, k, k))] + _bn(f"{p}.norm", cout)


def _lin(p, o, i):
    return [(f"{p}.weight", (o, i)), (f"{p}.bias", (o,))]


def _mlp(p, dims):
    out = []
    for j, (i, o) in enumerate(zip(dims[:-1], dims[1:])):
        out += _lin(f"{p}.layers.{j}", o, i)
    return out


def _mha(p, d):
    return [(f"{p}.in_proj_weight", (3 * d, d)), (f"{p}.in_proj_bias", (3 * d,))] + _lin(f"{p}.out_proj", d, d)


def rtdetr_param_shapes(cfg: RtdetrConfig):
    d, C = cfg.hidden_dim, cfg.num_classes + 1
    out = [("temper_param", (1,))]
    # ---- backbone: PResNet variant d (presnet.py:156-230)
    out += _cnl("backbone.conv1.conv1_1", 3, 32, 3) + _cnl("backbone.conv1.conv1_2", 32, 32, 3)
    out += _cnl("backbone.conv1.conv1_3", 32, 64, 3)
    bottleneck = cfg.depth >= 50
    exp = 4 if bottleneck else 1
    cin = 64
    for i, (cout, n) in enumerate(zip([64, 128, 256, 512], RESNET_CFG[cfg.depth])):
        for j in range(n):
            p = f"backbone.res_layers.{i}.blocks.{j}"
            stride = 2 if j == 0 and i > 0 else 1
            blk = []
            if j == 0:                       # shortcut=False on the first block of a stage
                sp = f"{p}.short.conv" if stride == 2 else f"{p}.short"   # variant d: pool + conv
                blk_short = _cnl(sp, cin, cout * exp, 1)
            if bottleneck:
                blk += _cnl(f"{p}.branch2a", cin, cout, 1) + _cnl(f"{p}.branch2b", cout, cout, 3)
                blk += _cnl(f"{p}.branch2c", cout, cout * exp, 1)
                out += blk + (blk_short if j == 0 else [])
            else:                            # BasicBlock registers `short` first (presnet.py:38-53)
                blk += _cnl(f"{p}.branch2a", cin, cout, 3) + _cnl(f"{p}.branch2b", cout, cout, 3)
                out += (blk_short if j == 0 else []) + blk
            cin = cout * exp
    # ---- decoder (RTDETRTransformer, rtdetr_decoder.py:372-505), registered before the encoder
    for lv in range(cfg.num_levels):
        out += _cnl(f"decoder.input_proj.{lv}", d, d, 1)
    P = cfg.nheads * cfg.num_levels * cfg.num_points
    for i in range(cfg.dec_layers):
        p = f"decoder.decoder.layers.{i}"
        out += _mha(f"{p}.self_attn", d) + [(f"{p}.norm1.weight", (d,)), (f"{p}.norm1.bias", (d,))]
        out += _lin(f"{p}.cross_attn.sampling_offsets", 2 * P, d) + _lin(f"{p}.cross_attn.attention_weights", P, d)
        out += _lin(f"{p}.cross_attn.value_proj", d, d) + _lin(f"{p}.cross_attn.output_proj", d, d)
        out += [(f"{p}.norm2.weight", (d,)), (f"{p}.norm2.bias", (d,))]
        out += _lin(f"{p}.linear1", cfg.dec_ff, d) + _lin(f"{p}.linear2", d, cfg.dec_ff)
        out += [(f"{p}.norm3.weight", (d,)), (f"{p}.norm3.bias", (d,))]
    for i in range(cfg.dec_layers):
        out += _mlp(f"decoder.decoder.sigma_embed.{i}", [d, d, d, 1])
    out += _mlp("decoder.query_pos_head", [2, 2 * d, d])
    out += _lin("decoder.enc_output.0", d, d) + [("decoder.enc_output.1.weight", (d,)), ("decoder.enc_output.1.bias", (d,))]
    out += _lin("decoder.enc_score_head", C, d) + _mlp("decoder.enc_bbox_head", [d, d, d, 2])
    for i in range(cfg.dec_layers):
        out += _lin(f"decoder.dec_score_head.{i}", C, d)
    for i in range(cfg.dec_layers):
        out += _mlp(f"decoder.dec_bbox_head.{i}", [d, d, d, 2])
    # ---- hybrid encoder (hybrid_encoder.py:196-300)
    for lv, c in enumerate(cfg.backbone_channels):
        out += [(f"encoder.input_proj.{lv}.0.weight", (d, c, 1, 1))] + _bn(f"encoder.input_proj.{lv}.1", d)
    out += [("encoder.encoder_fusion_input.weight", (d, 3 * d, 1, 1))]       # built, never called
    p = "encoder.encoder.0.layers.0"
    out += _mha(f"{p}.self_attn", d) + _lin(f"{p}.linear1", cfg.enc_ff, d) + _lin(f"{p}.linear2", d, cfg.enc_ff)
    out += [(f"{p}.norm1.weight", (d,)), (f"{p}.norm1.bias", (d,)), (f"{p}.norm2.weight", (d,)), (f"{p}.norm2.bias", (d,))]
    for i in range(cfg.num_levels - 1):
        out += _cnl(f"encoder.lateral_convs.{i}", d, d, 1)
    h = cfg.csp_hidden
    for blocks in ("fpn_blocks", "pan_blocks"):
        for i in range(cfg.num_levels - 1):
            p = f"encoder.{blocks}.{i}"
            out += _cnl(f"{p}.conv1", 2 * d, h, 1) + _cnl(f"{p}.conv2", 2 * d, h, 1)
            out += _cnl(f"{p}.bottlenecks.0.conv1", h, h, 3) + _cnl(f"{p}.bottlenecks.0.conv2", h, h, 1)
            if h != d:
                out += _cnl(f"{p}.conv3", h, d, 1)
    return out


def random_rtdetr_weights(cfg: RtdetrConfig, seed: int = 0):
    """Deterministic random weights (key -> float32 ndarray) that exercise every path: He-normal
    convs with non-trivial BatchNorm statistics (residual gains damped so activations stay O(1)
    through the bottlenecks), Xavier linears, random sampling offsets (sample points fall inside
    and outside the value maps) and attention logits, non-zero box/sigma heads."""
    rng = np.random.Generator(np.random.PCG64(seed))
    w = {}
    for key, shape in rtdetr_param_shapes(cfg):
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
            if "sampling_offsets" in key:
                a = a * 4.0
        elif key == "temper_param":
            a = rng.normal(0.0, 1.0, shape)
        else:   # 1-D: BN / LN affine or a bias
            if ".norm." in key or key.startswith("encoder.input_proj") and key.endswith((".1.weight", ".1.bias")):
                if key.endswith("weight"):
                    gain = 0.3 if ("branch2c" in key or "branch2b" in key and cfg.depth < 50) else 1.0
                    a = gain * rng.uniform(0.5, 1.0, shape)
                else:
                    a = rng.normal(0.0, 0.05, shape)
            elif "norm" in key and key.endswith("weight") or key == "decoder.enc_output.1.weight":
                a = 1.0 + rng.normal(0.0, 0.1, shape)
            elif "sampling_offsets" in key:
                a = rng.normal(0.0, 2.0, shape)
            else:
                a = rng.normal(0.0, 0.02, shape)
        w[key] = np.ascontiguousarray(a, dtype=np.float32)
    return w
