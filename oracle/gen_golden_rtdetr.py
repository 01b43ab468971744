"""Golden-vector generator for the UNC RT-DETR keypoint model.  Runs ONLY in
the build container, where /root/reference exists.

Loads the reference's own model files (UNC/src/zoo/rtdetr/{utils,denoising,hybrid_encoder,
rtdetr_decoder,rtdetr}.py, UNC/nn/backbone/{common,presnet}.py) as synthetic packages, with a
stand-in for the one symbol they need from the broken `src` package (`src.core.register`, an
identity class decorator for inference) and `box_ops` left empty (training-only denoising
helpers import it; torchvision is absent).  No reference code is copied; only numeric outputs
are written:

  tests/golden/rtdetr_keys_r{18,50}.json : the reference model's state_dict keys and shapes
  tests/golden/rtdetr_<tag>.npz          : config, seeds, the reference's outputs on seeded
                                           synthetic crops (pred_logits / pred_pts /
                                           pred_sigmas, aux layers, encoder top-k), the top-k
                                           query indices and per-stage checksums

Usage: python oracle/gen_golden_rtdetr.py
"""
from __future__ import annotations

import importlib.util
import json
import os
import sys
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
UNC = "/root/reference/Monocular Satellite Pose Estimation Based on Uncertainty Estimation and Self-Assessment"
sys.path.insert(0, os.path.join(REPO, "satellite-pose-estimation_amd"))

from spe.config import SpeConfig  # noqa: E402
from spe.rtdetr_spec import RtdetrConfig, random_rtdetr_weights  # noqa: E402
from spe.synthetic import synthetic_batch  # noqa: E402

CASES = {
    # tag: (cfg, batch, weight seed, image seed)
    "r18_s128": (RtdetrConfig(depth=18, input_size=128), 2, 21, 22),
    "r18_s256": (RtdetrConfig(depth=18, input_size=256), 2, 1, 2),
    "r50_s256": (RtdetrConfig(depth=50, input_size=256), 2, 3, 4),
}


def _load(name, path, pkg):
    spec = importlib.util.spec_from_file_location(name, path)
    m = importlib.util.module_from_spec(spec)
    m.__package__ = pkg
    sys.modules[name] = m
    spec.loader.exec_module(m)
    return m


def import_reference():
    core = types.ModuleType("src.core")
    core.register = lambda cls: cls
    src = types.ModuleType("src")
    src.__path__ = []
    src.core = core
    sys.modules.setdefault("src", src)
    sys.modules.setdefault("src.core", core)
    zoo = os.path.join(UNC, "src", "zoo", "rtdetr")
    pkg = types.ModuleType("unc_rtdetr")
    pkg.__path__ = [zoo]
    sys.modules["unc_rtdetr"] = pkg
    _load("unc_rtdetr.utils", os.path.join(zoo, "utils.py"), "unc_rtdetr")
    box_ops = types.ModuleType("unc_rtdetr.box_ops")           # training-only (denoising)
    box_ops.box_cxcywh_to_xyxy = box_ops.box_xyxy_to_cxcywh = None
    sys.modules["unc_rtdetr.box_ops"] = box_ops
    _load("unc_rtdetr.denoising", os.path.join(zoo, "denoising.py"), "unc_rtdetr")
    he = _load("unc_rtdetr.hybrid_encoder", os.path.join(zoo, "hybrid_encoder.py"), "unc_rtdetr")
    dec = _load("unc_rtdetr.rtdetr_decoder", os.path.join(zoo, "rtdetr_decoder.py"), "unc_rtdetr")
    rt = _load("unc_rtdetr.rtdetr", os.path.join(zoo, "rtdetr.py"), "unc_rtdetr")
    bbp = types.ModuleType("unc_backbone")
    bbp.__path__ = [os.path.join(UNC, "nn", "backbone")]
    sys.modules["unc_backbone"] = bbp
    _load("unc_backbone.common", os.path.join(UNC, "nn", "backbone", "common.py"), "unc_backbone")
    pres = _load("unc_backbone.presnet", os.path.join(UNC, "nn", "backbone", "presnet.py"), "unc_backbone")
    return pres, he, dec, rt


def build_reference(cfg: RtdetrConfig):
    """The speed-config model (UNC/configs/rtdetr_speed/rtdetr_r{18,50}vd_6x_speed_kl_*.yml)."""
    pres, he, dec, rt = import_reference()
    S = [cfg.input_size, cfg.input_size]
    bb = pres.PResNet(depth=cfg.depth, variant="d", return_idx=[1, 2, 3], freeze_at=-1, freeze_norm=False,
                      pretrained=False)
    enc = he.HybridEncoder(in_channels=cfg.backbone_channels, feat_strides=[8, 16, 32], hidden_dim=cfg.hidden_dim,
                           use_encoder_idx=[2], num_encoder_layers=1, nhead=cfg.nheads, dim_feedforward=cfg.enc_ff,
                           dropout=0.0, enc_act="gelu", expansion=cfg.expansion, depth_mult=1, act="silu",
                           eval_spatial_size=S)
    d = dec.RTDETRTransformer(num_classes=cfg.num_classes, feat_channels=[cfg.hidden_dim] * 3, feat_strides=[8, 16, 32],
                              hidden_dim=cfg.hidden_dim, num_levels=cfg.num_levels, num_queries=cfg.num_queries,
                              num_decoder_layers=cfg.dec_layers, dim_feedforward=cfg.dec_ff, num_denoising=0, eval_idx=-1,
                              eval_spatial_size=S)
    return rt.RTDETR(bb, enc, d).eval()


def _chk(a):
    a = np.asarray(a, np.float64)
    return np.array([a.sum(), np.abs(a).sum(), (a * a).sum(), a.ravel()[:: max(1, a.size // 97)].sum()])


def main():
    import torch
    torch.set_num_threads(os.cpu_count() or 8)
    out_dir = os.path.join(REPO, "tests", "golden")
    for depth in (18, 50):
        m = build_reference(RtdetrConfig(depth=depth))
        keys = [[k, list(v.shape)] for k, v in m.state_dict().items()]
        with open(os.path.join(out_dir, f"rtdetr_keys_r{depth}.json"), "w") as f:
            json.dump(keys, f)
    for tag, (cfg, B, wseed, iseed) in CASES.items():
        model = build_reference(cfg)
        w = random_rtdetr_weights(cfg, wseed)
        missing, unexpected = model.load_state_dict({k: torch.from_numpy(v) for k, v in w.items()}, strict=False)
        assert not unexpected and all(k.endswith("num_batches_tracked") for k in missing), (missing, unexpected)
        batch = synthetic_batch(SpeConfig(input_size=cfg.input_size), B, iseed)
        stages = {}
        model.backbone.register_forward_hook(lambda mod, i, o: stages.update(feats=[t.detach() for t in o]))
        model.encoder.register_forward_hook(lambda mod, i, o: stages.update(enc=[t.detach() for t in o]))
        topk = {}
        orig_topk = torch.topk

        def spy_topk(x, k, *a, **kw):
            r = orig_topk(x, k, *a, **kw)
            topk["ind"] = r[1].detach().clone()
            return r
        torch.topk = spy_topk
        try:
            with torch.no_grad():
                out = model(torch.from_numpy(batch["images"]))
        finally:
            torch.topk = orig_topk
        aux = out["aux_outputs"]
        rec = {
            "config": json.dumps(cfg.to_dict()), "batch": B, "weight_seed": wseed, "image_seed": iseed,
            "input_checksum": _chk(batch["images"]),
            "pred_logits": out["pred_logits"].numpy(), "pred_pts": out["pred_pts"].numpy(),
            "pred_sigmas": out["pred_sigmas"].numpy(),
            "aux_logits": np.stack([a["pred_logits"].numpy() for a in aux[:-1]]),
            "aux_pts": np.stack([a["pred_pts"].numpy() for a in aux[:-1]]),
            "aux_sigmas": np.stack([a["pred_sigmas"].numpy() for a in aux[:-1]]),
            "enc_topk_logits": aux[-1]["pred_logits"].numpy(), "enc_topk_bboxes": aux[-1]["pred_pts"].numpy(),
            "topk_ind": topk["ind"].numpy(), "clip_bbox": batch["clip_bbox"],
        }
        for i, t in enumerate(stages["feats"]):
            rec[f"chk_feat{i}"] = _chk(t.numpy())
        for i, t in enumerate(stages["enc"]):
            rec[f"chk_enc{i}"] = _chk(t.numpy())
        path = os.path.join(out_dir, f"rtdetr_{tag}.npz")
        np.savez_compressed(path, **rec)
        print("wrote", path, {k: np.asarray(v).shape for k, v in rec.items() if k != "config"})


if __name__ == "__main__":
    main()
