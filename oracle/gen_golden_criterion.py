"""Golden vectors for the set criterion (runs ONLY in the build container, where /root/reference
exists).

Feeds the reference's own outputs stored in tests/golden/model_<tag>.npz (pred_logits /
pred_points of the last decoder layer and the 5 aux layers) and seeded synthetic targets to the
reference's SetCriterion + HungarianMatcher (REV/models/detr_speed.py:103-261,
REV/models/matcher.py:35-88, built by REV/models/detr_speed.py:296-336 with the REV/main.py
defaults set_cost_class=1, set_cost_pts=5, pts_loss_coef=5, eos_coef=0.1, aux_loss=True) and
records the loss dict and the matching of every layer:

  tests/golden/criterion_<tag>.npz : tgt_labels [B,T], tgt_points [B,T,2], loss_names,
      loss_values, match_query [L,B,T] (query matched to target t, layer L-1 = last).

Usage: python oracle/gen_golden_criterion.py
"""
from __future__ import annotations

import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from gen_golden import CASES, REPO, _args, _import_reference  # noqa: E402

from spe.config import SpeConfig  # noqa: E402
from spe.synthetic import synthetic_batch  # noqa: E402


def targets_for(cfg, B, image_seed):
    """Targets as SpeedTrain(train=False) builds them (REV/datasets/speed.py:209-233): labels
    0..10, landmarks in crop-normalised coordinates ((lm - clip[:2]) scaled by S / crop size,
    then / S by Normalize)."""
    b = synthetic_batch(cfg, B, image_seed)
    clip = b["clip_bbox"]
    pts = (b["landmarks"] - clip[:, None, :2]) / (clip[:, None, 2:] - clip[:, None, :2])
    labels = np.tile(np.arange(pts.shape[1], dtype=np.int64), (B, 1))
    return labels, pts.astype(np.float32)


def main():
    import torch
    build_model, _ = _import_reference()
    for tag, (cfg, B, wseed, iseed) in CASES.items():
        g = np.load(os.path.join(REPO, "tests", "golden", f"model_{tag}.npz"))
        _, criterion, _ = build_model(_args(cfg))
        labels, pts = targets_for(cfg, B, iseed)
        targets = [{"labels": torch.from_numpy(labels[i]), "landmarks": torch.from_numpy(pts[i])} for i in range(B)]
        outputs = {"pred_logits": torch.from_numpy(g["pred_logits"]), "pred_points": torch.from_numpy(g["pred_points"]),
                   "aux_outputs": [{"pred_logits": torch.from_numpy(a), "pred_points": torch.from_numpy(p)}
                                   for a, p in zip(g["aux_logits"], g["aux_points"])]}
        with torch.no_grad():
            losses = criterion(outputs, targets)
            layers = outputs["aux_outputs"] + [{k: v for k, v in outputs.items() if k != "aux_outputs"}]
            match = np.full((len(layers), B, labels.shape[1]), -1, np.int32)
            for l, o in enumerate(layers):
                for b, (qi, ti) in enumerate(criterion.matcher(o, targets)):
                    match[l, b, ti.numpy()] = qi.numpy()
        names = sorted(losses)
        rec = {"config": json.dumps(cfg.to_dict()), "tgt_labels": labels, "tgt_points": pts,
               "loss_names": np.array(names), "loss_values": np.array([float(losses[k]) for k in names]),
               "match_query": match}
        path = os.path.join(REPO, "tests", "golden", f"criterion_{tag}.npz")
        np.savez_compressed(path, **rec)
        print("wrote", path, dict(zip(names, rec["loss_values"].round(5))))


if __name__ == "__main__":
    _ = SpeConfig
    main()
