"""Set criterion (Hungarian matcher + losses; REV/models/detr_speed.py:103-261,
REV/models/matcher.py:35-88).

CPU: the assignment restatement (oracle/criterion_ref.lsap) against scipy's
linear_sum_assignment itself -- square, tall (more queries than targets, scipy's transposed
path) and wide matrices, with integer costs so exact ties exercise the tie-break -- and the
loss restatement against the reference's own SetCriterion outputs (tests/golden/criterion_*.npz,
oracle/gen_golden_criterion.py) on the reference's own predictions.
GPU: spe_criterion (csrc/criterion.hip) against the same golden values and matchings, and the
HIP model's aux outputs feeding it end to end.

Tolerances: matchings exact; losses |rel| <= 1e-5 (the reference computes them in fp32).
"""
import json
import os

import numpy as np
import pytest
from scipy.optimize import linear_sum_assignment

import criterion_ref as cr
from conftest import GOLDEN

TAGS = ["s128_q11_l2", "s224_q30_l4", "s416_q11_l6"]


@pytest.mark.parametrize("shape", [(11, 11), (30, 11), (11, 30), (40, 11), (5, 5)])
@pytest.mark.parametrize("ints", [False, True])
def test_lsap_matches_scipy(shape, ints):
    rng = np.random.Generator(np.random.PCG64(shape[0] * 100 + shape[1] + ints))
    for _ in range(25):
        c = rng.integers(0, 4, shape).astype(np.float64) if ints else rng.normal(size=shape)
        r0, c0 = linear_sum_assignment(c)
        r1, c1 = cr.lsap(c)
        assert np.array_equal(r0, r1) and np.array_equal(c0, c1), c
        assert np.isclose(c[r0, c0].sum(), c[r1, c1].sum())


def _golden(tag):
    m = np.load(os.path.join(GOLDEN, f"model_{tag}.npz"))
    c = np.load(os.path.join(GOLDEN, f"criterion_{tag}.npz"))
    layers = [(a, p) for a, p in zip(m["aux_logits"], m["aux_points"])] + [(m["pred_logits"], m["pred_points"])]
    ref = dict(zip([str(n) for n in c["loss_names"]], c["loss_values"]))
    return layers, c, ref


@pytest.mark.parametrize("tag", TAGS)
def test_criterion_oracle_matches_reference(tag):
    layers, c, ref = _golden(tag)
    losses, match = cr.criterion(layers, c["tgt_labels"], c["tgt_points"])
    assert np.array_equal(match, c["match_query"])
    assert set(losses) == set(ref)
    for k, v in ref.items():
        assert abs(losses[k] - v) <= 1e-5 * max(1.0, abs(v)), (k, losses[k], v)


@pytest.mark.gpu
@pytest.mark.parametrize("tag", TAGS)
def test_criterion_hip_matches_reference(gpu_device, tag):
    import torch
    from spe.models import SetCriterion
    layers, c, ref = _golden(tag)
    dev = gpu_device
    outputs = {"pred_logits": torch.from_numpy(layers[-1][0]).to(dev), "pred_points": torch.from_numpy(layers[-1][1]).to(dev),
               "aux_outputs": [{"pred_logits": torch.from_numpy(a).to(dev), "pred_points": torch.from_numpy(p).to(dev)}
                               for a, p in layers[:-1]]}
    targets = [{"labels": torch.from_numpy(c["tgt_labels"][b]).to(dev), "landmarks": torch.from_numpy(c["tgt_points"][b]).to(dev)}
               for b in range(c["tgt_labels"].shape[0])]
    crit = SetCriterion()
    losses = crit(outputs, targets)
    assert np.array_equal(crit.last_match.cpu().numpy(), c["match_query"])
    assert set(losses) == set(ref)
    for k, v in ref.items():
        got = float(losses[k])
        assert abs(got - v) <= 1e-5 * max(1.0, abs(v)), (k, got, v)


@pytest.mark.gpu
def test_criterion_on_hip_model_aux_outputs(gpu_device):
    """fp32 HIP model with aux outputs (every decoder layer through decoder_norm + heads, like
    the reference's aux_loss=True forward) -> spe_criterion == the oracle on the same outputs."""
    import torch
    from spe.config import SpeConfig
    from spe.models import DETR, SetCriterion
    from spe.synthetic import random_weights
    g = np.load(os.path.join(GOLDEN, "model_s128_q11_l2.npz"))
    c = np.load(os.path.join(GOLDEN, "criterion_s128_q11_l2.npz"))
    cfg = SpeConfig(**json.loads(str(g["config"])))
    m = DETR(cfg, dtype="fp32", aux_loss=True)
    m.load_state_dict(random_weights(cfg, int(g["weight_seed"])))
    from spe.synthetic import synthetic_batch
    b = synthetic_batch(cfg, int(g["batch"]), int(g["image_seed"]))
    o = m(torch.from_numpy(b["images"]).to(gpu_device))
    torch.cuda.synchronize()
    aux = o["aux_outputs"]
    assert len(aux) == cfg.dec_layers - 1
    for l, a in enumerate(aux):
        assert np.abs(a["pred_points"].cpu().numpy() - g["aux_points"][l]).max() <= 1e-4
        assert np.abs(a["pred_logits"].cpu().numpy() - g["aux_logits"][l]).max() <= 2e-3
    targets = [{"labels": torch.from_numpy(c["tgt_labels"][i]).to(gpu_device),
                "landmarks": torch.from_numpy(c["tgt_points"][i]).to(gpu_device)} for i in range(len(c["tgt_labels"]))]
    losses = SetCriterion()(o, targets)
    layers = [(a["pred_logits"].cpu().numpy(), a["pred_points"].cpu().numpy()) for a in aux]
    layers.append((o["pred_logits"].cpu().numpy(), o["pred_points"].cpu().numpy()))
    ref, _ = cr.criterion(layers, c["tgt_labels"], c["tgt_points"])
    for k, v in ref.items():
        assert abs(float(losses[k]) - v) <= 1e-5 * max(1.0, abs(v)), k


@pytest.mark.gpu
def test_criterion_near_ties_match_oracle(gpu_device):
    """Near-tie cost matrices: the queries' points are a few ulps apart, so an assignment flips
    on the last bit of cost_pts*cp + cost_class*cc.  criterion.hip is built without FMA
    contraction, like the reference's separate fp32 torch ops; the matchings must equal the
    restatement's exactly.  The logits are all equal so the softmax is exactly 1/12 in every
    implementation (exp(0) = 1) and only the cost rounding decides."""
    import torch
    from spe.models import SetCriterion
    rng = np.random.Generator(np.random.PCG64(77))
    B, Q, T, C = 256, 11, 11, 12
    base_p = rng.uniform(0.2, 0.8, size=(B, 1, 2)).astype(np.float32)
    steps = rng.integers(-3, 4, size=(B, Q, 2))
    pts = (base_p + steps.astype(np.float32) * np.float32(6e-8)).astype(np.float32)
    logits = np.zeros((B, Q, C), np.float32)
    tgt_labels = np.stack([rng.permutation(C - 1)[:T] for _ in range(B)]).astype(np.int64)
    # targets spread over the crop: cp then carries a full mantissa and 5*cp is inexact, so a
    # contracted multiply-add rounds about a third of the costs differently and flips the
    # matching of 255 of these 256 images (checked on the restatement)
    tgt_points = rng.uniform(0, 1, size=(B, T, 2)).astype(np.float32)
    ref, match = cr.criterion([(logits, pts)], tgt_labels, tgt_points)
    d = gpu_device
    crit = SetCriterion()
    losses = crit({"pred_logits": torch.from_numpy(logits).to(d), "pred_points": torch.from_numpy(pts).to(d)},
                  [{"labels": torch.from_numpy(tgt_labels[b]).to(d), "landmarks": torch.from_numpy(tgt_points[b]).to(d)}
                   for b in range(B)])
    assert np.array_equal(crit.last_match.cpu().numpy().reshape(match.shape), match)
    for k, v in ref.items():
        assert abs(float(losses[k]) - v) <= 1e-5 * max(1.0, abs(v)), k
