"""UNC RT-DETR keypoint model: PResNet-vd + HybridEncoder + RTDETRTransformer
with the sigma head (UNC/src/zoo/rtdetr/*, UNC/nn/backbone/presnet.py).

CPU: the parameter space (spe.rtdetr_spec) equals the reference model's own state_dict keys
and shapes (tests/golden/rtdetr_keys_r*.json), and the torch-fp32 restatement
(oracle/rtdetr_ref.py) reproduces the reference's outputs recorded by
oracle/gen_golden_rtdetr.py (tests/golden/rtdetr_*.npz): same top-k query selection, outputs to
fp32 rounding.  GPU (tests marked gpu): the HIP path against the same goldens.

Tolerances (written here on purpose):
  oracle vs reference      pred_pts / pred_sigmas |d| <= 1e-5, logits |d| <= 1e-4, top-k exact
  HIP fp32 parity mode     pred_pts |d| <= 1e-4 (BASELINE keypoint tolerance), logits and
                           sigmas |d| <= 2e-3, top-k indices exact
  HIP bf16                 pred_pts |d| <= 3e-2, logits |d| <= 0.3 on queries whose selection
                           agrees with the reference (bf16 rounding can reorder near-tied
                           encoder scores; the selected sets must still overlap >= 80 %)
"""
import json
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN
from spe.config import SpeConfig
from spe.rtdetr_spec import RtdetrConfig, rtdetr_param_shapes, random_rtdetr_weights
from spe.synthetic import synthetic_batch
import rtdetr_ref

TAGS = ["r18_s128", "r18_s256", "r50_s256"]


def _golden(tag):
    g = np.load(os.path.join(GOLDEN, f"rtdetr_{tag}.npz"))
    cfg = RtdetrConfig(**json.loads(str(g["config"])))
    return g, cfg


def _chk(a):
    a = np.asarray(a, np.float64)
    return np.array([a.sum(), np.abs(a).sum(), (a * a).sum(), a.ravel()[:: max(1, a.size // 97)].sum()])


@pytest.mark.parametrize("depth", [18, 50])
def test_param_space_matches_reference_state_dict(depth):
    with open(os.path.join(GOLDEN, f"rtdetr_keys_r{depth}.json")) as f:
        ref = [(k, tuple(s)) for k, s in json.load(f) if not k.endswith("num_batches_tracked")]
    mine = [(k, tuple(s)) for k, s in rtdetr_param_shapes(RtdetrConfig(depth=depth))]
    assert mine == ref


@pytest.mark.parametrize("tag", TAGS)
def test_oracle_matches_reference_golden(tag):
    g, cfg = _golden(tag)
    w = random_rtdetr_weights(cfg, int(g["weight_seed"]))
    b = synthetic_batch(SpeConfig(input_size=cfg.input_size), int(g["batch"]), int(g["image_seed"]))
    np.testing.assert_allclose(_chk(b["images"]), g["input_checksum"], rtol=1e-6)
    trace = {}
    o = rtdetr_ref.forward(b["images"], w, cfg, trace)
    for i, t in enumerate(trace["feats"]):
        np.testing.assert_allclose(_chk(t.numpy()), g[f"chk_feat{i}"], rtol=1e-4)
    for i, t in enumerate(trace["enc"]):
        np.testing.assert_allclose(_chk(t.numpy()), g[f"chk_enc{i}"], rtol=1e-4)
    np.testing.assert_array_equal(trace["topk"].numpy(), g["topk_ind"])
    np.testing.assert_allclose(o["pred_pts"].numpy(), g["pred_pts"], atol=1e-5)
    np.testing.assert_allclose(o["pred_sigmas"].numpy(), g["pred_sigmas"], atol=1e-5)
    np.testing.assert_allclose(o["pred_logits"].numpy(), g["pred_logits"], atol=1e-4)
    np.testing.assert_allclose(o["aux_pts"].numpy(), g["aux_pts"], atol=1e-5)
    np.testing.assert_allclose(o["aux_logits"].numpy(), g["aux_logits"], atol=1e-4)
    np.testing.assert_allclose(o["enc_topk_logits"].numpy(), g["enc_topk_logits"], atol=1e-4)
    np.testing.assert_allclose(o["enc_topk_bboxes"].numpy(), g["enc_topk_bboxes"], atol=1e-5)


def test_oracle_postprocess_matches_reference_formula():
    """RTDETRPostProcessor (UNC/src/zoo/rtdetr/rtdetr_postprocessor.py:44-76) on golden outputs."""
    g, cfg = _golden("r18_s128")
    out = {k: torch.from_numpy(g[k]) for k in ("pred_logits", "pred_pts", "pred_sigmas")}
    pp = rtdetr_ref.postprocess(out, g["clip_bbox"])
    cb = g["clip_bbox"]
    px = g["pred_pts"][..., 0] * (cb[:, 2:3] - cb[:, 0:1]) + cb[:, 0:1]
    np.testing.assert_allclose(pp["points"][..., 0].numpy(), px, rtol=1e-6)
    np.testing.assert_allclose(pp["sigmas"].numpy(), np.exp(g["pred_sigmas"]), rtol=1e-6)
    np.testing.assert_allclose(pp["probs"].numpy().sum(-1), 1.0, rtol=1e-6)


_hip_models = {}


def _hip_model(cfg, dtype, wseed):
    from spe.rtdetr import RTDETR
    key = (cfg, dtype, wseed)
    if key not in _hip_models:
        m = RTDETR(cfg, dtype)
        m.load_state_dict(random_rtdetr_weights(cfg, wseed))
        _hip_models[key] = m
    return _hip_models[key]


def _hip_forward(tag, dtype, dev):
    g, cfg = _golden(tag)
    m = _hip_model(cfg, dtype, int(g["weight_seed"]))
    b = synthetic_batch(SpeConfig(input_size=cfg.input_size), int(g["batch"]), int(g["image_seed"]))
    o = m(torch.from_numpy(b["images"]).to(dev), clip_bbox=torch.from_numpy(g["clip_bbox"]).float().to(dev))
    torch.cuda.synchronize()
    return g, cfg, o


@pytest.mark.gpu
@pytest.mark.parametrize("tag", TAGS)
def test_hip_fp32_matches_reference(gpu_device, tag):
    g, cfg, o = _hip_forward(tag, "fp32", gpu_device)
    np.testing.assert_array_equal(o["topk"].cpu().numpy(), g["topk_ind"])
    c = lambda t: t.cpu().numpy()
    assert np.abs(c(o["pred_pts"]) - g["pred_pts"]).max() <= 1e-4
    assert np.abs(c(o["pred_logits"]) - g["pred_logits"]).max() <= 2e-3
    assert np.abs(c(o["pred_sigmas"]) - g["pred_sigmas"]).max() <= 2e-3
    aux = o["aux_outputs"]
    assert np.abs(np.stack([c(a["pred_pts"]) for a in aux[:-1]]) - g["aux_pts"]).max() <= 1e-4
    assert np.abs(np.stack([c(a["pred_logits"]) for a in aux[:-1]]) - g["aux_logits"]).max() <= 2e-3
    assert np.abs(np.stack([c(a["pred_sigmas"]) for a in aux[:-1]]) - g["aux_sigmas"]).max() <= 2e-3
    assert np.abs(c(aux[-1]["pred_pts"]) - g["enc_topk_bboxes"]).max() <= 1e-4
    assert np.abs(c(aux[-1]["pred_logits"]) - g["enc_topk_logits"]).max() <= 2e-3
    # fused RTDETRPostProcessor == the reference's formula on the reference's outputs
    ref = rtdetr_ref.postprocess({k: torch.from_numpy(g[k]) for k in ("pred_logits", "pred_pts", "pred_sigmas")},
                                 g["clip_bbox"])
    assert np.abs(c(o["points_px"]) - ref["points"].numpy()).max() <= 0.05
    assert np.abs(c(o["probs"]) - ref["probs"].numpy()).max() <= 1e-3
    assert np.abs(c(o["sigmas"]) - ref["sigmas"].numpy()).max() <= 5e-3 * max(1.0, float(ref["sigmas"].max()))


@pytest.mark.gpu
@pytest.mark.parametrize("tag", TAGS)
def test_hip_bf16_close_to_reference(gpu_device, tag):
    g, cfg, o = _hip_forward(tag, "bf16", gpu_device)
    sel, ref_sel = o["topk"].cpu().numpy(), g["topk_ind"]
    for b in range(sel.shape[0]):
        assert len(set(sel[b]) & set(ref_sel[b])) >= 0.8 * cfg.num_queries
        same = sel[b] == ref_sel[b]           # queries selected in the same rank
        if same.sum() == 0:
            continue
        assert np.abs(o["pred_pts"][b].cpu().numpy()[same] - g["pred_pts"][b][same]).max() <= 3e-2
        assert np.abs(o["pred_logits"][b].cpu().numpy()[same] - g["pred_logits"][b][same]).max() <= 0.3


@pytest.mark.gpu
def test_hip_batch_independence(gpu_device):
    """Image i's outputs do not depend on the rest of the batch (per-image top-k, level-major
    memory indexing)."""
    g, cfg = _golden("r18_s128")
    m = _hip_model(cfg, "fp32", int(g["weight_seed"]))
    b = synthetic_batch(SpeConfig(input_size=cfg.input_size), 4, 9)
    x = torch.from_numpy(b["images"]).to(gpu_device)
    full = m(x)
    part = m(x[1:3].contiguous())
    torch.cuda.synchronize()
    np.testing.assert_array_equal(full["topk"][1:3].cpu().numpy(), part["topk"].cpu().numpy())
    assert (full["pred_pts"][1:3] - part["pred_pts"]).abs().max().item() <= 1e-5


@pytest.mark.gpu
def test_hip_hs_output_feeds_score_head(gpu_device):
    """The optional hs output is the last decoder layer's output: the reference's last score head
    (rtdetr_decoder.py dec_score_head[-1]) applied to it gives pred_logits."""
    g, cfg = _golden("r18_s128")
    m = _hip_model(cfg, "fp32", int(g["weight_seed"]))
    w = random_rtdetr_weights(cfg, int(g["weight_seed"]))
    b = synthetic_batch(SpeConfig(input_size=cfg.input_size), int(g["batch"]), int(g["image_seed"]))
    o = m(torch.from_numpy(b["images"]).to(gpu_device), return_hs=True)
    torch.cuda.synchronize()
    hs = o["hs"].cpu().numpy().astype(np.float64)
    k = f"decoder.dec_score_head.{cfg.dec_layers - 1}"
    logits = hs @ w[f"{k}.weight"].T.astype(np.float64) + w[f"{k}.bias"]
    assert np.abs(logits - o["pred_logits"].cpu().numpy()).max() <= 1e-4


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", ["fp32", "bf16"])
def test_hip_nan_scores_select_valid_queries(gpu_device, dtype):
    """Every encoder score NaN (a NaN in the encoder score head; a NaN input image does not get
    there, since the fused ReLU epilogues map NaN to 0).  torch.topk ranks NaN above every number
    and returns the tied NaNs lowest index first; the HIP selection must pick the same valid,
    distinct tokens instead of faulting on an unset index."""
    from spe.rtdetr import RTDETR
    g, cfg = _golden("r18_s128")
    w = random_rtdetr_weights(cfg, int(g["weight_seed"]))
    w["decoder.enc_score_head.bias"] = w["decoder.enc_score_head.bias"].copy()
    w["decoder.enc_score_head.bias"][3] = np.nan
    m = RTDETR(cfg, dtype)
    m.load_state_dict(w)
    b = synthetic_batch(SpeConfig(input_size=cfg.input_size), 3, 31)
    o = m(torch.from_numpy(b["images"]).to(gpu_device))
    torch.cuda.synchronize()
    tk = o["topk"].cpu().numpy()
    for r in tk:
        np.testing.assert_array_equal(r, np.arange(cfg.num_queries))
