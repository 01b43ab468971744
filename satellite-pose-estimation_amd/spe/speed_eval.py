"""SPEED evaluator with the reference's interface and log schema
(REV/datasets/speed.py:337-421, REV/utils/speed_eval.py:245-262).

Two update paths feed the same per-image log:
  * update(predictions)            reference per-image path: {filename: {'points','logits'}}
                                   -> solver(points, logits) with the reference exception mapping;
  * update_batch(filenames, ...)   hot path: device pose records from PosePipeline / the batched
                                   solver + spe_speed_score, one D2H copy per batch.
"""
from __future__ import annotations

import json
import os

import numpy as np
import torch

from . import _lib
from .solver import SolverError


def speed_score(q_pr, t_pr, q_gt, t_gt):
    """REV/utils/speed_eval.py:245-262 (host, fp64)."""
    q_pr = np.asarray(q_pr, np.float64).flatten()
    t_pr = np.asarray(t_pr, np.float64).flatten()
    q_gt = np.asarray(q_gt, np.float64).flatten()
    t_gt = np.asarray(t_gt, np.float64).flatten()
    assert q_pr.shape[0] == q_gt.shape[0] == 4
    assert t_pr.shape[0] == t_gt.shape[0] == 3
    if q_pr[0] < 0:
        q_pr = q_pr * -1
    if q_gt[0] < 0:
        q_gt = q_gt * -1
    s_t = np.linalg.norm(t_pr - t_gt, ord=2) / np.linalg.norm(t_gt, ord=2)
    s_q = 2 * np.arccos(min(np.abs(np.dot(q_pr, q_gt)), 1))
    return s_t, s_q


def device_speed_score(quat, tvec, q_gt, t_gt, stream=None):
    """Per-image (s_t, s_q) on device via spe_speed_score. quat [B,4] f32, tvec [B,3] f64,
    q_gt [B,4] / t_gt [B,3] f64."""
    B = quat.shape[0]
    s_t = torch.empty(B, dtype=torch.float64, device=quat.device)
    s_q = torch.empty_like(s_t)
    _lib.check(_lib.lib().spe_speed_score(_lib.stream_ptr(stream), _lib.ptr(quat), _lib.ptr(tvec),
                                          _lib.ptr(q_gt), _lib.ptr(t_gt), B, _lib.ptr(s_t), _lib.ptr(s_q)),
               "spe_speed_score")
    return s_t, s_q


def load_ground_truth(gt):
    """gt: path to a SPEED json list (filename, q_vbs2tango, r_Vo2To_vbs_true) or such a list or
    a ready {filename: {'quat','tvec'}} dict (REV/datasets/speed.py:340-348)."""
    if isinstance(gt, dict):
        return gt
    if isinstance(gt, (str, os.PathLike)):
        with open(gt) as f:
            gt = json.load(f)
    out = {}
    for it in gt:
        r = {"quat": it["q_vbs2tango"], "tvec": it["r_Vo2To_vbs_true"]}
        if "bbox_xxyy" in it:
            # UNC SpeedEval's "area" (src/data/speed/speed_dataset.py:370-373), the operator
            # precedence kept: sqrt((x2 - x1) * y2 - y1) -- EPnPCeresSolver's threshold input
            b = it["bbox_xxyy"]
            r["area"] = float(np.sqrt((b[2] - b[0]) * b[3] - b[1]))
        out[it["filename"]] = r
    return out


class SpeedEval:
    def __init__(self, gt_file, solver):
        self.solver = solver
        self.ground_truth = load_ground_truth(gt_file)
        self.log = {}
        self.stats = ""

    def _record(self, filename, points, logits, quat_pr, tvec_pr, score_tvec, score_quat):
        gt = self.ground_truth[filename]
        self.log[filename] = {
            "points": np.around(points, decimals=2).tolist(),
            "logits": np.around(logits, decimals=6).tolist(),
            "quat_gt": gt["quat"],
            "tvec_gt": gt["tvec"],
            "quat_pr": np.around(quat_pr, decimals=6).tolist(),
            "tvec_pr": np.around(tvec_pr, decimals=6).tolist(),
            "score_tvec": np.around(score_tvec, decimals=8).item(),
            "score_quat": np.around(score_quat, decimals=8).item(),
            "score": np.around(score_quat + score_tvec, decimals=8).item(),
        }

    def update(self, predictions):
        """REV/datasets/speed.py:351-380 (per-image solver calls, zero pose on failure)."""
        for filename, ret in predictions.items():
            try:
                if "sigmas" in ret and getattr(self.solver, "mode", None) == _lib.SPE_PNP_EPNP_RANSAC_SIGMA:
                    quat_pr, tvec_pr = self.solver(ret["points"], ret["logits"], ret["sigmas"])
                else:
                    quat_pr, tvec_pr = self.solver(ret["points"], ret["logits"])
            except (IndexError, SolverError):
                quat_pr, tvec_pr = np.zeros(4), np.zeros(3)
            gt = self.ground_truth[filename]
            s_t, s_q = speed_score(quat_pr, tvec_pr, gt["quat"], gt["tvec"])
            self._record(filename, ret["points"], ret["logits"], quat_pr, tvec_pr, s_t, s_q)

    def update_batch(self, filenames, points_px, probs, poses, s_t=None, s_q=None, sigmas=None, assess=None):
        """Hot-path variant: `poses` is the dict returned by solver.solve_batch (device), optional
        device scores from device_speed_score.  Failed images carry zero poses (status != 0
        except RANSAC_FALLBACK), exactly as update() produces them.  With the sigma head the
        record also carries "sigma" (UNC/src/data/speed/speed_dataset.py:437, 8 dp) and, when
        `assess` (solver.self_assess output) is given, the self-assessment verdict."""
        sg = sigmas.detach().cpu().numpy() if sigmas is not None else None
        ms = assess["mean_sigma"].cpu().numpy() if assess is not None else None
        rl = assess["reliable"].cpu().numpy() if assess is not None else None
        pts = points_px.detach().cpu().numpy()
        prb = probs.detach().cpu().numpy()
        quat = poses["quat"].double().cpu().numpy()
        tvec = poses["tvec"].cpu().numpy()
        st_dev = s_t.cpu().numpy() if s_t is not None else None
        sq_dev = s_q.cpu().numpy() if s_q is not None else None
        for i, fn in enumerate(filenames):
            gt = self.ground_truth[fn]
            if st_dev is None:
                a, b = speed_score(quat[i], tvec[i], gt["quat"], gt["tvec"])
            else:
                a, b = float(st_dev[i]), float(sq_dev[i])
            self._record(fn, pts[i], prb[i], quat[i], tvec[i], a, b)
            if sg is not None:
                self.log[fn]["sigma"] = np.around(sg[i], decimals=8).tolist()
            if rl is not None:
                self.log[fn]["mean_sigma"] = float(np.around(ms[i], decimals=8))
                self.log[fn]["reliable"] = bool(rl[i])

    def summarize(self):
        """REV/datasets/speed.py:382-421, including its quirk: the "median" fields are taken of
        the already-averaged scalars, so they equal the means."""
        items = list(self.log.values())
        scores = np.asarray([it["score"] for it in items])
        tvec_score = np.asarray([it["score_tvec"] for it in items])
        quat_score = np.asarray([it["score_quat"] for it in items])
        tvec_abs = np.stack([np.abs(np.asarray(it["tvec_pr"]) - np.asarray(it["tvec_gt"])) for it in items])
        scores = np.mean(scores).item()
        tvec_score = np.mean(tvec_score).item()
        quat_score = np.mean(quat_score).item()
        self.stats = "tvec score: {:.6f}, quat score: {:.6f}, final score: {:.6f}; ".format(
            tvec_score, quat_score, scores)
        self.stats += "median tvec: {:.6f}, median quat: {:.6f}; ".format(
            np.median(tvec_score).item(), np.median(quat_score).item())
        tvec_abs_mean = np.mean(tvec_abs, 0).tolist()
        tvec_abs_median = np.median(tvec_abs, 0).tolist()
        self.stats += ("mean tvec abs: [{:.6f}, {:.6f}, {:.6f}], median tvec abs:"
                       "[{:.6f}, {:.6f}, {:.6f}]").format(*(tvec_abs_mean + tvec_abs_median))
        if any("reliable" in it for it in items):
            kept = [it["score"] for it in items if it.get("reliable")]
            self.stats += "; self-assessment: {:d}/{:d} reliable, final score (reliable): {}".format(
                len(kept), len(items), "{:.6f}".format(float(np.mean(kept))) if kept else "n/a")
        return self.stats
