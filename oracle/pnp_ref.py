"""ORACLE (test infrastructure only — never imported by the product path).

ctypes front-end of oracle/pnp_ref.c (the CPU restatement of the reference solver chain,
REV/utils/speed_eval.py:143-262, UNC/utils/speed_eval.py:269-420) plus numpy restatements of
the SPEED score (REV/utils/speed_eval.py:245-262) and of the per-image correspondence
selection (REV/utils/speed_eval.py:152-206), used as checkers by tests/, smoke() and the
bench's cpu_baseline leg.
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from collections import OrderedDict

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "build", "liboracle_pnp.so")
MAXN = 16

MODE_EPNP, MODE_RANSAC_P3P_LM, MODE_EPNP_RANSAC_SIGMA, MODE_EPNP_LM, MODE_EPNP_CERES = 0, 1, 2, 3, 4
ST_OK, ST_NO_FG, ST_CV_ERROR, ST_RANSAC_FALLBACK, ST_UNPINNED = 0, 1, 2, 3, 4

_lib = None


def build():
    subprocess.check_call(["make", "-s", "-C", HERE])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        _lib = ctypes.CDLL(LIB)
        P = ctypes.c_void_p
        _lib.oracle_pnp_batch.argtypes = [P, P, P, ctypes.c_int, ctypes.c_int, ctypes.c_int, P, P, ctypes.c_int,
                                          ctypes.c_float, ctypes.c_int, ctypes.c_double, P, P, P, P, P, P, P]
        _lib.oracle_repro_th.argtypes = [ctypes.c_double, ctypes.c_int]
        _lib.oracle_repro_th.restype = ctypes.c_float
        _lib.oracle_epnp.argtypes = [ctypes.c_int, P, P, P, P, P]
        _lib.oracle_project.argtypes = [ctypes.c_int, P, P, P, P, P]
        _lib.oracle_sigma_lm_core.argtypes = [ctypes.c_int, P, P, P, ctypes.c_double, P, P]
        _lib.oracle_rodrigues.argtypes = [P, P]
        _lib.oracle_blender_quat.argtypes = [P, P]
        _lib.oracle_np_sum_f32.argtypes = [P, ctypes.c_int]
        _lib.oracle_np_sum_f32.restype = ctypes.c_float
        _lib.oracle_speed_score.argtypes = [P, P, P, P, P, P]
        _lib.oracle_last_trace.argtypes = [P]
    return _lib


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p) if a is not None else None


def pnp_batch(points, probs, K, world, mode=MODE_RANSAC_P3P_LM, repro=20.0, sigmas=None, iters=100, conf=0.99,
              repro_per_image=None):
    """points [B,Q,2] px, probs [B,Q,C] -> dict(quat [B,4], tvec [B,3], status [B], n_corr [B],
    corr_label [B,16], inlier_mask [B]).  repro_per_image [B] (optional) replaces `repro` per image
    (the EPnPCeresSolver's area threshold, repro_th)."""
    points = np.ascontiguousarray(points, np.float32)
    probs = np.ascontiguousarray(probs, np.float32)
    B, Q, C = probs.shape
    sig = None if sigmas is None else np.ascontiguousarray(sigmas, np.float32)
    K = np.ascontiguousarray(K, np.float64)
    world = np.ascontiguousarray(world, np.float64)
    out = dict(quat=np.zeros((B, 4)), tvec=np.zeros((B, 3)), status=np.zeros(B, np.int32),
               n_corr=np.zeros(B, np.int32), corr_label=np.full((B, MAXN), -1, np.int32),
               inlier_mask=np.zeros(B, np.uint32))
    lib().oracle_pnp_batch(_p(points), _p(probs), _p(sig), B, Q, C, _p(K), _p(world), mode, repro, iters, conf,
                           _p(out["quat"]), _p(out["tvec"]), _p(out["status"]), _p(out["n_corr"]),
                           _p(out["corr_label"]), _p(out["inlier_mask"]),
                           _p(None if repro_per_image is None else np.ascontiguousarray(repro_per_image, np.float32)))
    return out


TRACE_FIELDS = ("epnp_err1", "epnp_err2", "epnp_err3", "epnp_pick", "epnp_calls", "ransac_best_iter",
                "ransac_inliers", "ransac_iters", "ransac_mask", "ransac_margin_point", "ransac_margin_px")


def pnp_trace(points, probs, K, world, mode=MODE_RANSAC_P3P_LM, repro=20.0, iters=100, conf=0.99):
    """Per image, the solver's discrete decisions (oracle/pnp_ref.c trace_t): the last EPnP
    solve's three beta-approximation errors and pick, the RANSAC best model's iteration, inlier
    count / mask and the point nearest the threshold.  Returns (pnp_batch result, list of dicts)."""
    points = np.ascontiguousarray(points, np.float32)
    probs = np.ascontiguousarray(probs, np.float32)
    res, tr = [], []
    for b in range(points.shape[0]):
        res.append(pnp_batch(points[b:b + 1], probs[b:b + 1], K, world, mode=mode, repro=repro, iters=iters, conf=conf))
        t = np.zeros(len(TRACE_FIELDS))
        lib().oracle_last_trace(_p(t))
        d = dict(zip(TRACE_FIELDS, t.tolist()))
        for k in ("epnp_pick", "epnp_calls", "ransac_best_iter", "ransac_inliers", "ransac_iters", "ransac_mask",
                  "ransac_margin_point"):
            d[k] = int(d[k])
        tr.append(d)
    if not res:
        return pnp_batch(points, probs, K, world, mode=mode, repro=repro, iters=iters, conf=conf), tr
    out = {k: np.concatenate([r[k] for r in res]) for k in res[0]}
    return out, tr


def repro_th(area, input_size=256):
    """EPnPCeresSolver.get_repro_th (UNC/utils/speed_eval_ceres.py:53-58)."""
    return float(lib().oracle_repro_th(float(area), int(input_size)))


def speedeval_area(bbox_xxyy):
    """UNC SpeedEval's area field as written (src/data/speed/speed_dataset.py, ground_truth
    'area'): np.sqrt((x2 - x1) * y2 - y1) -- the reference's precedence, kept."""
    x1, y1, x2, y2 = [float(v) for v in bbox_xxyy]
    return float(np.sqrt((x2 - x1) * y2 - y1))


def epnp(wld, img, K):
    wld = np.ascontiguousarray(wld, np.float32).reshape(-1, 3)
    img = np.ascontiguousarray(img, np.float32).reshape(-1, 2)
    r, t = np.zeros(3), np.zeros(3)
    lib().oracle_epnp(len(wld), _p(wld), _p(img), _p(np.ascontiguousarray(K, np.float64)), _p(r), _p(t))
    return r, t


def project(wld, rvec, tvec, K):
    wld = np.ascontiguousarray(wld, np.float32).reshape(-1, 3)
    uv = np.zeros((len(wld), 2), np.float32)
    lib().oracle_project(len(wld), _p(wld), _p(np.ascontiguousarray(rvec, np.float64).reshape(3)),
                         _p(np.ascontiguousarray(tvec, np.float64).reshape(3)), _p(np.ascontiguousarray(K, np.float64)),
                         _p(uv))
    return uv


def sigma_lm_core(wld, xn, w, delta, rvec, tvec):
    """The sigma-weighted Huber LM on normalised observations xn [n,2] with row weights w [n,2]."""
    wld = np.ascontiguousarray(wld, np.float64).reshape(-1, 3)
    r = np.array(rvec, np.float64).reshape(3).copy()
    t = np.array(tvec, np.float64).reshape(3).copy()
    lib().oracle_sigma_lm_core(len(wld), _p(wld), _p(np.ascontiguousarray(xn, np.float64).reshape(-1)),
                               _p(np.ascontiguousarray(w, np.float64).reshape(-1)), float(delta), _p(r), _p(t))
    return r, t


def rodrigues(rvec):
    R = np.zeros(9)
    lib().oracle_rodrigues(_p(np.ascontiguousarray(rvec, np.float64).reshape(3)), _p(R))
    return R.reshape(3, 3)


def blender_quat(R):
    q = np.zeros(4, np.float32)
    lib().oracle_blender_quat(_p(np.ascontiguousarray(R, np.float64).reshape(9)), _p(q))
    return q


def speed_score(q_pr, t_pr, q_gt, t_gt):
    """numpy restatement of REV/utils/speed_eval.py:245-262."""
    q_pr = np.asarray(q_pr, np.float64).flatten()
    t_pr = np.asarray(t_pr, np.float64).flatten()
    q_gt = np.asarray(q_gt, np.float64).flatten()
    t_gt = np.asarray(t_gt, np.float64).flatten()
    if q_pr[0] < 0:
        q_pr = -q_pr
    if q_gt[0] < 0:
        q_gt = -q_gt
    s_t = np.linalg.norm(t_pr - t_gt) / np.linalg.norm(t_gt)
    s_q = 2 * np.arccos(min(np.abs(np.dot(q_pr, q_gt)), 1))
    return s_t, s_q


def select_correspondences(points, probs):
    """REV/utils/speed_eval.py:152-206: label = argmax, drop no-object, best-score query per
    label, first-seen label order.  Returns (labels[list], points float32 [n,2])."""
    labels = probs.argmax(1)
    scores = probs.max(1)
    P = OrderedDict()
    for q in range(len(labels)):
        lab = int(labels[q])
        if lab == probs.shape[1] - 1:
            continue
        P.setdefault(lab, []).append((points[q, 0], points[q, 1], scores[q]))
    labs, pts = [], []
    for lab, lst in P.items():
        arr = np.asarray(lst)
        best = arr[:, -1].argmax()
        labs.append(lab)
        pts.append(arr[best, :2])
    return labs, np.asarray(pts, np.float32).reshape(-1, 2)


def sigma_weights_f32(sig):
    """UNC/utils/speed_eval.py:283-288 (ceres_pnp) on the selected float32 sigmas [n, 2]: numpy
    float32 sqrt, + 1e-6 and 1 / x, the axis-0 sum accumulated row by row in float32, the
    division in float32.  (oracle/pnp_ref.c sigma_lm and the HIP solver compute the same.)"""
    s = np.asarray(sig, np.float32)
    w1 = (np.float32(1.0) / (np.sqrt(s) + np.float32(1e-6))).astype(np.float32)
    tot = np.zeros(2, np.float32)
    for row in w1:
        tot = (tot + row).astype(np.float32)
    return (w1 / tot).astype(np.float32)


def self_assess(probs, sigmas, status, corr_label, inlier_mask, score_th=0.5, sigma_th=5.0, min_inliers=4):
    """Self-assessment filter (BASELINE config 4).  No reference code exists (parity unpinned):
    the rule restates include/spe.h spe_self_assess, built on the commented per-keypoint gate
    `s_ > 0.5 and sig.mean() < 5` of UNC/utils/speed_eval_ceres.py:110-114 and on the
    reference's selection (best-score query per label, REV/utils/speed_eval.py:152-200).
    Per image: (mean_sigma f32, n_confident int, reliable bool)."""
    B, Q, C = probs.shape
    ms = np.zeros(B, np.float32)
    nc = np.zeros(B, np.int32)
    rel = np.zeros(B, bool)
    for b in range(B):
        best_q, best_s = {}, {}
        for q in range(Q):
            lab = int(probs[b, q].argmax())
            if lab == C - 1:
                continue
            sc = probs[b, q, lab]
            if lab not in best_q or sc > best_s[lab]:
                best_q[lab], best_s[lab] = q, sc
        inl = int(inlier_mask[b]) & 0xFFFFFFFF if int(status[b]) in (ST_OK, ST_RANSAC_FALLBACK) else 0
        ssum, n, conf = np.float32(0), 0, 0
        for j in range(MAXN):
            if not (inl >> j) & 1:
                continue
            lab = int(corr_label[b, j])
            if lab < 0 or lab not in best_q:
                continue
            sx, sy = sigmas[b, best_q[lab]].astype(np.float32)
            ssum = np.float32(ssum + np.float32(sx + sy))
            n += 1
            if best_s[lab] > np.float32(score_th) and np.float32(0.5) * np.float32(sx + sy) < np.float32(sigma_th):
                conf += 1
        ms[b] = np.float32(ssum / np.float32(2 * n)) if n else np.float32(np.inf)
        nc[b] = conf
        rel[b] = n > 0 and conf >= min_inliers and ms[b] < np.float32(sigma_th)
    return ms, nc, rel
