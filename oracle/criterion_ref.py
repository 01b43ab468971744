"""ORACLE (test infrastructure only — never imported by the product path).

numpy restatement of the reference's set criterion, the part of evaluate()
(REV/engine.py:99-112) that logs losses:

  HungarianMatcher.forward   REV/models/matcher.py:35-88: cost = set_cost_pts * cdist_L1(points,
                             target points) - set_cost_class * softmax(logits)[:, target label]
                             (fp32, torch's order), then scipy.optimize.linear_sum_assignment per
                             image on the [Q, T] matrix (fp64)
  SetCriterion.loss_labels   REV/models/detr_speed.py:129-155: weighted cross entropy over every
                             query (matched -> its target label, else no-object 11 with weight
                             eos_coef), class_error = 100 - top-1 accuracy on the matched queries
                             (last layer only)
  loss_cardinality           :157-171: mean |#queries not predicting no-object - #targets|
  loss_points                :173-189: smooth L1 (beta = 1/200, REV/utils/smooth_l1_loss.py:103-121)
                             summed over matched pairs / num_points (targets per rank, >= 1)
  forward                    :214-261: last layer plus every aux layer (suffix _i)

`lsap` restates scipy's rectangular linear-sum-assignment (shortest augmenting path, Crouse
2016, as in scipy/optimize/_lsap: rows <= columns, transposed otherwise; ties between
equal-cost columns go to a free column, else the first) and is pinned against scipy itself
(importable here and on the GPU box) in tests/test_criterion.py.  The loss values are pinned
against the reference's own SetCriterion through tests/golden/criterion_*.npz
(oracle/gen_golden_criterion.py).
"""
from __future__ import annotations

import numpy as np

NUM_CLASSES = 11          # REV/models/detr_speed.py:305 (no-object = 11)


def lsap(cost):
    """Minimum-cost assignment of an [nr, nc] matrix -> (row_ind ascending, col_ind)."""
    c = np.asarray(cost, np.float64)
    transpose = c.shape[0] > c.shape[1]
    if transpose:
        c = c.T
    nr, nc = c.shape
    u, v = np.zeros(nr), np.zeros(nc)
    col4row, row4col = np.full(nr, -1), np.full(nc, -1)
    for cur in range(nr):
        spc = np.full(nc, np.inf)
        path = np.full(nc, -1)
        sr, sc = np.zeros(nr, bool), np.zeros(nc, bool)
        remaining = list(range(nc - 1, -1, -1))
        min_val, i, sink = 0.0, cur, -1
        while sink == -1:
            sr[i] = True
            index, lowest = -1, np.inf
            for it, j in enumerate(remaining):
                r = min_val + c[i, j] - u[i] - v[j]
                if r < spc[j]:
                    path[j] = i
                    spc[j] = r
                if spc[j] < lowest or (spc[j] == lowest and row4col[j] == -1):
                    lowest, index = spc[j], it
            min_val = lowest
            if not np.isfinite(min_val):
                raise ValueError("cost matrix is infeasible")
            j = remaining[index]
            if row4col[j] == -1:
                sink = j
            else:
                i = row4col[j]
            sc[j] = True
            remaining[index] = remaining[-1]
            remaining.pop()
        u[cur] += min_val
        for r_ in range(nr):
            if sr[r_] and r_ != cur:
                u[r_] += min_val - spc[col4row[r_]]
        for j_ in range(nc):
            if sc[j_]:
                v[j_] -= min_val - spc[j_]
        j = sink
        while True:
            i = path[j]
            row4col[j] = i
            col4row[i], j = j, col4row[i]
            if i == cur:
                break
    if transpose:
        order = np.argsort(col4row, kind="stable")
        return col4row[order], np.arange(nr)[order]
    return np.arange(nr), col4row.copy()


def softmax32(x):
    x = np.asarray(x, np.float32)
    e = np.exp(x - x.max(-1, keepdims=True))
    return (e / e.sum(-1, keepdims=True)).astype(np.float32)


def match(logits, points, tgt_labels, tgt_points, cost_class=1.0, cost_pts=5.0, solver=lsap):
    """REV/models/matcher.py:60-88 for one image: [Q] query index matched to each target (-1 none)."""
    prob = softmax32(logits)
    cc = -prob[:, tgt_labels]
    cp = np.abs(points[:, None, :].astype(np.float32) - tgt_points[None, :, :].astype(np.float32)).sum(-1)
    C = (np.float32(cost_pts) * cp + np.float32(cost_class) * cc).astype(np.float32)
    qi, ti = solver(C.astype(np.float64))
    out = np.full(len(tgt_labels), -1, np.int64)
    out[ti] = qi
    return out


def smooth_l1(d, beta=1.0 / 200.0):
    d = np.abs(d)
    return np.where(d < beta, 0.5 * d * d / beta, d - 0.5 * beta)


def layer_losses(logits, points, tgt_labels, tgt_points, m, eos_coef=0.1, num_points=None, log=True):
    """Losses of one decoder layer for a batch; m [B, T] matched query per target."""
    B, Q, C = logits.shape
    T = tgt_labels.shape[1]
    tc = np.full((B, Q), NUM_CLASSES, np.int64)
    for b in range(B):
        tc[b, m[b]] = tgt_labels[b]
    lp = logits.astype(np.float64) - logits.max(-1, keepdims=True)
    lp = lp - np.log(np.exp(lp).sum(-1, keepdims=True))
    w = np.where(tc == NUM_CLASSES, eos_coef, 1.0)
    nll = -np.take_along_axis(lp, tc[..., None], -1)[..., 0]
    out = {"loss_ce": float((w * nll).sum() / w.sum())}
    if log:
        pred = logits.argmax(-1)
        matched_pred = np.concatenate([pred[b, m[b]] for b in range(B)])
        matched_tgt = np.concatenate([tgt_labels[b] for b in range(B)])
        out["class_error"] = float(100.0 - 100.0 * (matched_pred == matched_tgt).mean())
    card = (logits.argmax(-1) != C - 1).sum(1)
    out["cardinality_error"] = float(np.abs(card - T).mean())
    npts = max(float(B * T), 1.0) if num_points is None else num_points
    src = np.concatenate([points[b, m[b]] for b in range(B)]).astype(np.float64)
    tgt = np.concatenate([tgt_points[b] for b in range(B)]).astype(np.float64)
    out["loss_points"] = float(smooth_l1(src - tgt).sum() / npts)
    return out


def criterion(layers, tgt_labels, tgt_points, cost_class=1.0, cost_pts=5.0, eos_coef=0.1, solver=lsap):
    """layers: list of (logits [B,Q,C], points [B,Q,2]), aux first, last layer last.
    Returns (loss dict with the reference's keys, match [L, B, T])."""
    L = len(layers)
    B = tgt_labels.shape[0]
    losses, ms = {}, []
    for l, (lg, pt) in enumerate(layers):
        m = np.stack([match(lg[b], pt[b], tgt_labels[b], tgt_points[b], cost_class, cost_pts, solver)
                      for b in range(B)])
        ms.append(m)
        last = l == L - 1
        d = layer_losses(lg, pt, tgt_labels, tgt_points, m, eos_coef, log=last)
        losses.update(d if last else {f"{k}_{l}": v for k, v in d.items()})
    return losses, np.stack(ms)
