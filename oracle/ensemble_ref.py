"""ORACLE (test infrastructure only — never imported by the product path).

numpy restatement of the reference's multi-checkpoint ensemble solver front end:
Multi_Mean_PoseSolver (REV/utils/speed_eval.py:42-140, driven by gen_submission,
REV/gen_submission_multi.py:145-186):

  * per model, label = argmax of PostProcess's probabilities, background (label 11) dropped,
    points appended per label in model order then query order (a defaultdict: labels keep the
    order in which they are first seen)
  * mean_and_filter (:54-71): per label, the float32 mean of its points; with 3 or more points,
    the fp64 Euclidean distances to that mean (scipy cdist), their population std, and the
    float32 mean of the points closer than 3 std
  * the fused points, in first-seen label order, go to the same P3P-RANSAC + LM solve as
    SimplePoseSolver (:103-139)

numpy's reductions are restated operation for operation: an axis-0 mean of an [n, 2] float32
array accumulates row by row in float32 and divides in float32; np.std of the 1-D fp64
distances uses numpy's pairwise summation (sequential below 8 elements, 8 accumulators above).
When no point is closer than 3 std (every point of a label coincides, std 0, or all distances
are equal) the reference's inlier set is empty and np.mean gives a NaN point; so does this
restatement, and the NaN point then goes to the solver like the reference's.  The reference module imports
cv2/mathutils and cannot be imported here, so this restatement is pinned by the known-answer
cases in tests/test_ensemble.py only (parity unpinned against the reference code itself).
"""
from __future__ import annotations

import numpy as np


def pairwise_sum(a):
    """numpy's pairwise summation of a contiguous 1-D fp64 array (n < 128 block)."""
    a = np.asarray(a, np.float64)
    n = len(a)
    if n < 8:
        res = 0.0
        for x in a:
            res += x
        return res
    r = [a[j] for j in range(8)]
    i = 8
    while i < n - (n % 8):
        for j in range(8):
            r[j] += a[i + j]
        i += 8
    res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]))
    while i < n:
        res += a[i]
        i += 1
    return res


def mean_rows_f32(p):
    s = np.zeros(2, np.float32)
    for row in p:
        s = (s + row).astype(np.float32)
    return (s / np.float32(len(p))).astype(np.float32)


def mean_and_filter(points):
    """points: float32 [n, 2] of one label -> fused float32 [2]."""
    p = np.asarray(points, np.float32)
    m = mean_rows_f32(p)
    if len(p) < 3:
        return m
    d = np.sqrt(((p.astype(np.float64) - m.astype(np.float64)) ** 2).sum(1))
    mu = pairwise_sum(d) / len(d)
    sd = np.sqrt(pairwise_sum((d - mu) ** 2) / len(d))
    keep = d < sd * 3
    if not keep.any():
        return np.full(2, np.nan, np.float32)    # np.mean of an empty selection (module docstring)
    return mean_rows_f32(p[keep])


def fuse(multi_points, multi_probs, num_classes=12):
    """multi_points [M][Q][2], multi_probs [M][Q][C] of one image -> (labels, fused [n][2])."""
    order, pts = [], {}
    for points, probs in zip(multi_points, multi_probs):
        labels = np.asarray(probs).argmax(1)
        for q, l in enumerate(labels):
            if l == num_classes - 1:
                continue
            if l not in pts:
                order.append(int(l))
                pts[l] = []
            pts[l].append(np.asarray(points[q], np.float32))
    fused = np.array([mean_and_filter(np.vstack(pts[l])) for l in order], np.float32).reshape(-1, 2)
    return order, fused


def fuse_batch(multi_points, multi_probs, num_classes=12):
    """[M][B][Q][2], [M][B][Q][C] -> (points [B][C-1][2], one-hot probs [B][C-1][C]) in the
    layout the single-model solver selects from: row i = i-th first-seen label, rest background."""
    mp, mr = np.asarray(multi_points, np.float32), np.asarray(multi_probs, np.float32)
    M, B = mp.shape[:2]
    K = num_classes - 1
    pts = np.zeros((B, K, 2), np.float32)
    prb = np.zeros((B, K, num_classes), np.float32)
    prb[:, :, num_classes - 1] = 1.0
    for b in range(B):
        order, fused = fuse(mp[:, b], mr[:, b], num_classes)
        for i, l in enumerate(order):
            pts[b, i] = fused[i]
            prb[b, i] = 0.0
            prb[b, i, l] = 1.0
    return pts, prb
