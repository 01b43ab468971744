"""Shared seeded cases for parity tests (SURVEY.md §8(d) solver stress set)."""
import numpy as np

from spe.config import world_points, project


def solver_stress_set(B, seed=0, Q=11, C=12, noise=2.0, outlier_frac=0.1, degenerate_frac=0.05):
    """Per image: labels a random permutation of 0..10 (+ duplicates / no-object queries), points
    = GT projection + N(0, noise px) + uniform outliers, a few images with <=3 or 0 foreground
    labels.  Returns points [B,Q,2] f32 px, probs [B,Q,C] f32, q [B,4], t [B,3], sigmas [B,Q,2]."""
    rng = np.random.default_rng(seed)
    W = world_points()
    pts = np.zeros((B, Q, 2), np.float32)
    probs = np.zeros((B, Q, C), np.float32)
    qs, ts = np.zeros((B, 4)), np.zeros((B, 3))
    sig = rng.uniform(0.5, 20.0, (B, Q, 2)).astype(np.float32)
    for b in range(B):
        q = rng.normal(size=4); q /= np.linalg.norm(q)
        t = np.array([rng.normal(0, .3), rng.normal(0, .3), rng.uniform(3, 30)])
        qs[b], ts[b] = q, t
        lm = project(W, q, t)
        labels = rng.permutation(Q) % (C - 1)
        r = rng.random()
        if r < degenerate_frac / 2:
            labels[:] = C - 1                             # no foreground
        elif r < degenerate_frac:
            keep = rng.integers(1, 4)                      # 1..3 foreground labels
            labels[keep:] = C - 1
        else:
            ndup = rng.integers(0, 3)
            for _ in range(ndup):                          # duplicated labels / dropped queries
                labels[rng.integers(Q)] = rng.integers(C)
        logits = rng.normal(0, 1, (Q, C)).astype(np.float32)
        logits[np.arange(Q), labels] += rng.uniform(3, 6, Q).astype(np.float32)
        e = np.exp(logits - logits.max(1, keepdims=True))
        probs[b] = e / e.sum(1, keepdims=True)
        p = lm[np.minimum(labels, C - 2)] + rng.normal(0, noise, (Q, 2))
        nout = rng.binomial(Q, outlier_frac)
        if nout:
            idx = rng.choice(Q, nout, replace=False)
            p[idx] += rng.uniform(-400, 400, (nout, 2))
        pts[b] = p.astype(np.float32)
    return pts, probs, qs, ts, sig
