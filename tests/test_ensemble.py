"""Multi-checkpoint ensemble front end (Multi_Mean_PoseSolver, REV/utils/speed_eval.py:42-140;
SURVEY §8f.3) and the submission writer (REV/utils/submission.py).

CPU: the restatement's numpy-reduction helpers pinned against numpy itself (pairwise sums, axis-0
float32 means, population std -- exact equality), the 3-sigma filter's known answers, label
order, and the CSV layout.  GPU: spe_ensemble_fuse == the restatement bit for bit, and the fused
batch solved by spe_pnp_batch == oracle/pnp_ref.c on the oracle's fused points.
"""
import numpy as np
import pytest

import ensemble_ref as er


def test_numpy_reductions_restated_exactly():
    rng = np.random.Generator(np.random.PCG64(1))
    for n in range(1, 41):
        d = rng.exponential(3.0, n)
        assert er.pairwise_sum(d) == np.sum(d)
        mu = er.pairwise_sum(d) / n
        assert np.sqrt(er.pairwise_sum((d - mu) ** 2) / n) == np.std(d)
    for n in range(1, 14):
        p = (rng.normal(size=(n, 2)) * 300 + 900).astype(np.float32)
        assert np.array_equal(er.mean_rows_f32(p), np.mean(p, axis=0))


def test_three_sigma_filter_known_answers():
    base = np.array([[100.0, 200.0]], np.float32)
    near = base + np.linspace(-1, 1, 11, dtype=np.float32)[:, None]
    # 11 close points + 1 far: the far one lies beyond 3 std of the distances and is dropped
    pts = np.vstack([near, [[400.0, 200.0]]]).astype(np.float32)
    assert np.allclose(er.mean_and_filter(pts), near.mean(0), atol=1e-4)
    # the rule written with numpy / scipy directly: distances (not values) against 3 std
    from scipy.spatial.distance import cdist
    rng = np.random.Generator(np.random.PCG64(4))
    for n in (3, 4, 5, 8, 13):
        for _ in range(20):
            p = (rng.normal(size=(n, 2)) * 5 + 500).astype(np.float32)
            p[0] += rng.uniform(-200, 200, 2).astype(np.float32)
            m = np.mean(p, axis=0, keepdims=True)
            d = cdist(p, m).flatten()
            keep = d < np.std(d) * 3
            assert np.array_equal(er.mean_and_filter(p), np.mean(p[keep], axis=0).flatten())
    # n < 3: mean without the filter
    assert np.array_equal(er.mean_and_filter(near[:2]), np.mean(near[:2], axis=0))
    # all coincide: std 0, no point below 3 std, the reference's np.mean of nothing is NaN
    same = np.repeat(base, 4, 0)
    with np.errstate(invalid="ignore", divide="ignore"), pytest.warns(RuntimeWarning):
        ref = np.mean(same[np.zeros(4, bool)], axis=0)
    assert np.isnan(ref).all() and np.isnan(er.mean_and_filter(same)).all()
    # equal distances on a circle around the mean: std ~0 again, empty inlier set
    ring = (base + np.array([[3, 0], [-3, 0], [0, 3], [0, -3]], np.float32)).astype(np.float32)
    m = np.mean(ring, axis=0, keepdims=True)
    d = cdist(ring, m).flatten()
    assert not (d < np.std(d) * 3).any() and np.isnan(er.mean_and_filter(ring)).all()


def test_fuse_label_order_and_background():
    C = 12
    p1 = np.zeros((3, C), np.float32); p1[0, 5] = p1[1, 11] = p1[2, 2] = 1
    p2 = np.zeros((3, C), np.float32); p2[0, 2] = p2[1, 7] = p2[2, 5] = 1
    x1 = np.array([[1, 1], [9, 9], [2, 2]], np.float32)
    x2 = np.array([[4, 4], [7, 7], [3, 3]], np.float32)
    order, fused = er.fuse([x1, x2], [p1, p2])
    assert order == [5, 2, 7]                                   # first seen: model 0 q0, q2, model 1 q1
    assert np.allclose(fused, [[2, 2], [3, 3], [7, 7]])


def test_submission_csv(tmp_path):
    from spe.submission import SubmissionWriter
    w = SubmissionWriter()
    w.append_real_test("img000002real.jpg", [1, 0, 0, 0], [0.1, 0.2, 5.0])
    w.append_test("img000009.jpg", [0.5, 0.5, 0.5, 0.5], [0, 0, 7])
    w.append_test("img000001.jpg", [0, 1, 0, 0], [1, 2, 3])
    path = w.export(str(tmp_path), suffix="t")
    rows = open(path).read().splitlines()
    assert rows == ["img000001.jpg,0,1,0,0,1,2,3", "img000009.jpg,0.5,0.5,0.5,0.5,0,0,7",
                    "img000002real.jpg,1,0,0,0,0.1,0.2,5.0"]


def _ensemble_inputs(M, B, Q=11, seed=0):
    from spe.config import Camera, world_points, project
    from spe.synthetic import random_pose
    rng = np.random.Generator(np.random.PCG64(seed))
    W = world_points()
    q, t = random_pose(rng, B)
    lm = np.stack([project(W, q[i], t[i]) for i in range(B)])
    pts = np.zeros((M, B, Q, 2), np.float32)
    prb = np.full((M, B, Q, 12), 0.01, np.float32)
    for m in range(M):
        for b in range(B):
            perm = rng.permutation(11)[:Q]
            for k in range(Q):
                lab = perm[k] if rng.random() > 0.15 else 11               # some background queries
                prb[m, b, k, lab] = 0.9
                if lab < 11:
                    pts[m, b, k] = lm[b, lab] + rng.normal(0, 2.0, 2)
                    if rng.random() < 0.1:
                        pts[m, b, k] += rng.uniform(-300, 300, 2)          # gross outlier
    return pts, prb


@pytest.mark.gpu
@pytest.mark.parametrize("M", [1, 3, 12])
def test_ensemble_fuse_hip_matches_oracle(gpu_device, M):
    import torch
    from spe.solver import Multi_Mean_PoseSolver
    pts, prb = _ensemble_inputs(M, 24, seed=M)
    s = Multi_Mean_PoseSolver()
    fp, fr = s.fuse_batch([torch.from_numpy(p).to(gpu_device) for p in pts],
                          [torch.from_numpy(r).to(gpu_device) for r in prb])
    torch.cuda.synchronize()
    rp, rr = er.fuse_batch(pts, prb)
    assert np.array_equal(fr.cpu().numpy(), rr)
    # labels whose 3-sigma inlier set is empty are NaN on both sides (frequent at M = 3: three
    # distances to their mean rarely leave one below 3 std)
    assert np.array_equal(fp.cpu().numpy(), rp, equal_nan=True)
    if M == 3:
        assert np.isnan(rp).any()


@pytest.mark.gpu
def test_ensemble_solve_matches_oracle(gpu_device):
    import torch
    import pnp_ref
    from spe.config import Camera, world_points
    from spe.solver import Multi_Mean_PoseSolver
    pts, prb = _ensemble_inputs(3, 64, seed=9)
    s = Multi_Mean_PoseSolver()
    o = s.solve_batch_multi([torch.from_numpy(p).to(gpu_device) for p in pts],
                            [torch.from_numpy(r).to(gpu_device) for r in prb])
    torch.cuda.synchronize()
    rp, rr = er.fuse_batch(pts, prb)
    assert np.isnan(rp).any(axis=(1, 2)).sum() > 8     # NaN fused points reach the solver
    ref = pnp_ref.pnp_batch(rp, rr, Camera.K, world_points(), mode=pnp_ref.MODE_RANSAC_P3P_LM, repro=25.0)
    np.testing.assert_array_equal(o["status"].cpu().numpy(), ref["status"])
    # a NaN point never reprojects within the threshold: it is never a RANSAC inlier
    np.testing.assert_array_equal(o["n_corr"].cpu().numpy(), ref["n_corr"])
    np.testing.assert_array_equal(o["inlier_mask"].cpu().numpy().astype(np.uint32), ref["inlier_mask"])
    ok = ref["status"] == 0
    assert np.abs(o["tvec"].cpu().numpy()[ok] - ref["tvec"][ok]).max() <= 1e-6 * np.abs(ref["tvec"][ok]).max()
    # NaN fused points are drawn into minimal samples like any other correspondence (OpenCV's
    # sampler does not look at values; how cv2 itself treats NaN image points is parity
    # unpinned), but a hypothesis built from one is NaN and never wins: the accepted poses are
    # finite and no NaN correspondence is in an inlier set
    assert np.isfinite(o["quat"].cpu().numpy()[ok]).all() and np.isfinite(o["tvec"].cpu().numpy()[ok]).all()
    # (the inlier mask is over correspondence slots; fused row i is correspondence i)
    mask = o["inlier_mask"].cpu().numpy().astype(np.int64)
    for b, q in zip(*np.nonzero(np.isnan(rp).any(-1))):
        assert not (mask[b] >> q) & 1
    # the reference's per-image call (numpy lists in, numpy out)
    q1, t1 = s([p[0] for p in pts], [r[0] for r in prb])
    assert np.allclose(t1, o["tvec"][0].cpu().numpy())
