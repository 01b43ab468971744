"""Parity pinned to the reference's own code for the solver front end, the sigma weights, the
ensemble fusion, the SPEED score and the evaluator.

tests/golden/solver_front_ref.npz and tests/golden/speedeval_ref.json were recorded by
oracle/gen_golden_solver_front.py, which imports REV/utils/speed_eval.py, REV/datasets/speed.py
and UNC/utils/speed_eval.py with recording stand-ins for cv2 / mathutils / PyCeres (absent here):
what SimplePoseSolver / Multi_Mean_PoseSolver / SimplePoseSolverSigma hand to
cv2.solvePnPRansac (the selected or fused correspondences, in the reference's order), the
sigma weights ceres_pnp hands to PyCeres, speed_score's outputs, and SpeedEval's log + stats.

CPU: the oracles and the host mirror against those recordings, bit for bit.
GPU (marked gpu): the HIP selection, fusion and score kernels against them.  Tolerances: every
integer / label / order output exact; selected and fused points exact (NaN included); poses
from the HIP solver on raw queries bit-identical to the same solver on the reference's selected
correspondences; score kernel |d| <= 1e-12 (s_t) / 1e-9 (s_q), as the device acos differs from
glibc's in the last bits.
"""
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN
import ensemble_ref as er
import pnp_ref

G = np.load(os.path.join(GOLDEN, "solver_front_ref.npz"))


def _sel(n, labels, obj, b):
    k = max(int(n[b]), 0)                     # n = -1: the reference raised IndexError
    return labels[b, :k].tolist(), obj[b, :k]


# ------------------------------------------------------------------------------------- CPU
def test_oracle_selection_matches_reference():
    n, lab, obj = G["sel_n"], G["sel_labels"], G["sel_obj"]
    assert (n == -1).any() and (n >= 1).sum() > 80
    for b in range(len(n)):
        labs, pts = pnp_ref.select_correspondences(G["sel_points"][b], G["sel_probs"][b])
        if n[b] == -1:                                  # the reference's IndexError
            assert labs == []
            continue
        rl, ro = _sel(n, lab, obj, b)
        assert labs == rl, b
        np.testing.assert_array_equal(pts, ro)


def test_oracle_sigma_selection_and_weights_match_reference():
    """UNC SimplePoseSolverSigma: the same selection plus each selected query's sigma; ceres_pnp's
    per-axis weights (1/(sqrt(s)+1e-6)) / sum over the inliers, computed by numpy in float32."""
    n, lab, obj, cost = G["sig_n"], G["sig_labels"], G["sig_obj"], G["sig_cost"]
    for b in range(len(n)):
        pts, probs, sig = G["sig_points"][b], G["sig_probs"][b], G["sig_sigmas"][b]
        labs, sel = pnp_ref.select_correspondences(pts, probs)
        if n[b] == -1:
            assert labs == []
            continue
        rl, ro = _sel(n, lab, obj, b)
        assert labs == rl
        np.testing.assert_array_equal(sel, ro)
        k = n[b]
        np.testing.assert_array_equal(cost[b, :k, 0], ro[:, 0].astype(np.float64))   # u (undistort stand-in: identity)
        np.testing.assert_array_equal(cost[b, :k, 2], ro[:, 1].astype(np.float64))
        # selected sigma = that of the best-score query per label
        best = [max((q for q in range(len(probs)) if probs[q].argmax() == l), key=lambda q: (probs[q, l], -q))
                for l in rl]
        s = sig[best].astype(np.float32)
        w = pnp_ref.sigma_weights_f32(s)
        np.testing.assert_array_equal(cost[b, :k, 1], w[:, 0].astype(np.float64))
        np.testing.assert_array_equal(cost[b, :k, 3], w[:, 1].astype(np.float64))


@pytest.mark.parametrize("M", [3, 5])
def test_oracle_ensemble_fusion_matches_reference(M):
    mp, mr = G[f"ens{M}_points"], G[f"ens{M}_probs"]
    n, lab, obj = G[f"ens{M}_n"], G[f"ens{M}_labels"], G[f"ens{M}_obj"]
    nan_seen = False
    for b in range(mp.shape[1]):
        order, fused = er.fuse(mp[:, b], mr[:, b])
        rl, ro = _sel(n, lab, obj, b)
        assert order == rl
        assert np.array_equal(fused, ro, equal_nan=True)
        nan_seen |= bool(np.isnan(ro).any())
    assert nan_seen or M == 5


def test_score_matches_reference():
    from spe.speed_eval import speed_score
    x, ref = G["score_in"], G["score_out"]
    for r, o in zip(x, ref):
        for f in (pnp_ref.speed_score, speed_score):
            got = np.asarray(f(r[0:4], r[4:7], r[7:11], r[11:14]), np.float64)
            assert np.array_equal(got, o, equal_nan=True), (f, r, got, o)


def _speedeval_ref():
    with open(os.path.join(GOLDEN, "speedeval_ref.json")) as f:
        return json.load(f)


class _GivenSolver:
    def __init__(self, results):
        self.results, self.i = results, 0

    def __call__(self, points, logits):
        from spe.solver import SolverError
        r = self.results[self.i]
        self.i += 1
        if r["kind"] == "index_error":
            raise IndexError("given")
        if r["kind"] == "cv2_error":
            raise SolverError("given")
        # np.asarray(mathutils quaternion): float64 holding float32 values
        return np.asarray(r["quat"], np.float32).astype(np.float64), np.asarray(r["tvec"], np.float64)


def test_speedeval_log_and_stats_match_reference():
    """spe.speed_eval.SpeedEval.update + summarize == the reference's SpeedEval on the same
    solver results: JSON-identical log (rounding, failure mapping) and the same stats string."""
    from spe.speed_eval import SpeedEval
    ref = _speedeval_ref()
    gt, res = ref["gt"], ref["results"]
    ev = SpeedEval(gt, _GivenSolver(res))
    for i in range(0, len(gt), 5):
        ev.update({gt[j]["filename"]: {"points": np.asarray(res[j]["points"], np.float32),
                                       "logits": np.asarray(res[j]["logits"], np.float32)}
                   for j in range(i, min(i + 5, len(gt)))})
    ev.summarize()
    assert json.dumps(ev.log) == json.dumps(ref["log"])
    assert ev.stats == ref["stats"]


def test_speedeval_batch_path_matches_reference():
    """The hot-path update_batch (device-style pose records, host scores) gives the same log
    and stats as the reference's per-image update."""
    import torch
    from spe.speed_eval import SpeedEval
    ref = _speedeval_ref()
    gt, res = ref["gt"], ref["results"]
    ok = [r["kind"] == "ok" for r in res]
    quat = torch.tensor([r["quat"] if o else [0.0] * 4 for r, o in zip(res, ok)], dtype=torch.float32)
    tvec = torch.tensor([r["tvec"] if o else [0.0] * 3 for r, o in zip(res, ok)], dtype=torch.float64)
    status = torch.tensor([0 if o else (1 if r["kind"] == "index_error" else 2) for r, o in zip(res, ok)],
                          dtype=torch.int32)
    ev = SpeedEval(gt, None)
    ev.update_batch([g["filename"] for g in gt], torch.tensor([r["points"] for r in res], dtype=torch.float32),
                    torch.tensor([r["logits"] for r in res], dtype=torch.float32),
                    {"quat": quat, "tvec": tvec, "status": status})
    ev.summarize()
    assert json.dumps(ev.log) == json.dumps(ref["log"])
    assert ev.stats == ref["stats"]


# ------------------------------------------------------------------------------------- GPU
def _onehot_layout(n, lab, obj, Q=11, C=12):
    """The reference's selected correspondences as solver input rows: row i = i-th correspondence
    (one-hot label), the rest background, so the solver's first-seen order is the reference's."""
    B = len(n)
    pts = np.zeros((B, Q, 2), np.float32)
    prb = np.zeros((B, Q, C), np.float32)
    prb[:, :, C - 1] = 1.0
    for b in range(B):
        for i in range(max(n[b], 0)):
            pts[b, i] = obj[b, i]
            prb[b, i] = 0.0
            prb[b, i, lab[b, i]] = 1.0
    return pts, prb


def _solve(mode, pts, probs, sig=None, repro=20.0):
    import torch
    from spe.solver import PoseSolver
    dev = torch.device("cuda:0")
    o = PoseSolver(mode=mode, repro=repro).solve_batch(
        torch.from_numpy(pts).to(dev), torch.from_numpy(probs).to(dev),
        torch.from_numpy(sig).to(dev) if sig is not None else None)
    torch.cuda.synchronize()
    return {k: v.cpu().numpy() for k, v in o.items()}


@pytest.mark.gpu
@pytest.mark.parametrize("mode", [0, 1])
def test_hip_selection_matches_reference(gpu_device, mode):
    n, lab, obj = G["sel_n"], G["sel_labels"], G["sel_obj"]
    h = _solve(mode, G["sel_points"], G["sel_probs"])
    np.testing.assert_array_equal(h["status"][n == -1], 1)            # IndexError -> status 1
    has = n > 0
    np.testing.assert_array_equal(h["n_corr"][has], n[has])
    for b in np.nonzero(has)[0]:
        np.testing.assert_array_equal(h["corr_label"][b, :n[b]], lab[b, :n[b]])
    # the selected POINTS: the raw-query solve equals the solve of the reference's selection
    p1, r1 = _onehot_layout(n, lab, obj)
    h1 = _solve(mode, p1, r1)
    for k in ("status", "n_corr", "corr_label", "inlier_mask", "quat", "tvec"):
        np.testing.assert_array_equal(h[k][has], h1[k][has], err_msg=k)


@pytest.mark.gpu
def test_hip_sigma_selection_matches_reference(gpu_device):
    """sigma-weighted EPnP-RANSAC (mode 2): raw queries + sigmas solve exactly like the
    reference's selected correspondences carrying the reference's selected sigmas."""
    n, lab, obj = G["sig_n"], G["sig_labels"], G["sig_obj"]
    pts, probs, sig = G["sig_points"], G["sig_probs"], G["sig_sigmas"]
    h = _solve(2, pts, probs, sig, 25.0)
    has = n > 0
    np.testing.assert_array_equal(h["n_corr"][has], n[has])
    p1, r1 = _onehot_layout(n, lab, obj)
    s1 = np.ones_like(p1)
    for b in np.nonzero(has)[0]:
        for i, l in enumerate(lab[b, :n[b]]):
            best = max((q for q in range(11) if probs[b, q].argmax() == l), key=lambda q: (probs[b, q, l], -q))
            s1[b, i] = sig[b, best]
    h1 = _solve(2, p1, r1, s1, 25.0)
    for k in ("status", "corr_label", "inlier_mask", "quat", "tvec"):
        np.testing.assert_array_equal(h[k][has], h1[k][has], err_msg=k)


@pytest.mark.gpu
@pytest.mark.parametrize("M", [3, 5])
def test_hip_ensemble_fusion_matches_reference(gpu_device, M):
    import torch
    from spe.solver import Multi_Mean_PoseSolver
    mp, mr = G[f"ens{M}_points"], G[f"ens{M}_probs"]
    n, lab, obj = G[f"ens{M}_n"], G[f"ens{M}_labels"], G[f"ens{M}_obj"]
    fp, fr = Multi_Mean_PoseSolver().fuse_batch([torch.from_numpy(p).to(gpu_device) for p in mp],
                                                [torch.from_numpy(r).to(gpu_device) for r in mr])
    fp, fr = fp.cpu().numpy(), fr.cpu().numpy()
    for b in range(len(n)):
        k = max(n[b], 0)
        assert np.array_equal(fp[b, :k], obj[b, :k], equal_nan=True), b
        np.testing.assert_array_equal(fr[b, :k].argmax(-1), lab[b, :k])
        assert (fr[b, k:].argmax(-1) == 11).all()


@pytest.mark.gpu
def test_hip_score_matches_reference(gpu_device):
    import torch
    from spe.speed_eval import device_speed_score
    x, ref = G["score_in"], G["score_out"]
    d = gpu_device
    s_t, s_q = device_speed_score(torch.from_numpy(x[:, 0:4].astype(np.float32)).to(d),
                                  torch.from_numpy(x[:, 4:7]).to(d), torch.from_numpy(x[:, 7:11]).to(d),
                                  torch.from_numpy(x[:, 11:14]).to(d))
    s_t, s_q = s_t.cpu().numpy(), s_q.cpu().numpy()
    # the kernel takes the solver's float32 quaternion: compare with the reference on that input
    from spe.speed_eval import speed_score
    for i, r in enumerate(x):
        a, b = speed_score(r[0:4].astype(np.float32), r[4:7], r[7:11], r[11:14])
        assert np.isnan(s_t[i]) == np.isnan(a) and np.isnan(s_q[i]) == np.isnan(b), i
        if not np.isnan(a):
            assert abs(s_t[i] - a) <= 1e-12
        if not np.isnan(b):
            assert abs(s_q[i] - b) <= 1e-9


# ------------------------------------------------------------------ EPnPCeresSolver (a18, UNC)
def _ceres_inputs():
    th = np.array([pnp_ref.repro_th(a) for a in G["ceres_area"]], np.float32)
    return G["ceres_points"], G["ceres_probs"], G["ceres_sigmas"], th


def test_oracle_epnp_ceres_matches_reference():
    """UNC EPnPCeresSolver.__call__ run by oracle/gen_golden_solver_front.py through to its return
    value (the reference's own control flow: area threshold, selection, inliers err < th, sigma
    weights over the inliers, Huber 0.001, revert-if-worse; OpenCV / PyCeres / mathutils as the
    oracle's primitives) against oracle/pnp_ref.c's mode 4: thresholds, statuses, inlier sets and
    poses identical."""
    pts, probs, sig, th = _ceres_inputs()
    ok = G["ceres_status"] == 0
    np.testing.assert_array_equal(th[np.isfinite(G["ceres_th"])], G["ceres_th"][np.isfinite(G["ceres_th"])])
    assert set(np.unique(th)) >= {1.5, 20.0} and ok.sum() > 60 and G["ceres_reverted"].sum() > 5
    K, W = pnp_ref_K()
    o = pnp_ref.pnp_batch(pts, probs, K, W, mode=pnp_ref.MODE_EPNP_CERES, sigmas=sig, repro_per_image=th)
    np.testing.assert_array_equal(o["status"], G["ceres_status"])
    has = G["ceres_n"] > 0
    np.testing.assert_array_equal(o["n_corr"][has], G["ceres_n"][has])
    for b in np.nonzero(has)[0]:
        np.testing.assert_array_equal(o["corr_label"][b, :G["ceres_n"][b]], G["ceres_labels"][b, :G["ceres_n"][b]])
    lm = ok & (G["ceres_lm_ran"] == 1)
    np.testing.assert_array_equal(o["inlier_mask"][lm], G["ceres_inliers"][lm])
    np.testing.assert_array_equal(o["tvec"][ok], G["ceres_tvec"][ok])
    np.testing.assert_array_equal(o["quat"][ok], G["ceres_quat"][ok])


def pnp_ref_K():
    from spe.config import Camera, world_points
    return Camera.K, world_points()


def test_host_repro_th_matches_reference():
    """spe.solver.EPnPCeresSolver.get_repro_th == the thresholds the reference computed."""
    from spe.solver import EPnPCeresSolver
    s = EPnPCeresSolver()
    fin = np.isfinite(G["ceres_th"])
    got = np.array([s.get_repro_th(a) for a in G["ceres_area"]])
    np.testing.assert_array_equal(got[fin], G["ceres_th"][fin])


@pytest.mark.gpu
def test_hip_epnp_ceres_matches_reference(gpu_device):
    """The HIP solver's mode 4 (EPnPCeresSolver) on raw queries + sigmas + per-image area
    thresholds against the reference's recorded run: statuses (IndexError / cv2.error mapping),
    selection, inlier sets exact; poses |dq| <= 1e-5, |dt|/|t| <= 1e-6 (the fp64 LM of the device
    and of the oracle primitives the recording used)."""
    import torch
    from spe.solver import EPnPCeresSolver
    pts, probs, sig, th = _ceres_inputs()
    d = gpu_device
    o = EPnPCeresSolver().solve_batch(torch.from_numpy(pts).to(d), torch.from_numpy(probs).to(d),
                                      torch.from_numpy(sig).to(d), area=G["ceres_area"])
    torch.cuda.synchronize()
    o = {k: v.cpu().numpy() for k, v in o.items()}
    np.testing.assert_array_equal(o["status"], G["ceres_status"])
    has = G["ceres_n"] > 0
    np.testing.assert_array_equal(o["n_corr"][has], G["ceres_n"][has])
    for b in np.nonzero(has)[0]:
        np.testing.assert_array_equal(o["corr_label"][b, :G["ceres_n"][b]], G["ceres_labels"][b, :G["ceres_n"][b]])
    ok = G["ceres_status"] == 0
    lm = ok & (G["ceres_lm_ran"] == 1)
    np.testing.assert_array_equal(o["inlier_mask"][lm].astype(np.uint32), G["ceres_inliers"][lm])
    dq = np.abs(o["quat"][ok].astype(np.float64) - G["ceres_quat"][ok]).max()
    dt = (np.linalg.norm(o["tvec"][ok] - G["ceres_tvec"][ok], axis=1) / np.linalg.norm(G["ceres_tvec"][ok], axis=1)).max()
    assert dq <= 1e-5 and dt <= 1e-6, (dq, dt)
