"""Golden-vector generator for the solver front end, the ensemble fusion, the SPEED score and the
evaluator (SURVEY §8a rows a14, a18 selection, a19; §8f.3).  Runs ONLY in the build container,
where /root/reference exists.

The reference modules that hold these pieces import third-party packages absent here (cv2,
mathutils, PyCeres, albumentations): REV/utils/speed_eval.py, REV/datasets/speed.py,
UNC/utils/speed_eval.py.  Their own code for the pieces below is pure numpy/scipy, so they are
imported with recording stand-ins for those packages and run on seeded inputs:

  * selection  SimplePoseSolver.__call__ (REV/utils/speed_eval.py:164-206): the stand-in
               cv2.solvePnPRansac records the (wld_pts, obj_pts) it is handed -- the selected
               correspondences in the reference's order -- and raises cv2.error; an empty
               selection raises the reference's own IndexError (:203-206)
  * ensemble   Multi_Mean_PoseSolver.__call__ (:78-101, mean_and_filter :59-76): the fused
               points in first-seen label order, as handed to solvePnPRansac
  * sigma      SimplePoseSolverSigma.__call__ (UNC/utils/speed_eval.py:332-420) + ceres_pnp
               (:269-319): the stand-in solvePnPRansac records the selection and reports every
               correspondence an inlier; the stand-in cv2.undistortPoints returns its input and
               PyCeres.CreatePnPCostFunction records (u, w_u, v, w_v, X, Y, Z, 1, 0) per point, i.e.
               the selected points and the reference's sigma weights (1/(sqrt(s)+1e-6)) / sum;
               PyCeres.Solve then aborts the call
  * ceres      EPnPCeresSolver.__call__ (UNC/utils/speed_eval_ceres.py:43-169, ceres_pnp :172-243)
               run through to its return value: the stand-ins cv2.solvePnPGeneric(EPNP),
               cv2.projectPoints, cv2.undistortPoints, cv2.Rodrigues, PyCeres.Solve (the sigma LM on
               the recorded cost-function arguments, written into `camera` in place) and
               mathutils.Matrix.to_quaternion are the oracle's restated primitives (oracle/pnp_ref.c);
               the reference's own code supplies the area threshold (get_repro_th), the selection,
               the inlier set err < th, the sigma normalisation over the inliers, the HuberLoss
               scale and the revert-if-worse rule.  The module reads world_pt_path at import and
               predates numpy 1.24's ragged-array error: its `open` is pointed at the reference's
               all_result.json and its np.asarray falls back to dtype=object on ragged input, as
               numpy 1.19-1.23 did
  * score      speed_score (REV/utils/speed_eval.py:245-262) on sign-flip, zero-pose, NaN and
               |dot| > 1 cases
  * evaluator  SpeedEval.update / summarize (REV/datasets/speed.py:337-421) with a solver that
               returns given poses or raises IndexError / cv2.error: the log and stats string

Nothing from the reference is written except these numeric outputs:
  tests/golden/solver_front_ref.npz, tests/golden/speedeval_ref.json
Usage: python oracle/gen_golden_solver_front.py
"""
from __future__ import annotations

import importlib.util
import json
import os
import shutil
import sys
import tempfile
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
REF = "/root/reference"
REV = os.path.join(REF, "Revisiting Monocular Satellite Pose Estimation With Transformer")
UNC = os.path.join(REF, "Monocular Satellite Pose Estimation Based on Uncertainty Estimation and Self-Assessment")
sys.path.insert(0, os.path.join(REPO, "satellite-pose-estimation_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))

REC = {"ransac": [], "cost": [], "mode": "abort", "generic": [], "solve": []}


class _Abort(Exception):
    pass


def _stub_modules():
    cv2 = types.ModuleType("cv2")
    cv2.error = type("error", (Exception,), {})
    cv2.SOLVEPNP_ITERATIVE, cv2.SOLVEPNP_EPNP, cv2.SOLVEPNP_P3P = 0, 1, 2
    cv2.INTER_CUBIC, cv2.BORDER_CONSTANT = 2, 0

    def solvePnPRansac(wld, obj, K, dist, useExtrinsicGuess=False, flags=0, reprojectionError=8.0):
        REC["ransac"].append({"wld": np.array(wld), "obj": np.array(obj), "flags": flags,
                              "repro": float(reprojectionError)})
        if REC["mode"] == "abort":
            raise cv2.error("recorded by the generator's stand-in")
        n = len(obj)
        return True, np.zeros((3, 1)), np.array([[0.0], [0.0], [10.0]]), np.arange(n, dtype=np.int32)[:, None]

    cv2.solvePnPRansac = solvePnPRansac

    def undistortPoints(pts, K, dist):
        if REC["mode"] != "ceres":
            return np.array(pts)
        # zero distortion: ((u - cx) / fx, (v - cy) / fy) in double, stored in the input's float32
        p = np.asarray(pts, np.float64).reshape(-1, 2)
        x = (p[:, 0] - K[0, 2]) * (1.0 / K[0, 0])
        y = (p[:, 1] - K[1, 2]) * (1.0 / K[1, 1])
        return np.stack([x, y], 1).astype(np.asarray(pts).dtype).reshape(np.shape(pts))

    def solvePnPGeneric(wld, obj, K, dist, flags=0):
        import pnp_ref
        assert flags == cv2.SOLVEPNP_EPNP
        if len(obj) < 4:                        # CV_Assert(npoints >= 4) in solvePnPGeneric
            REC["generic"].append({"wld": np.array(wld), "obj": np.array(obj), "r": None, "t": None})
            raise cv2.error("EPnP needs >= 4 points")
        r, t = pnp_ref.epnp(np.asarray(wld, np.float32), np.asarray(obj, np.float32), K)
        REC["generic"].append({"wld": np.array(wld), "obj": np.array(obj), "r": r.copy(), "t": t.copy()})
        return 1, (r.reshape(3, 1),), (t.reshape(3, 1),), np.zeros((1, 1))

    def projectPoints(wld, r, t, K, dist):
        import pnp_ref
        uv = pnp_ref.project(np.asarray(wld, np.float32).reshape(-1, 3), np.asarray(r, np.float64).reshape(3),
                             np.asarray(t, np.float64).reshape(3), K)
        return uv.reshape(-1, 1, 2), None

    def Rodrigues(r):
        import pnp_ref
        return pnp_ref.rodrigues(np.asarray(r, np.float64).reshape(3)), None

    cv2.undistortPoints = undistortPoints
    cv2.solvePnPGeneric, cv2.projectPoints, cv2.Rodrigues = solvePnPGeneric, projectPoints, Rodrigues
    sys.modules["cv2"] = cv2

    mu = types.ModuleType("mathutils")

    class Matrix:
        def __init__(self, R):
            self.R = np.asarray(R, np.float64)

        def to_quaternion(self):
            import pnp_ref
            return [float(v) for v in pnp_ref.blender_quat(self.R)]   # Blender's float32 components

    mu.Matrix = Matrix
    mu.Quaternion = lambda *a, **k: None
    sys.modules["mathutils"] = mu

    pc = types.ModuleType("PyCeres")

    class Problem:
        def __init__(self):
            self.costs, self.loss, self.camera = [], None, None

        def AddResidualBlock(self, cost, loss, camera):
            REC["cost"][-1].append(cost)
            self.costs.append(cost)
            self.loss, self.camera = loss, camera

    def Solve(options, problem, summary):
        if REC["mode"] != "ceres":
            raise _Abort()
        import pnp_ref
        if not problem.costs:                  # an empty problem leaves the camera as it is
            REC["solve"].append(None)
            return
        c = np.asarray(problem.costs, np.float64)          # (x, wx, y, wy, X, Y, Z) per residual
        cam = problem.camera
        r, t = pnp_ref.sigma_lm_core(c[:, 4:7], c[:, [0, 2]], c[:, [1, 3]], problem.loss[1], cam[:3], cam[3:])
        cam[:3], cam[3:] = r, t
        REC["solve"].append({"delta": problem.loss[1], "max_iter": options.max_num_iterations,
                             "camera": cam.copy()})

    pc.Problem, pc.Solve = Problem, Solve
    pc.HuberLoss = lambda s: ("huber", s)
    pc.CreatePnPCostFunction = lambda *a: tuple(float(x) for x in a)
    pc.SolverOptions = lambda: types.SimpleNamespace()
    pc.LinearSolverType = types.SimpleNamespace(DENSE_QR=0)
    pc.Summary = lambda: None
    sys.modules["PyCeres"] = pc

    alb = types.ModuleType("albumentations")
    alb.__getattr__ = lambda name: (lambda *a, **k: None)
    sys.modules["albumentations"] = alb
    tv = types.ModuleType("torchvision")
    tv.__path__ = []
    tvt = types.ModuleType("torchvision.transforms")
    tvt.__path__ = []
    tvf = types.ModuleType("torchvision.transforms.functional")
    tv.transforms, tvt.functional = tvt, tvf
    sys.modules.update({"torchvision": tv, "torchvision.transforms": tvt, "torchvision.transforms.functional": tvf})


def _load(name, path):
    spec = importlib.util.spec_from_file_location(name, path)
    m = importlib.util.module_from_spec(spec)
    sys.modules[name] = m
    spec.loader.exec_module(m)
    return m


def _import_rev():
    """REV's utils.utils / utils.speed_eval / datasets.speed under their own package names
    (the container's HuggingFace `datasets` would shadow REV/datasets)."""
    for k in [k for k in sys.modules if k in ("utils", "datasets") or k.startswith(("utils.", "datasets."))]:
        del sys.modules[k]
    for pkg in ("utils", "datasets"):
        p = types.ModuleType(pkg)
        p.__path__ = [os.path.join(REV, pkg)]
        sys.modules[pkg] = p
    uu = _load("utils.utils", os.path.join(REV, "utils", "utils.py"))
    se = _load("utils.speed_eval", os.path.join(REV, "utils", "speed_eval.py"))
    ds = _load("datasets.speed", os.path.join(REV, "datasets", "speed.py"))
    return uu, se, ds


def _import_unc():
    for k in [k for k in sys.modules if k == "utils" or k.startswith("utils.")]:
        del sys.modules[k]
    p = types.ModuleType("utils")
    p.__path__ = [os.path.join(UNC, "utils")]
    sys.modules["utils"] = p
    _load("utils.utils", os.path.join(UNC, "utils", "utils.py"))
    return _load("utils.speed_eval", os.path.join(UNC, "utils", "speed_eval.py"))


def _compat_numpy():
    """numpy as the reference ran it (1.19-1.23): np.asarray of a ragged nested list gives a
    dtype=object array (with a warning) instead of numpy >= 1.24's ValueError."""
    shim = types.ModuleType("numpy_compat")
    shim.__dict__.update(np.__dict__)

    def asarray(a, dtype=None, *args, **kw):
        try:
            return np.asarray(a, dtype, *args, **kw)
        except ValueError:
            if dtype is not None or not isinstance(a, (list, tuple)):
                raise
            rows = [list(r) for r in a]
            out = np.empty((len(rows), len(rows[0])), dtype=object)
            for i, r in enumerate(rows):
                for j, v in enumerate(r):
                    out[i, j] = v
            return out
    shim.asarray = asarray
    return shim


def _import_unc_ceres(world_json):
    """UNC/utils/speed_eval_ceres.py with its import-time open() of the authors' absolute path
    pointed at the reference's all_result.json and the numpy 1.19-1.23 ragged-array semantics."""
    import builtins
    path = os.path.join(UNC, "utils", "speed_eval_ceres.py")
    spec = importlib.util.spec_from_file_location("utils.speed_eval_ceres", path)
    m = importlib.util.module_from_spec(spec)
    sys.modules["utils.speed_eval_ceres"] = m

    def _open(f, *a, **k):
        if isinstance(f, str) and f.endswith("all_result.json"):
            f = world_json
        return builtins.open(f, *a, **k)
    m.open = _open
    spec.loader.exec_module(m)
    m.np = _compat_numpy()
    return m


def _label_of(wld_row, W32):
    hit = np.nonzero((W32 == np.asarray(wld_row, np.float32)).all(1))[0]
    assert len(hit) == 1
    return int(hit[0])


def _pack_selection(recs, W32, n_img, maxn=11):
    """recorded solvePnPRansac inputs -> n [B] (-1 = IndexError), labels [B,maxn], obj [B,maxn,2]."""
    n = np.full(n_img, -1, np.int32)
    lab = np.full((n_img, maxn), -1, np.int32)
    obj = np.full((n_img, maxn, 2), np.nan, np.float32)
    for i, r in enumerate(recs):
        if r is None:
            continue
        k = len(r["obj"])
        n[i] = k
        lab[i, :k] = [_label_of(w[0], W32) for w in r["wld"]]
        obj[i, :k] = r["obj"][:, 0, :]
    return n, lab, obj


def _selection_inputs(B=96, seed=0):
    """The stress set plus exact score ties between queries of one label, all-background
    images and images with 1..3 labels."""
    from helpers import solver_stress_set
    pts, probs, q, t, sig = solver_stress_set(B, seed=seed)
    rng = np.random.default_rng(seed + 1)
    for b in range(0, B, 9):            # duplicate a query's label with an identical score
        q0, q1 = rng.choice(11, 2, replace=False)
        probs[b, q1] = probs[b, q0]
        pts[b, q1] += 5.0
    probs[3, :, :] = 0.0
    probs[3, :, 11] = 1.0               # all background -> IndexError
    return pts, probs, sig


def _ensemble_inputs(M, B, seed):
    from helpers import solver_stress_set
    pts, probs, _, _, _ = solver_stress_set(B, seed=seed)
    rng = np.random.default_rng(seed)
    mp = np.stack([pts + rng.normal(0, 3.0, pts.shape).astype(np.float32) for _ in range(M)])
    mr = np.stack([probs for _ in range(M)])
    for m in range(1, M):               # models disagree on some labels
        for b in range(B):
            qq = rng.choice(11, 2, replace=False)
            mr[m, b, qq] = mr[m, b, qq[::-1]]
    mp[:, 0, 0] = mp[0, 0, 0]           # a label whose points coincide (std 0)
    return mp.astype(np.float32), mr.astype(np.float32)


def _score_inputs(seed=5):
    rng = np.random.default_rng(seed)
    N = 48
    q = rng.normal(size=(N, 4))
    qg = rng.normal(size=(N, 4))
    qg /= np.linalg.norm(qg, axis=1, keepdims=True)
    t = rng.normal(size=(N, 3)) + [0, 0, 8]
    tg = rng.normal(size=(N, 3)) + [0, 0, 8]
    q[:8] /= np.linalg.norm(q[:8], axis=1, keepdims=True)
    q[8:12] = 0.0
    t[8:12] = 0.0                       # the failure pose
    q[12:16] = qg[12:16] * 1.0000001    # |dot| slightly above 1 -> clamped
    q[16:20] = -qg[16:20]               # sign flip
    q[20, 1] = np.nan
    t[21, 2] = np.nan
    return np.concatenate([q, t, qg, tg], 1)


def main():
    import torch  # noqa: F401  (REV/datasets/speed.py imports torch)
    _stub_modules()
    tmp = tempfile.mkdtemp()
    cwd = os.getcwd()
    os.makedirs(os.path.join(tmp, "data", "annos"))
    os.makedirs(os.path.join(tmp, "data", "speed"))
    shutil.copy(os.path.join(REV, "all_result.json"), os.path.join(tmp, "data", "annos", "all_result.json"))
    os.chdir(tmp)
    try:
        uu, se, ds = _import_rev()
        import argparse
        solver = se.SimplePoseSolver(argparse.Namespace(repro=20))
        W32 = np.asarray(solver.W_Pt, np.float32)
        out = {}

        # ---- selection (a14)
        pts, probs, sig = _selection_inputs()
        recs = []
        for b in range(len(pts)):
            REC["ransac"].clear()
            try:
                solver(pts[b], probs[b])
                raise AssertionError("stand-in solvePnPRansac must raise")
            except IndexError:
                recs.append(None)
            except sys.modules["cv2"].error:
                assert REC["ransac"][0]["flags"] == 2 and REC["ransac"][0]["repro"] == 20.0
                recs.append(REC["ransac"][0])
        out.update(sel_points=pts, sel_probs=probs)
        out["sel_n"], out["sel_labels"], out["sel_obj"] = _pack_selection(recs, W32, len(pts))

        # ---- ensemble fusion (f3)
        msolver = se.Multi_Mean_PoseSolver(argparse.Namespace(repro=25))
        for M, B, seed in ((3, 48, 9), (5, 32, 10)):
            mp, mr = _ensemble_inputs(M, B, seed)
            recs = []
            for b in range(B):
                REC["ransac"].clear()
                try:
                    msolver([mp[m, b] for m in range(M)], [mr[m, b] for m in range(M)])
                except IndexError:
                    recs.append(None)
                except sys.modules["cv2"].error:
                    recs.append(REC["ransac"][0])
            out[f"ens{M}_points"], out[f"ens{M}_probs"] = mp, mr
            out[f"ens{M}_n"], out[f"ens{M}_labels"], out[f"ens{M}_obj"] = _pack_selection(recs, W32, B)

        # ---- score (a19)
        sc_in = _score_inputs()
        sc_out = np.array([se.speed_score(r[0:4], r[4:7], r[7:11], r[11:14]) for r in sc_in], np.float64)
        out.update(score_in=sc_in, score_out=sc_out)

        # ---- evaluator (a19): SpeedEval.update + summarize with given solver results
        rng = np.random.default_rng(12)
        n_ev = 24
        gt = []
        results = []
        for i in range(n_ev):
            qg = rng.normal(size=4)
            qg /= np.linalg.norm(qg)
            tg = rng.normal(size=3) + [0, 0, 9]
            gt.append({"filename": f"img{i:05d}.jpg", "q_vbs2tango": qg.tolist(), "r_Vo2To_vbs_true": tg.tolist()})
            kind = "ok" if i % 7 else ("index_error" if i % 14 else "cv2_error")
            qp = (qg + rng.normal(0, 0.02, 4)).astype(np.float32)
            tp = tg + rng.normal(0, 0.05, 3)
            results.append({"kind": kind, "quat": qp.tolist(), "tvec": tp.tolist(),
                            "points": (rng.uniform(0, 1900, (11, 2)).astype(np.float32)).tolist(),
                            "logits": (rng.dirichlet(np.ones(12), 11).astype(np.float32)).tolist()})
        with open(os.path.join(tmp, "data", "speed", "gt.json"), "w") as f:
            json.dump(gt, f)

        class GivenSolver:
            def __init__(self):
                self.i = 0

            def __call__(self, points, logits):
                r = results[self.i]
                self.i += 1
                if r["kind"] == "index_error":
                    raise IndexError("given")
                if r["kind"] == "cv2_error":
                    raise sys.modules["cv2"].error("given")
                # like SimplePoseSolver's np.asarray(mathutils quaternion): float64 of float32 values
                return np.asarray(r["quat"], np.float32).astype(np.float64), np.asarray(r["tvec"], np.float64)

        ev = ds.SpeedEval("gt.json", GivenSolver())
        for i in range(0, n_ev, 5):        # several update() calls, like evaluate's batches
            ev.update({gt[j]["filename"]: {"points": np.asarray(results[j]["points"], np.float32),
                                           "logits": np.asarray(results[j]["logits"], np.float32)}
                       for j in range(i, min(i + 5, n_ev))})
        ev.summarize()
        speedeval = {"gt": gt, "results": results, "log": ev.log, "stats": ev.stats}

        # ---- sigma selection + weights (a18, UNC)
        use = _import_unc()
        use.world_pt_path = os.path.join(tmp, "data", "annos", "all_result.json")
        ssolver = use.SimplePoseSolverSigma()
        REC["mode"] = "inliers"
        spts, sprobs, ssig = _selection_inputs(64, seed=3)
        recs, costs = [], np.full((len(spts), 11, 9), np.nan)
        for b in range(len(spts)):
            REC["ransac"].clear()
            REC["cost"].append([])
            try:
                ssolver(spts[b], sprobs[b], ssig[b])
                raise AssertionError("stand-in PyCeres.Solve must abort")
            except IndexError:
                recs.append(None)
            except _Abort:
                assert REC["ransac"][0]["flags"] == 1 and REC["ransac"][0]["repro"] == 25.0
                recs.append(REC["ransac"][0])
                c = np.asarray(REC["cost"][-1], np.float64)
                costs[b, :len(c)] = c
        out.update(sig_points=spts, sig_probs=sprobs, sig_sigmas=ssig, sig_cost=costs)
        out["sig_n"], out["sig_labels"], out["sig_obj"] = _pack_selection(recs, W32, len(spts))

        # ---- EPnPCeresSolver (a18, UNC), run through to its return value
        uc = _import_unc_ceres(os.path.join(REV, "all_result.json"))
        assert np.array_equal(uc.Camera.K, se.Camera.K)
        csolver = uc.build_epnp_sigma_solver()          # input_size 256, the module's default
        REC["mode"] = "ceres"
        cpts, cprobs, csig = _selection_inputs(96, seed=21)
        rng = np.random.default_rng(22)
        area = rng.uniform(10.0, 700.0, len(cpts))      # thresholds 1.5 .. 20 (get_repro_th)
        area[:6] = [20.0, 38.0, 40.0, 300.0, 512.0, 1e4]
        nb = len(cpts)
        c_th = np.full(nb, np.nan)
        c_status = np.zeros(nb, np.int32)               # 0 pose returned, 1 IndexError, 2 cv2.error
        c_inl = np.zeros(nb, np.uint32)
        c_quat, c_tvec = np.zeros((nb, 4)), np.zeros((nb, 3))
        c_reverted = np.zeros(nb, np.int32)
        c_lm_ran = np.zeros(nb, np.int32)
        c_cost = np.full((nb, 11, 7), np.nan)
        c_rec = []

        def c_lm_ran_b():
            return bool(REC["solve"]) and REC["solve"][0] is not None
        for b in range(nb):
            for k in ("ransac", "generic", "solve"):
                REC[k].clear()
            REC["cost"].append([])
            csolver.reprojectionError = None
            try:
                q, t = csolver(cpts[b], cprobs[b], area[b], csig[b])
                c_quat[b], c_tvec[b] = q, np.asarray(t, np.float64).reshape(3)
                c_reverted[b] = int(c_lm_ran_b() and np.array_equal(c_tvec[b], REC["generic"][0]["t"]))
            except IndexError:
                c_status[b] = 1
            except sys.modules["cv2"].error:
                c_status[b] = 2
            if csolver.reprojectionError is not None:
                c_th[b] = csolver.reprojectionError
            c_lm_ran[b] = int(len(REC["solve"]) > 0 and REC["solve"][0] is not None)
            if REC["solve"] and REC["solve"][0] is not None:
                assert REC["solve"][0]["delta"] == 0.001 and REC["solve"][0]["max_iter"] == 20
            g = REC["generic"][0] if REC["generic"] else None
            c_rec.append(g)
            cst = np.asarray(REC["cost"][-1], np.float64)
            if len(cst):
                c_cost[b, :len(cst)] = cst
                wsel = np.asarray(g["wld"], np.float32).reshape(-1, 3)
                for row in cst:                  # inlier bits over the selection order
                    hit = np.nonzero((wsel == row[4:7].astype(np.float32)).all(1))[0]
                    assert len(hit) == 1
                    c_inl[b] |= np.uint32(1 << int(hit[0]))
        out.update(ceres_points=cpts, ceres_probs=cprobs, ceres_sigmas=csig, ceres_area=area, ceres_th=c_th,
                   ceres_status=c_status, ceres_inliers=c_inl, ceres_quat=c_quat, ceres_tvec=c_tvec,
                   ceres_reverted=c_reverted, ceres_lm_ran=c_lm_ran, ceres_cost=c_cost)
        out["ceres_n"], out["ceres_labels"], out["ceres_obj"] = _pack_selection(
            [None if g is None else {"wld": g["wld"], "obj": g["obj"]} for g in c_rec], W32, nb)
    finally:
        os.chdir(cwd)
        shutil.rmtree(tmp)

    gdir = os.path.join(REPO, "tests", "golden")
    np.savez_compressed(os.path.join(gdir, "solver_front_ref.npz"), **out)
    with open(os.path.join(gdir, "speedeval_ref.json"), "w") as f:
        json.dump(speedeval, f)
    print("wrote solver_front_ref.npz", {k: v.shape for k, v in out.items()})
    print("stats:", speedeval["stats"])


if __name__ == "__main__":
    main()
