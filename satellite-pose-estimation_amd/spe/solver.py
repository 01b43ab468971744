"""Pose solvers with the reference's interface (REV/utils/speed_eval.py:21-242,
UNC/utils/speed_eval.py:322-420, UNC/utils/speed_eval_ceres.py:43-169), executed by the
batched HIP solver kernel (csrc/pnp.hip) through spe_pnp_batch.

    solver = build_solver(args)                 # args.repro (20), args.solver
    quat, tvec = solver(points, logits)         # one image, numpy, like the reference
    poses = solver.solve_batch(points_px, probs) # whole batch on device (hot path)

Failures raise exactly what the reference raises so SpeedEval.update maps them to a zero
pose: IndexError when no foreground label survives, SolverError (the cv2.error stand-in)
when OpenCV would assert (fewer than 4 correspondences) or leave its output undefined.
"""
from __future__ import annotations

import numpy as np
import torch

from . import _lib
from .config import Camera, world_points

MODES = {"epnp": _lib.SPE_PNP_EPNP, "ransac_p3p_lm": _lib.SPE_PNP_RANSAC_P3P_LM,
         "epnp_ransac_sigma": _lib.SPE_PNP_EPNP_RANSAC_SIGMA, "epnp_lm": _lib.SPE_PNP_EPNP_LM,
         "epnp_ceres": _lib.SPE_PNP_EPNP_CERES}


class SolverError(RuntimeError):
    """Raised where the reference's cv2 call raises cv2.error."""


class PoseSolver:
    """Holds the 11 world landmarks (REV/utils/speed_eval.py:28-39) and camera K."""

    def __init__(self, mode=_lib.SPE_PNP_RANSAC_P3P_LM, repro=20.0, ransac_iters=100, confidence=0.99):
        self.W_Pt = world_points()
        self.K = Camera.K.copy()
        self.mode = mode
        self.reprojectionError = float(repro)
        self.ransac_iters = int(ransac_iters)
        self.confidence = float(confidence)
        self._dev = {}

    def _consts(self, device):
        key = str(device)
        if key not in self._dev:
            self._dev[key] = (torch.as_tensor(self.K, dtype=torch.float64, device=device).contiguous(),
                              torch.as_tensor(self.W_Pt, dtype=torch.float64, device=device).contiguous())
        return self._dev[key]

    def solve_batch(self, points_px, probs, sigmas=None, stream=None, out=None, repro_per_image=None):
        """points_px [B,Q,2], probs [B,Q,C] (+ sigmas [B,Q,2]) device fp32 -> dict of device
        tensors quat [B,4] f32, tvec [B,3] f64, rvec, status, n_corr, corr_label [B,16],
        inlier_mask [B].  repro_per_image: device fp32 [B] thresholds replacing
        reprojectionError image by image (EPnPCeresSolver)."""
        B, Q, C = probs.shape
        dev = probs.device
        Kd, Wd = self._consts(dev)
        if out is None:
            out = dict(quat=torch.empty(B, 4, device=dev), tvec=torch.empty(B, 3, dtype=torch.float64, device=dev),
                       rvec=torch.empty(B, 3, dtype=torch.float64, device=dev),
                       status=torch.empty(B, dtype=torch.int32, device=dev),
                       n_corr=torch.empty(B, dtype=torch.int32, device=dev),
                       corr_label=torch.empty(B, 16, dtype=torch.int32, device=dev),
                       inlier_mask=torch.empty(B, dtype=torch.int32, device=dev))
        _lib.check(_lib.lib().spe_pnp_batch(
            _lib.stream_ptr(stream), _lib.ptr(points_px.contiguous()), _lib.ptr(probs.contiguous()),
            _lib.ptr(sigmas.contiguous() if sigmas is not None else None), B, Q, C, _lib.ptr(Kd), _lib.ptr(Wd),
            self.mode, self.reprojectionError, self.ransac_iters, self.confidence, _lib.ptr(out["quat"]),
            _lib.ptr(out["tvec"]), _lib.ptr(out["rvec"]), _lib.ptr(out["status"]), _lib.ptr(out["n_corr"]),
            _lib.ptr(out["corr_label"]), _lib.ptr(out["inlier_mask"]),
            _lib.ptr(repro_per_image.float().contiguous() if repro_per_image is not None else None)), "spe_pnp_batch")
        return out

    def self_assess(self, probs, sigmas, poses, score_th=0.5, sigma_th=5.0, min_inliers=4, stream=None):
        """Self-assessment filter over a solve_batch result (BASELINE config 4; definition and
        its unpinned status: include/spe.h spe_self_assess, after the commented gate of
        UNC/utils/speed_eval_ceres.py:110-114).  Returns device tensors mean_sigma [B] f32,
        n_confident [B] i32, reliable [B] bool."""
        B, Q, C = probs.shape
        dev = probs.device
        out = dict(mean_sigma=torch.empty(B, device=dev), n_confident=torch.empty(B, dtype=torch.int32, device=dev),
                   reliable=torch.empty(B, dtype=torch.uint8, device=dev))
        _lib.check(_lib.lib().spe_self_assess(
            _lib.stream_ptr(stream), _lib.ptr(probs.contiguous()), _lib.ptr(sigmas.contiguous()),
            _lib.ptr(poses["status"]), _lib.ptr(poses["corr_label"]), _lib.ptr(poses["inlier_mask"]), B, Q, C,
            float(score_th), float(sigma_th), int(min_inliers), _lib.ptr(out["mean_sigma"]),
            _lib.ptr(out["n_confident"]), _lib.ptr(out["reliable"])), "spe_self_assess")
        out["reliable"] = out["reliable"].bool()
        return out

    def find_index(self, logits):
        return logits.argmax(1), logits.max(1)

    def __call__(self, points, logits, sigmas=None, device=None):
        """One image, numpy in / numpy out (REV/utils/speed_eval.py:164-242)."""
        points = np.asarray(points, dtype=np.float32)
        logits = np.asarray(logits, dtype=np.float32)
        assert points.shape[0] == logits.shape[0], "[Solver]: num_queries!"
        dev = device or torch.device("cuda")
        p = torch.from_numpy(points[None].copy()).to(dev)
        l = torch.from_numpy(logits[None].copy()).to(dev)
        s = torch.from_numpy(np.asarray(sigmas, np.float32)[None].copy()).to(dev) if sigmas is not None else None
        o = self.solve_batch(p, l, s)
        st = int(o["status"][0].item())
        if st == _lib.SPE_PNP_NO_FG:
            raise IndexError("no foreground keypoint")
        if st in (_lib.SPE_PNP_CV_ERROR, _lib.SPE_PNP_UNPINNED):
            raise SolverError(f"solver status {st}")
        return o["quat"][0].double().cpu().numpy(), o["tvec"][0].cpu().numpy()


class SimplePoseSolver(PoseSolver):
    """cv2.solvePnPRansac(P3P, reprojectionError=args.repro) + solvePnPGeneric(ITERATIVE)
    (REV/utils/speed_eval.py:143-242)."""

    def __init__(self, args=None):
        super().__init__(_lib.SPE_PNP_RANSAC_P3P_LM, getattr(args, "repro", 20) if args is not None else 20)


class SimplePoseSolverSigma(PoseSolver):
    """EPnP-RANSAC (reprojection 25) + sigma-weighted Huber LM (UNC/utils/speed_eval.py:322-420)."""

    def __init__(self, args=None):
        super().__init__(_lib.SPE_PNP_EPNP_RANSAC_SIGMA, 25.0)


class EPnPSolver(PoseSolver):
    """solvePnPGeneric(EPNP) on all selected points (UNC/utils/speed_eval_ceres.py:153-169, epnp_init);
    BASELINE config 2 ("EPnP only, no RANSAC").  inlier_mask: epnp_init's set, reprojection error
    < reprojectionError."""

    def __init__(self, args=None, refine=False):
        super().__init__(_lib.SPE_PNP_EPNP_LM if refine else _lib.SPE_PNP_EPNP, 20.0)


class EPnPCeresSolver(PoseSolver):
    """UNC EPnPCeresSolver (UNC/utils/speed_eval_ceres.py:43-243): EPnP on every selected point,
    inliers = reprojection error < the threshold of the image's box area (get_repro_th), the
    sigma-weighted Huber(0.001) LM on the inliers, and the EPnP pose kept when the refined error
    sum over all points is larger.  A batch carries one threshold per image."""

    def __init__(self, input_size=256):
        super().__init__(_lib.SPE_PNP_EPNP_CERES, 20.0)
        self.input_size = input_size

    def repro_th(self, area):
        """The threshold of one box area (UNC/utils/speed_eval_ceres.py:53-58: int() truncation, then
        [1.5, 20]) without touching the solver's state."""
        repro = int(area / self.input_size * 10)
        return float(min(max(repro, 1.5), 20))

    def get_repro_th(self, area):
        """UNC/utils/speed_eval_ceres.py:53-58: sets reprojectionError for the next __call__, as the
        reference does (its per-image call path)."""
        self.reprojectionError = self.repro_th(area)
        return self.reprojectionError

    def solve_batch(self, points_px, probs, sigmas=None, stream=None, out=None, repro_per_image=None, area=None):
        """As PoseSolver.solve_batch with one threshold per image: `area` (B box areas) or
        `repro_per_image` (device fp32 [B]) is required -- the reference has no batch-wide
        threshold for this solver (get_repro_th runs per image, :90)."""
        if repro_per_image is None:
            if area is None:
                raise ValueError("EPnPCeresSolver.solve_batch needs the per-image box areas (area=) or thresholds "
                                 "(repro_per_image=): the reference derives every image's threshold from its area")
            repro_per_image = torch.tensor([self.repro_th(float(a)) for a in area], dtype=torch.float32,
                                           device=probs.device)
        repro_per_image = repro_per_image.float().contiguous()
        o = super().solve_batch(points_px, probs, sigmas, stream=stream, out=out, repro_per_image=repro_per_image)
        # the kernel may still read the thresholds on `stream` after this returns
        if stream is not None:
            repro_per_image.record_stream(stream)
        o["repro_per_image"] = repro_per_image
        return o

    def __call__(self, points, logits, area, sigma, device=None):
        """One image, the reference's signature (:70): numpy in / numpy out."""
        self.get_repro_th(area)
        return PoseSolver.__call__(self, points, logits, sigma, device=device)


class Multi_Mean_PoseSolver(PoseSolver):
    """Multi-checkpoint ensemble (REV/utils/speed_eval.py:42-140): the M models' keypoints are
    fused per label (mean after a 3-sigma filter, first-seen label order) on the device
    (spe_ensemble_fuse) and solved like SimplePoseSolver (P3P-RANSAC + LM)."""

    def __init__(self, args=None):
        super().__init__(_lib.SPE_PNP_RANSAC_P3P_LM, getattr(args, "repro", 25) if args is not None else 25)

    def fuse_batch(self, multi_points_px, multi_probs, stream=None):
        """lists of M device tensors [B,Q,2] / [B,Q,C] -> fused points [B,C-1,2], probs [B,C-1,C]."""
        pts = torch.stack(list(multi_points_px)).float().contiguous()
        prb = torch.stack(list(multi_probs)).float().contiguous()
        M, B, Q, C = prb.shape
        fp = torch.empty(B, C - 1, 2, device=prb.device)
        fr = torch.empty(B, C - 1, C, device=prb.device)
        _lib.check(_lib.lib().spe_ensemble_fuse(_lib.stream_ptr(stream), _lib.ptr(pts), _lib.ptr(prb), M, B, Q, C,
                                                _lib.ptr(fp), _lib.ptr(fr)), "spe_ensemble_fuse")
        return fp, fr

    def solve_batch_multi(self, multi_points_px, multi_probs, stream=None):
        fp, fr = self.fuse_batch(multi_points_px, multi_probs, stream=stream)
        return self.solve_batch(fp, fr, stream=stream)

    def __call__(self, multi_points, multi_logits, device=None):
        """One image, numpy lists in / numpy out, the reference's call (gen_submission)."""
        assert isinstance(multi_points, list) and isinstance(multi_logits, list)
        assert len(multi_points) == len(multi_logits)
        dev = device or torch.device("cuda")
        mp = [torch.from_numpy(np.asarray(p, np.float32)[None].copy()).to(dev) for p in multi_points]
        ml = [torch.from_numpy(np.asarray(l, np.float32)[None].copy()).to(dev) for l in multi_logits]
        fp, fr = self.fuse_batch(mp, ml)
        return PoseSolver.__call__(self, fp[0].cpu().numpy(), fr[0].cpu().numpy(), device=dev)


def build_solver(args=None):
    """REV/utils/speed_eval.py:21-22 (SimplePoseSolver); `args.solver` selects the variant."""
    name = getattr(args, "solver", "ransac_p3p_lm") if args is not None else "ransac_p3p_lm"
    if name == "ransac_p3p_lm":
        return SimplePoseSolver(args)
    if name == "epnp_ransac_sigma":
        return SimplePoseSolverSigma(args)
    if name in ("epnp", "epnp_lm"):
        return EPnPSolver(args, refine=name == "epnp_lm")
    if name == "epnp_ceres":
        return EPnPCeresSolver(getattr(args, "input_size", 256) if args is not None else 256)
    raise ValueError(f"unknown solver {name}")
