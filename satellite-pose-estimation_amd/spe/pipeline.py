"""Whole-batch device pipeline of the evaluate() hot loop (REV/engine.py:91-123 without the
logging-only criterion): [raw frames -> validation transform (spe.datasets, optional)] ->
images -> backbone/transformer/heads + fused PostProcess -> batched PnP -> SPEED scores, all
on the device with no host round trip.  Optionally captured
into a HIP graph (torch.cuda.CUDAGraph drives hipStreamBeginCapture on ROCm): spe_forward,
spe_pnp_batch and spe_speed_score never allocate or synchronise.
"""
from __future__ import annotations

import torch

from .models import DETR
from .solver import PoseSolver
from .speed_eval import device_speed_score


class PosePipeline:
    def __init__(self, model: DETR, solver: PoseSolver, batch: int, device="cuda", use_graph: bool = False,
                 self_assess: bool = True, overlap: bool = False, raw_frames=None):
        self.model, self.solver, self.B = model, solver, batch
        self.self_assess = self_assess
        # overlap: the solver / score / self-assessment of batch i run on a second HIP stream
        # while the forward of batch i+1 runs on the caller's stream (the solver occupies one
        # wave per image, far from filling the chip, and its latency is fp64-bound).  Results of
        # a run() are then complete only after wait(out) (or a device synchronize).
        self.overlap = overlap and not use_graph
        self.solve_stream = torch.cuda.Stream(device=device) if self.overlap else None
        self.device = torch.device(device)
        S, Q = model.cfg.input_size, model.cfg.num_queries
        dev = self.device
        self.images = torch.zeros(batch, 3, S, S, device=dev)
        self.clip_bbox = torch.zeros(batch, 4, device=dev)
        self.q_gt = torch.zeros(batch, 4, dtype=torch.float64, device=dev)
        self.t_gt = torch.zeros(batch, 3, dtype=torch.float64, device=dev)
        self.q_gt[:, 0] = 1
        self.t_gt[:, 2] = 10
        model.workspace(batch, dev)
        # raw_frames = (H, W, C): each run() starts from uint8 frames + detector boxes resident in
        # HBM (load_frames) and runs the validation transform on the device first
        self.frames = self.bbox = self.transform = None
        if raw_frames is not None:
            from .datasets import SpeedValTransform
            H, W, C = raw_frames
            self.frames = torch.zeros((batch, H, W) + ((C,) if C == 3 else ()), dtype=torch.uint8, device=dev)
            self.bbox = torch.zeros(batch, 4, dtype=torch.float64, device=dev)
            self.transform = SpeedValTransform(S)
            self.pp_out = {"images": self.images, "clip_bbox": self.clip_bbox,
                           "status": torch.zeros(batch, dtype=torch.int32, device=dev)}
        self.use_graph = use_graph
        self.graph = None
        self.out = None
        _ = Q

    def _solve(self, fo, stream=None):
        sig = fo.get("sigmas")
        poses = self.solver.solve_batch(fo["points_px"], fo["probs"], sig, stream=stream)
        s_t, s_q = device_speed_score(poses["quat"], poses["tvec"], self.q_gt, self.t_gt, stream=stream)
        out = {"forward": fo, "poses": poses, "s_t": s_t, "s_q": s_q}
        if sig is not None and self.self_assess:
            out["assess"] = self.solver.self_assess(fo["probs"], sig, poses, stream=stream)   # config-4 filter
        return out

    def _body(self):
        if self.transform is not None:
            self.transform(self.frames, self.bbox, out=self.pp_out)
        fo = self.model(self.images, clip_bbox=self.clip_bbox)
        if not self.overlap:
            return self._solve(fo)
        s1 = self.solve_stream
        s1.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s1):
            for t in fo.values():
                t.record_stream(s1)          # forward outputs are consumed on the solver stream
            out = self._solve(fo, stream=s1)
        out["stream"] = s1
        return out

    def wait(self, out=None):
        """Make the caller's stream wait for a run()'s solver work (no-op without overlap)."""
        out = out if out is not None else self.out
        if out is not None and out.get("stream") is not None:
            torch.cuda.current_stream().wait_stream(out["stream"])

    def load(self, images, clip_bbox, q_gt=None, t_gt=None):
        self.images.copy_(images, non_blocking=True)
        self.clip_bbox.copy_(clip_bbox, non_blocking=True)
        if q_gt is not None:
            self.q_gt.copy_(q_gt, non_blocking=True)
            self.t_gt.copy_(t_gt, non_blocking=True)

    def load_frames(self, frames, bbox_xxyy, q_gt=None, t_gt=None):
        """Raw-frame mode: uint8 frames [B,H,W(,3)] + detector boxes [B,4] (fp64)."""
        self.frames.copy_(frames, non_blocking=True)
        self.bbox.copy_(torch.as_tensor(bbox_xxyy, dtype=torch.float64), non_blocking=True)
        if q_gt is not None:
            self.q_gt.copy_(q_gt, non_blocking=True)
            self.t_gt.copy_(t_gt, non_blocking=True)

    def run(self):
        if not self.use_graph:
            self.out = self._body()
            return self.out
        if self.graph is None:
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                self._body()                       # warm-up: allocations happen outside capture
            torch.cuda.current_stream().wait_stream(s)
            self.graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(self.graph):
                self.out = self._body()
        self.graph.replay()
        return self.out
