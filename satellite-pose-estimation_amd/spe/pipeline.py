"""Whole-batch device pipeline of the evaluate() hot loop (REV/engine.py:91-123 without the
logging-only criterion): [JPEG files -> decode] -> [raw frames -> validation transform
(spe.datasets, optional)] ->
images -> backbone/transformer/heads + fused PostProcess -> batched PnP -> SPEED scores, all
on the device with no host round trip.  Optionally captured
into a HIP graph (torch.cuda.CUDAGraph drives hipStreamBeginCapture on ROCm): spe_forward,
spe_pnp_batch and spe_speed_score never allocate or synchronise.
"""
from __future__ import annotations

import torch

from . import _lib
from .models import DETR
from .solver import PoseSolver
from .speed_eval import device_speed_score


_STREAMS = {}


def pipeline_stream(device, role: str):
    """One HIP stream per (device, role) for every pipeline of the process.  A process has a few
    hardware queues (GPU_MAX_HW_QUEUES, 4 by default) that its streams are dealt onto; pipelines
    that each made their own streams (the bench times a parity and a host-input line beside the main
    one) would keep adding streams that end up sharing queues.  Pipelines on one device therefore
    share their solver / decoder / encoder / copy streams (work on them is stream-ordered, correct
    for any interleaving of the pipelines)."""
    d = torch.device(device)
    idx = d.index if d.index is not None or d.type != "cuda" else torch.cuda.current_device()
    key = (d.type, idx, role)
    st = _STREAMS.get(key)
    if st is None:
        _STREAMS[key] = st = torch.cuda.Stream(device=d)
    return st


class PosePipeline:
    def __init__(self, model: DETR, solver: PoseSolver, batch: int, device="cuda", use_graph: bool = False,
                 self_assess: bool = True, overlap: bool = False, raw_frames=None, overlap_decode: bool = False,
                 jpeg_max_bytes: int = 0, overlap_backbone: bool = False, host_input: bool = False):
        self.model, self.solver, self.B = model, solver, batch
        self.self_assess = self_assess
        # overlap: the solver / score / self-assessment of batch i run on a second HIP stream
        # while the forward of batch i+1 runs on the caller's stream (the solver occupies one
        # wave per image, far from filling the chip, and its latency is fp64-bound).  Results of
        # a run() are then complete only after wait(out) (or a device synchronize).
        # overlap_decode (implies overlap): the forward is split at the encoder memory
        # (spe_forward_stages) and batch i's decoder + heads run on a third stream beside batch
        # i+1's backbone/encoder; two workspaces alternate between in-flight batches.  The
        # decoder is ~55 launches of few-row kernels that leave most CUs idle on their own.
        # overlap_backbone (implies overlap_decode): the encode stage splits once more at the
        # encoder input (SPE_STAGE_BACKBONE / SPE_STAGE_TRANSFORMER): batch i's encoder layers run
        # on a fourth stream beside batch i+1's backbone -- the VALU-bound attention beside the
        # HBM-bound convolutions -- with three workspaces rotating between in-flight batches.
        self.overlap_decode = (overlap_decode or overlap_backbone) and not use_graph
        self.overlap_backbone = overlap_backbone and self.overlap_decode
        self.overlap = (overlap or self.overlap_decode) and not use_graph
        self.solve_stream = pipeline_stream(device, "solve") if self.overlap else None
        self.device = torch.device(device)
        S, Q = model.cfg.input_size, model.cfg.num_queries
        dev = self.device
        self.images = torch.zeros(batch, 3, S, S, device=dev)
        self.clip_bbox = torch.zeros(batch, 4, device=dev)
        self.q_gt = torch.zeros(batch, 4, dtype=torch.float64, device=dev)
        self.t_gt = torch.zeros(batch, 3, dtype=torch.float64, device=dev)
        self.q_gt[:, 0] = 1
        self.t_gt[:, 2] = 10
        # EPnPCeresSolver: one reprojection threshold per image from its box area (load(area=...))
        self.per_image_th = getattr(solver, "mode", None) == _lib.SPE_PNP_EPNP_CERES
        self.repro = torch.full((batch,), float(getattr(solver, "reprojectionError", 20.0)), device=dev)
        if not overlap_decode:
            model.workspace(batch, dev)           # sized outside any graph capture
        if self.overlap_decode:
            self.dec_stream = pipeline_stream(device, "decode")
            self.enc_stream = pipeline_stream(device, "encode") if self.overlap_backbone else None
            self.nslot = 3 if self.overlap_backbone else 2
            # the staged slots own their workspaces: a direct model(...) call or another
            # pipeline on the same model never writes into a slot's encoder memory
            self.ws2 = [model.new_workspace(batch, dev) for _ in range(self.nslot)]
            # per-slot snapshots of what the later stages read (a load() for the next batch may
            # overwrite the staging buffers while this batch's decoder / solver still run)
            self.slot_clip = [torch.zeros(batch, 4, device=dev) for _ in range(self.nslot)]
            self.slot_q = [torch.zeros(batch, 4, dtype=torch.float64, device=dev) for _ in range(self.nslot)]
            self.slot_t = [torch.zeros(batch, 3, dtype=torch.float64, device=dev) for _ in range(self.nslot)]
            self.slot_repro = [torch.zeros(batch, device=dev) for _ in range(self.nslot)]
            self.dec_done = [None] * self.nslot
            self.solve_done = [None] * self.nslot
            self.calls = 0
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
        # jpeg_max_bytes > 0 (with raw_frames = (H, W, 1)): each run() starts from the frames' JPEG
        # files in HBM (load_jpeg) and decodes them on the device first (spe.datasets.JpegDecoder)
        self.decoder = None
        if jpeg_max_bytes > 0:
            from .datasets import JpegDecoder
            H, W, C = raw_frames
            if C != 1:
                raise ValueError("JPEG input: grayscale frames (raw_frames = (H, W, 1))")
            self.decoder = JpegDecoder(H, W, jpeg_max_bytes)
            self.jpeg = None
            self.dec_out = {"frames": self.frames, "status": torch.zeros(batch, dtype=torch.int32, device=dev)}
        # host_input: each run() takes its batch from pinned host memory (load_host: the 8-bit crops
        # to_tensor + Normalize make the model input from, plus boxes / ground truth), the next B of
        # the pool in turn, as REV/engine.py:92's samples.to(device) does per batch.  The H2D copy goes
        # on its own stream into the batch's slot buffers and the backbone waits for it only; with
        # the staged overlap the copy of batch i runs under batch i-1's compute.
        self.host_input = host_input
        if host_input:
            if use_graph or raw_frames is not None:
                raise ValueError("host_input: eager, crop-level input (no graph, no raw frames)")
            n = self.nslot if self.overlap_decode else 1
            self.copy_stream = pipeline_stream(device, "copy")
            self.host = None
            self.host_next = 0
            self.dev_crops = [None] * n
            self.copied = [None] * n
            self.h2d_bytes = 0
        self.use_graph = use_graph
        self.graph = None
        self.out = None
        _ = Q

    def _solve(self, fo, stream=None, q_gt=None, t_gt=None, repro=None):
        sig = fo.get("sigmas")
        if self.per_image_th:
            poses = self.solver.solve_batch(fo["points_px"], fo["probs"], sig, stream=stream,
                                            repro_per_image=self.repro if repro is None else repro)
        else:
            poses = self.solver.solve_batch(fo["points_px"], fo["probs"], sig, stream=stream)
        q_gt = self.q_gt if q_gt is None else q_gt
        t_gt = self.t_gt if t_gt is None else t_gt
        s_t, s_q = device_speed_score(poses["quat"], poses["tvec"], q_gt, t_gt, stream=stream)
        out = {"forward": fo, "poses": poses, "s_t": s_t, "s_q": s_q}
        if sig is not None and self.self_assess:
            out["assess"] = self.solver.self_assess(fo["probs"], sig, poses, stream=stream)   # config-4 filter
        return out

    def _decode(self):
        if self.decoder is not None:
            self.decoder(*self.jpeg, out=self.dec_out)

    def _h2d(self, slot, after=()):
        """Host-input mode: copy the next pool batch (pinned) into this slot's device buffers on the
        copy stream, after the events in `after` (the slot's previous batch done with them); returns
        the copy's completion event."""
        h = self.host
        if h is None:
            raise RuntimeError("host_input pipeline: load_host() first")
        j = self.host_next
        self.host_next = (j + self.B) % h["crops"].shape[0]
        cs = self.copy_stream
        for ev in after:
            if ev is not None:
                cs.wait_event(ev)
        if self.dev_crops[slot] is None:
            self.dev_crops[slot] = torch.empty((self.B,) + tuple(h["crops"].shape[1:]), dtype=torch.uint8,
                                               device=self.device)
        clip = self.slot_clip[slot] if self.overlap_decode else self.clip_bbox
        q = self.slot_q[slot] if self.overlap_decode else self.q_gt
        t = self.slot_t[slot] if self.overlap_decode else self.t_gt
        with torch.cuda.stream(cs):
            self.dev_crops[slot].copy_(h["crops"][j:j + self.B], non_blocking=True)
            clip.copy_(h["clip"][j:j + self.B], non_blocking=True)
            q.copy_(h["q"][j:j + self.B], non_blocking=True)
            t.copy_(h["t"][j:j + self.B], non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(cs)
        self.h2d_bytes = self.dev_crops[slot].numel() + clip.numel() * 4 + (q.numel() + t.numel()) * 8
        return ev

    def load_host(self, crops, clip_bbox, q_gt, t_gt):
        """Host-input mode: the pool every run() takes its next B images from -- 8-bit crops
        [N,S,S] / [N,S,S,3], boxes [N,4], quaternions [N,4], translations [N,3] (N a multiple of
        B), kept in pinned host memory."""
        if not self.host_input:
            raise ValueError("load_host: pipeline built without host_input")
        if crops.shape[0] % self.B or crops.dtype != torch.uint8:
            raise ValueError("load_host: uint8 crops, a whole number of batches")
        self.host = {"crops": crops.contiguous().pin_memory(),
                     "clip": clip_bbox.to(torch.float32).contiguous().pin_memory(),
                     "q": q_gt.to(torch.float64).contiguous().pin_memory(),
                     "t": t_gt.to(torch.float64).contiguous().pin_memory()}
        self.copy_stream.synchronize()                 # (a prefetch of the previous pool is dropped)
        self.copied = [None] * len(self.copied)
        self.host_next = 0

    def _body_staged(self):
        main = torch.cuda.current_stream()
        slot = self.calls % self.nslot
        self.calls += 1
        self._decode()
        if self.transform is not None:
            self.transform(self.frames, self.bbox, out=self.pp_out)
        images = self.images
        if self.host_input:
            # the copy into this slot was issued one run() ahead (below); the slot's previous batch
            # (i - nslot) is done with its crops / snapshots once its decoder and solver are
            ev = self.copied[slot]
            if ev is None:
                ev = self._h2d(slot, after=(self.dec_done[slot], self.solve_done[slot]))
            self.copied[slot] = None
            main.wait_event(ev)
            images = self.dev_crops[slot]
            self.slot_repro[slot].copy_(self.repro)
        else:
            if self.dec_done[slot] is not None:
                main.wait_event(self.dec_done[slot])      # batch i-nslot's decoder is done with this workspace
            if self.solve_done[slot] is not None:
                main.wait_event(self.solve_done[slot])    # ... and its solver / score with the slot's snapshots
            self.slot_clip[slot].copy_(self.clip_bbox)
            self.slot_q[slot].copy_(self.q_gt)
            self.slot_t[slot].copy_(self.t_gt)
            self.slot_repro[slot].copy_(self.repro)
        if self.overlap_backbone:
            self.model.encode(images, self.ws2[slot], stream=main, part="backbone")
            e = self.enc_stream
            e.wait_stream(main)
            with torch.cuda.stream(e):
                self.model.encode(None, self.ws2[slot], stream=e, part="transformer", B=self.B)
        else:
            self.model.encode(images, self.ws2[slot], stream=main)
            e = main
        d = self.dec_stream
        d.wait_stream(e)
        with torch.cuda.stream(d):
            fo = self.model.decode(self.B, self.ws2[slot], clip_bbox=self.slot_clip[slot], stream=d)
            ev = torch.cuda.Event()
            ev.record(d)
            self.dec_done[slot] = ev
        s1 = self.solve_stream
        s1.wait_stream(d)
        with torch.cuda.stream(s1):
            for t in fo.values():
                t.record_stream(s1)
            out = self._solve(fo, stream=s1, q_gt=self.slot_q[slot], t_gt=self.slot_t[slot],
                              repro=self.slot_repro[slot])
            ev = torch.cuda.Event()
            ev.record(s1)
            self.solve_done[slot] = ev
        out["stream"] = s1
        if self.host_input:
            # prefetch: the next batch's H2D goes out now, under this batch's compute
            nxt = self.calls % self.nslot
            self.copied[nxt] = self._h2d(nxt, after=(self.dec_done[nxt], self.solve_done[nxt]))
        return out

    def _body(self):
        if self.overlap_decode:
            return self._body_staged()
        self._decode()
        if self.transform is not None:
            self.transform(self.frames, self.bbox, out=self.pp_out)
        images = self.images
        if self.host_input:
            # one slot: the copy waits for the previous forward (which read the crops) on this stream
            prev = torch.cuda.Event()
            prev.record(torch.cuda.current_stream())
            torch.cuda.current_stream().wait_event(self._h2d(0, after=(prev,)))
            images = self.dev_crops[0]
        fo = self.model(images, clip_bbox=self.clip_bbox)
        if not self.overlap:
            return self._solve(fo)
        s1 = self.solve_stream
        # the ground truth is snapshotted on the caller's stream: a load() of the next batch may
        # overwrite q_gt / t_gt while this batch's score still runs on the solver stream
        q_gt, t_gt, repro = self.q_gt.clone(), self.t_gt.clone(), self.repro.clone()
        s1.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s1):
            for t in list(fo.values()) + [q_gt, t_gt, repro]:
                t.record_stream(s1)          # consumed on the solver stream
            out = self._solve(fo, stream=s1, q_gt=q_gt, t_gt=t_gt, repro=repro)
        out["stream"] = s1
        return out

    def wait(self, out=None):
        """Make the caller's stream wait for a run()'s solver work (no-op without overlap)."""
        out = out if out is not None else self.out
        if out is not None and out.get("stream") is not None:
            torch.cuda.current_stream().wait_stream(out["stream"])

    def load(self, images, clip_bbox, q_gt=None, t_gt=None, area=None):
        """area (EPnPCeresSolver): the B box areas its per-image thresholds come from."""
        self.images.copy_(images, non_blocking=True)
        self.clip_bbox.copy_(clip_bbox, non_blocking=True)
        if q_gt is not None:
            self.q_gt.copy_(q_gt, non_blocking=True)
            self.t_gt.copy_(t_gt, non_blocking=True)
        self._load_area(area)

    def _load_area(self, area):
        if area is not None:
            if not self.per_image_th:
                raise ValueError("area= is the EPnPCeresSolver's threshold input; this pipeline's solver takes none")
            self.repro.copy_(torch.tensor([self.solver.repro_th(float(a)) for a in area], dtype=torch.float32))
        elif self.per_image_th:
            raise ValueError("EPnPCeresSolver pipeline: load(..., area=) needs the images' box areas")

    def load_frames(self, frames, bbox_xxyy, q_gt=None, t_gt=None, area=None):
        """Raw-frame mode: uint8 frames [B,H,W(,3)] + detector boxes [B,4] (fp64)."""
        self._load_area(area)
        self.frames.copy_(frames, non_blocking=True)
        self.bbox.copy_(torch.as_tensor(bbox_xxyy, dtype=torch.float64), non_blocking=True)
        if q_gt is not None:
            self.q_gt.copy_(q_gt, non_blocking=True)
            self.t_gt.copy_(t_gt, non_blocking=True)

    def load_jpeg(self, data, offsets, sizes, bbox_xxyy, q_gt=None, t_gt=None, area=None):
        """JPEG mode: the batch's files packed into one device byte buffer (JpegDecoder.pack; kept
        by reference, not copied) + detector boxes [B,4]."""
        self._load_area(area)
        self.jpeg = (data, offsets, sizes)
        self.bbox.copy_(torch.as_tensor(bbox_xxyy, dtype=torch.float64), non_blocking=True)
        if q_gt is not None:
            self.q_gt.copy_(q_gt, non_blocking=True)
            self.t_gt.copy_(t_gt, non_blocking=True)

    def run(self):
        if not self.use_graph:
            self.out = self._body()
            return self.out
        if self.graph is None:
            # warm-up and capture on the SAME stream: the model workspace and the solver's
            # scratch are keyed by (device, stream), so the warm-up sizes exactly the buffers the
            # captured launches use and nothing is allocated during capture
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                ref = self._body()
            torch.cuda.current_stream().wait_stream(s)
            self.graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(self.graph, stream=s):
                self.out = self._body()
            # self-check: two replays separated by a synchronise must reproduce the eager
            # warm-up exactly (same kernels, same inputs); see spe/_lib.py on packet capture
            for _ in range(2):
                torch.cuda.synchronize()
                self.graph.replay()
            torch.cuda.synchronize()
            pairs = [(ref["forward"][k], self.out["forward"][k]) for k in ref["forward"]]
            pairs += [(ref["poses"][k], self.out["poses"][k]) for k in ("status", "quat", "tvec")]
            if not all(torch.equal(a, b) for a, b in pairs):
                self.graph = None
                raise RuntimeError("HIP graph replay of the pose pipeline differs from eager execution: run with "
                                   "DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 set before HIP initialises (spe/_lib.py)")
            return self.out
        self.graph.replay()
        return self.out
