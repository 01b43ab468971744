"""Multi-GPU plumbing: one process per GPU, torch.distributed over RCCL ("nccl" backend on
ROCm) or gloo on CPU (tests).  Mirrors REV/utils/misc.py:415-440 (env:// rank discovery).

The path is data-parallel: images shard over ranks with identical weights.  The only exchange
is one all-gather of fixed-size per-image pose records (RECORD_LEN fp64 each) so every rank's
SpeedEval sees the whole dataset — new behaviour relative to the reference, whose rank-local
summarize() reports per-shard scores (REV/engine.py:122-128).
"""
from __future__ import annotations

import os

import torch
import torch.distributed as dist

# quat(4) tvec(3) s_t s_q status
RECORD_LEN = 10


def init_distributed_mode(backend=None):
    """Returns (rank, world_size, local_rank); single process when RANK/WORLD_SIZE are unset."""
    if "RANK" not in os.environ or "WORLD_SIZE" not in os.environ:
        return 0, 1, 0
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    local = int(os.environ.get("LOCAL_RANK", 0))
    if not dist.is_initialized():
        if backend is None:
            # SPE_DIST_BACKEND=gloo: the rehearsal of the multi-rank path with every rank on one
            # GPU (RCCL needs one device per rank)
            backend = os.environ.get("SPE_DIST_BACKEND") or ("nccl" if torch.cuda.is_available() else "gloo")
        if backend == "nccl":
            torch.cuda.set_device(local)
        dist.init_process_group(backend=backend, init_method="env://", world_size=world, rank=rank)
    return rank, world, local


def is_dist():
    return dist.is_available() and dist.is_initialized()


def shard(n_total, rank, world):
    """Contiguous shard [lo, hi) of n_total images for `rank`."""
    per = (n_total + world - 1) // world
    lo = min(rank * per, n_total)
    return lo, min(lo + per, n_total)


def pack_records(quat, tvec, s_t, s_q, status):
    """[B, RECORD_LEN] fp64 pose records (device)."""
    return torch.cat([quat.double(), tvec.double(), s_t[:, None], s_q[:, None], status.double()[:, None]], 1)


def all_gather_records(rec):
    """All-gather equal-size record blocks from every rank -> [world*B, RECORD_LEN]."""
    if not is_dist() or dist.get_world_size() == 1:
        return rec
    parts = [torch.empty_like(rec) for _ in range(dist.get_world_size())]
    dist.all_gather(parts, rec.contiguous())
    return torch.cat(parts, 0)


def exchange_pose_records(poses, s_t, s_q, stream=None):
    """The bench / pipeline's per-batch exchange: pack this rank's pose records and all-gather
    them, ordered after the batch's solver work (issued on `stream`, the solver's stream, when
    given).  Returns [world*B, RECORD_LEN] (this rank's block alone when not distributed)."""
    if stream is not None:
        with torch.cuda.stream(stream):
            return all_gather_records(pack_records(poses["quat"], poses["tvec"], s_t, s_q, poses["status"]))
    return all_gather_records(pack_records(poses["quat"], poses["tvec"], s_t, s_q, poses["status"]))


def all_gather_log(log: dict) -> dict:
    """Merge every rank's SpeedEval.log (host objects, evaluate() path)."""
    if not is_dist() or dist.get_world_size() == 1:
        return log
    parts = [None] * dist.get_world_size()
    dist.all_gather_object(parts, log)
    merged = {}
    for p in parts:
        merged.update(p)
    return merged
