"""Throughput of the keypoint-set pose path on MI355X (BASELINE.json metric).

One step = one batch of synthetic SPEED-shaped 416x416 crops, resident in HBM, through
backbone -> transformer -> keypoint heads + fused PostProcess -> batched PnP -> SPEED score
(+ one RCCL all-gather of the per-image pose records when N > 1).  Default workload is
BASELINE config 2: ResNet50-s8 + 6/6 transformer, 11 queries, bf16, bs=64 per GPU, EPnP only.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

Prints ONE JSON line (rank 0).  The dominant kernel's launches are bracketed with HIP events
on the launch stream during the timed region (spe_model_profile_*) for the roofline object.
"""
import argparse
import glob
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "satellite-pose-estimation_amd"))

# TFLOP/s, GB/s (MI355X_MICROARCH.md).  fp32x3 runs every product as three bf16 MFMAs (hi.hi +
# hi.lo + lo.hi), so its ceiling for the model's algorithmic flops is a third of the bf16 peak.
# fp32x6 (the accuracy-contract mode) runs its GEMMs / convolutions on six bf16 MFMAs per product and
# its attention as fp32x3: the ceiling for a launch depends on its class (peak_for).
PEAK = {"bf16": {"mfma": 2500.0}, "fp32": {"mfma": 157.3}, "fp32x3": {"mfma": 2500.0 / 3},
        "fp32x6": {"mfma": 2500.0 / 6}, "fp32h3": {"mfma": 2500.0 / 3}, "hbm": 8000.0}


# BASELINE.json north_star: ">= 10k img/s on 8 x MI355X at 416x416 bs=256, RANSAC-PnP + GN refinement"
NORTH_STAR_GLOBAL_BATCH = 256
PARITY_MODE_TEXT = {"fp32x6": "fp32 storage; GEMMs / convolutions at near-fp32 precision (three-way split, six bf16 "
                              "products), attention as fp32x3 (DESIGN.md section 4)",
                    "fp32x3": "fp32 storage, split-bf16 MFMA (hi.hi + hi.lo + lo.hi)",
                    "fp32": "fp32 storage, exact-f32 MFMA",
                    "fp32h3": "fp32 storage; GEMMs and convolutions at near-fp32 precision as three fp16 MFMAs on a "
                              "power-of-two-scaled two-way fp16 split, encoder attention as fp32x3, decoder attention "
                              "exact fp32 (DESIGN.md section 4)"}


def peak_for(dtype, kind, queries=None):
    """MFMA ceiling (TFLOP/s of model flops) of launch class `kind` in mode `dtype` (`queries`: the
    model's Q -- fp32h3's decoder cross-attention runs on the three-fp16-product kernel for Q <= 12,
    xattn_h3.hip, and on the exact-f32 one otherwise)."""
    if dtype == "fp32h3" and kind == "attn.dec_cross" and queries is not None and queries <= 12:
        return PEAK["fp32h3"]["mfma"]
    if dtype in ("fp32x6", "fp32h3") and kind.startswith("attn.dec"):   # the decoder's attention: exact f32
        return PEAK["fp32"]["mfma"]
    if dtype in ("fp32x6", "fp32h3") and kind.startswith("attn."):     # the encoder's: fp32x3
        return PEAK["fp32x3"]["mfma"]
    return PEAK[dtype]["mfma"]
# profiler symbol of each launch class (to match profiles/*kernel_stats.csv rows)
# (rocprofv3 prints the attention kernels mangled: it does not demangle the __bf16 / _Float16
# template arguments, DF16b / DF16_)
# (bf16 models' encoder attention: bf16 q/k, fp16 V^T and P -- attn16_kernel<0, bf16, f16>)
KIND_SYMBOL = {"attn.enc": "_ZN12_GLOBAL__N_113attn16_kernelILi0EDF16bDF16_Lb1EEEv8AttnArgs",
               "attn.dec_self": "_ZN12_GLOBAL__N_113attn16_kernelILi1EDF16bDF16bEEv8AttnArgs",
               "attn.dec_cross": "xattn_kernel", "ffn.enc": "ffn_pipe_kernel<3, true, 6>", "ffn.dec": "ffn_ln_kernel<2, 3>"}


# BASELINE.json configs: per-GPU shapes (configs 3-5 are quoted at bs=256 over 8 GPUs = 32/GPU)
PRESETS = {
    2: dict(batch=64, size=416, queries=11, layers=6, solver="epnp", sigma_head=0),
    3: dict(batch=32, size=416, queries=11, layers=6, solver="ransac_p3p_lm", sigma_head=0),
    4: dict(batch=32, size=416, queries=11, layers=6, solver="epnp_ransac_sigma", sigma_head=1),
    5: dict(batch=32, size=640, queries=40, layers=6, solver="ransac_p3p_lm", sigma_head=0, attn_dtype="fp16"),
}
CONFIG_NAME = {
    2: "BASELINE config 2: ResNet50-s8 + {L}/{L} DETR, {Q} queries, {S}x{S}, solver={solver}",
    3: "BASELINE config 3: ResNet50-s8 + {L}/{L} DETR, {Q} queries, {S}x{S}, RANSAC-P3P + LM refine (solver={solver})",
    4: "BASELINE config 4: ResNet50-s8 + {L}/{L} DETR + sigma head, {Q} queries, {S}x{S}, sigma-weighted "
       "EPnP-RANSAC + self-assessment filter (solver={solver})",
    5: "BASELINE config 5: ResNet50-s8 + {L}/{L} DETR, {Q} queries, {S}x{S} (train_resnet50s8_query40), "
       "{A} MFMA encoder attention, solver={solver}",
}


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--model", default="detr", choices=["detr", "rtdetr_r18", "rtdetr_r50"],
                   help="detr: the REV DETR keypoint model (BASELINE configs); rtdetr_*: the UNC RT-DETR sigma model "
                        "(SURVEY 8f.4) at its speed config (256x256, 30 queries, 3 decoder layers, sigma-weighted "
                        "EPnP-RANSAC + self-assessment)")
    p.add_argument("--config", type=int, default=2, choices=sorted(PRESETS),
                   help="BASELINE.json configs[k-1] preset (2 = the headline metric's workload); explicit flags override")
    p.add_argument("--batch", type=int, default=None, help="images per GPU per step")
    p.add_argument("--size", type=int, default=None)
    p.add_argument("--queries", type=int, default=None)
    p.add_argument("--layers", type=int, default=None)
    p.add_argument("--solver", default=None, choices=["epnp", "epnp_lm", "ransac_p3p_lm", "epnp_ransac_sigma", "epnp_ceres"])
    p.add_argument("--sigma-head", type=int, default=None, choices=[0, 1])
    p.add_argument("--dtype", default="bf16", choices=["bf16", "fp32", "fp32x3", "fp32x6", "fp32h3"],
                   help="bf16: throughput mode; fp32: exact-f32 MFMA parity mode; fp32x3: fp32 storage with "
                        "split-bf16 MFMA (the fast parity mode)")
    p.add_argument("--attn-dtype", dest="attn_dtype", default=None, choices=["bf16", "fp16"],
                   help="encoder self-attention operand type (bf16 models; config 5 preset: fp16)")
    p.add_argument("--weights", default="pose-consistent", choices=["pose-consistent", "label-diverse", "random"],
                   help="label-diverse: random init made query-diverse so the solver sees >= 4 "
                        "correspondences like a trained model (spe.synthetic.bench_weights); pose-consistent "
                        "(default, DETR): label-diverse + the point head fitted on the timed batch so each "
                        "query predicts its label's landmark projection + N(0, 2 px) + 10%% outliers "
                        "(spe.synthetic.fit_point_head), so RANSAC finds consensus and the refinement runs")
    p.add_argument("--parity-dtype", default="fp32h3", choices=["fp32h3", "fp32x6", "fp32x3", "fp32"],
                   help="the parity mode timed after the main line in the same process (parity_mode object: its "
                        "own ms_per_step, value, roofline and accuracy against the exact-f32 mode)")
    p.add_argument("--no-parity", action="store_true", help="skip the parity_mode timing")
    p.add_argument("--host-input-last", action="store_true",
                   help="time the host_input object after the device-resident line (default: before it; timed "
                        "second it measured ~12 %% slower in this process, while scripts/lab/host_input_ab.py, "
                        "alternating the two pipelines, measures 10.38 vs 10.40 ms)")
    p.add_argument("--no-host-input", action="store_true",
                   help="skip the host_input object (the same step fed from pinned host memory: 8-bit crops "
                        "copied H2D every step on a copy stream, REV/engine.py:92)")
    p.add_argument("--north-star", action="store_true",
                   help="also time the north-star shape at N = 1 (default only for N > 1): global batch 256 over the "
                        "ranks, RANSAC-P3P + LM, bf16 and the parity dtype, accuracy against exact f32")
    p.add_argument("--no-north-star", action="store_true", help="skip the north_star object for N > 1")
    p.add_argument("--no-accuracy", action="store_true",
                   help="skip the post-timing accuracy check of a bf16 run against the fp32 parity mode")
    p.add_argument("--no-overlap", action="store_true",
                   help="run the solver on the forward's stream (default: solver of batch i overlaps the forward of i+1)")
    p.add_argument("--no-overlap-backbone", action="store_true",
                   help="run batch i's encoder layers on the backbone's stream (default: on their own stream beside "
                        "batch i+1's backbone, three workspaces)")
    p.add_argument("--no-overlap-decode", action="store_true",
                   help="keep each batch's decoder + heads on the forward's stream (default: batch i's "
                        "decoder runs on its own stream beside batch i+1's backbone/encoder, two workspaces)")
    p.add_argument("--raw-frames", action="store_true",
                   help="start every step from 1920x1200 8-bit frames + detector boxes in HBM: the "
                        "validation transform (crop, cv2-cubic resize, normalise; spe.datasets) runs "
                        "on the device inside the timed step")
    p.add_argument("--jpeg", action="store_true",
                   help="with --raw-frames: start every step from the frames' baseline-JPEG files (Pillow-encoded, "
                        "quality 90) in HBM, decoded on the device (spe.datasets.JpegDecoder) inside the timed step")
    p.add_argument("--cpu-seconds", type=float, default=15.0)
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--launch-table", default=None,
                   help="write every launch of the profiled step (kind, ms, flops, bytes, roofline floor) as JSON")
    a = p.parse_args()
    if a.model != "detr":
        for k, v in dict(batch=64, size=256, queries=30, layers=3, solver="epnp_ransac_sigma", sigma_head=1).items():
            if getattr(a, k) is None:
                setattr(a, k, v)
    for k, v in PRESETS[a.config].items():
        if getattr(a, k) is None:
            setattr(a, k, v)
    if a.attn_dtype is None or a.dtype != "bf16":
        a.attn_dtype = a.dtype
    return a


def usable_cpus():
    """CPUs this process may run on: the affinity mask, capped by a cgroup CPU quota when one is
    set (a GPU box's share of a large host is enforced that way; os.cpu_count() shows the host)."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
        if q != "max":
            n = min(n, max(1, int(int(q) // int(per))))
    except (OSError, ValueError):
        pass
    return n


def host_cpu():
    """CPU model, logical CPUs, physical cores of this host and the CPUs usable by this process
    (BASELINE.md section 3 fields)."""
    name, cores = "unknown", set()
    phys = core = None
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                k, _, v = line.partition(":")
                k, v = k.strip(), v.strip()
                if k == "model name" and name == "unknown":
                    name = v
                elif k == "physical id":
                    phys = v
                elif k == "core id":
                    core = v
                elif not k and phys is not None and core is not None:
                    cores.add((phys, core))
                    phys = core = None
        if phys is not None and core is not None:
            cores.add((phys, core))
    except OSError:
        pass
    return {"cpu_model": name, "host_logical_cpus": os.cpu_count(), "host_physical_cores": len(cores) or None,
            "usable_cpus": usable_cpus(), "omp_num_threads_env": os.environ.get("OMP_NUM_THREADS")}


def _baseline_record(n, dt, threads, sample):
    v = n / dt
    return {"value": v, "unit": "images/s", "cores": threads, "threads_used": threads,
            "value_per_core": v / threads, "kind": "port",
            "threads_note": "torch.set_num_threads(all CPUs usable by this process: affinity mask capped by the "
                            "cgroup quota); one thread per usable CPU",
            "kind_note": "the reference's evaluate() cannot run here (cv2 / mathutils / torchvision absent and the "
                         "reference never ships to the GPU box): oracle/ restatement of the same path timed instead",
            **host_cpu(), "sample": sample}


def cpu_baseline(cfg, seconds, solver="epnp"):
    """Oracle port (torch-fp32 CPU model + C solver) timed on this host's cores on a bounded
    sample of the same workload: single images of the bench's shape, repeated until `seconds`
    elapse."""
    import torch
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import model_ref
    import pnp_ref
    from spe.config import Camera, world_points
    from spe.synthetic import random_weights, synthetic_batch
    mode = {"epnp": pnp_ref.MODE_EPNP, "epnp_lm": pnp_ref.MODE_EPNP_LM, "ransac_p3p_lm": pnp_ref.MODE_RANSAC_P3P_LM,
            "epnp_ransac_sigma": pnp_ref.MODE_EPNP_RANSAC_SIGMA}[solver]
    threads = usable_cpus()
    torch.set_num_threads(threads)
    w = random_weights(cfg, 0)
    b = synthetic_batch(cfg, 1, 99)
    W, K = world_points(), Camera.K
    n, t0 = 0, time.perf_counter()
    with torch.no_grad():
        while True:
            o = model_ref.forward(b["images"], w, cfg)
            pp = model_ref.postprocess(o["pred_logits"], o["pred_points"], b["clip_bbox"], o.get("pred_sigmas"))
            sg = pp[0]["sigmas"][None] if "sigmas" in pp[0] else None
            pnp_ref.pnp_batch(pp[0]["points"][None], pp[0]["logits"][None], K, W, mode=mode,
                              repro=25.0 if mode == pnp_ref.MODE_EPNP_RANSAC_SIGMA else 20.0, sigmas=sg)
            n += 1
            if time.perf_counter() - t0 >= seconds:
                break
    dt = time.perf_counter() - t0
    return _baseline_record(n, dt, threads,
                            f"{n} single-image passes ({cfg.input_size}x{cfg.input_size}, Q={cfg.num_queries}, "
                            f"{cfg.enc_layers}/{cfg.dec_layers}{', sigma head' if cfg.sigma_head else ''}, fp32 "
                            f"torch-CPU model + C {solver} oracle) in {dt:.1f}s")


def cpu_baseline_rtdetr(rcfg, seconds):
    """Oracle port of the UNC RT-DETR model (torch-fp32 CPU restatement + C sigma-EPnP-RANSAC
    solver) on single images, like cpu_baseline."""
    import torch
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import pnp_ref
    import rtdetr_ref
    from spe.config import Camera, SpeConfig, world_points
    from spe.rtdetr_spec import random_rtdetr_weights
    from spe.synthetic import synthetic_batch
    threads = usable_cpus()
    torch.set_num_threads(threads)
    w = random_rtdetr_weights(rcfg, 0)
    b = synthetic_batch(SpeConfig(input_size=rcfg.input_size), 1, 99)
    W, K = world_points(), Camera.K
    n, t0 = 0, time.perf_counter()
    with torch.no_grad():
        while True:
            o = rtdetr_ref.forward(b["images"], w, rcfg)
            pp = rtdetr_ref.postprocess(o, b["clip_bbox"])
            pnp_ref.pnp_batch(pp["points"].numpy(), pp["probs"].numpy(), K, W, mode=pnp_ref.MODE_EPNP_RANSAC_SIGMA,
                              repro=25.0, sigmas=pp["sigmas"].numpy())
            n += 1
            if time.perf_counter() - t0 >= seconds:
                break
    dt = time.perf_counter() - t0
    return _baseline_record(n, dt, threads,
                            f"{n} single-image passes (RT-DETR r{rcfg.depth}vd {rcfg.input_size}x{rcfg.input_size}, "
                            f"Q={rcfg.num_queries}, fp32 torch-CPU restatement + C epnp_ransac_sigma oracle) in {dt:.1f}s")


def bench_data(cfg, B, rank):
    """Rank `rank`'s timed images: pool images [rank*B, rank*B + B) (spe.synthetic.bench_images)."""
    from spe.synthetic import bench_images
    return bench_images(cfg, rank * B, B)


def pose_consistent_weights(w, cfg, rank, world, dev, rcfg=None, chunk=32):
    """Shapes without a committed head fixture (config 5, RT-DETR): fit the point head
    (spe.synthetic.fit_point_head) on the decoder outputs of the whole bench pool
    (spe.synthetic.BENCH_POOL images, independent of the rank count), computed by the exact-f32
    mode on rank 0, which fits and broadcasts the head -- so the weights depend neither on the
    bf16 kernels under test nor on the number of ranks.  RT-DETR (rcfg): the last decoder layer's
    dec_bbox_head, whose points are sigmoid(head(hs) + inverse_sigmoid(the previous layer's
    points)) (UNC src/zoo/rtdetr/rtdetr_decoder.py:336-337) -- the fit gets those logits as its
    offset."""
    import torch
    import torch.distributed as dist
    from spe.synthetic import BENCH_POOL, bench_images, fit_point_head, keypoint_targets
    prefix = "point_embed" if rcfg is None else f"decoder.dec_bbox_head.{rcfg.dec_layers - 1}"
    keys = [f"{prefix}.layers.{j}.{k}" for j in range(3) for k in ("weight", "bias")]
    fit = None
    if rank == 0:
        data = bench_images(cfg, 0, BENCH_POOL)
        if rcfg is None:
            from spe.models import DETR
            m = DETR(cfg, dtype="fp32")
        else:
            from spe.rtdetr import RTDETR
            m = RTDETR(rcfg, dtype="fp32", aux_outputs=True)
        m.load_state_dict(w)
        hs, logits, off = [], [], []
        for i in range(0, BENCH_POOL, chunk):
            o = m(torch.from_numpy(data["images"][i:i + chunk]).to(dev), return_hs=True)
            hs.append(o["hs"].float().cpu())
            logits.append(o["pred_logits"].float().cpu())
            if rcfg is not None:
                ref = o["aux_outputs"][rcfg.dec_layers - 2]["pred_pts"].clamp(0.0, 1.0)
                off.append(torch.log(ref.clamp(min=1e-5) / (1 - ref).clamp(min=1e-5)).float().cpu())  # inverse_sigmoid
        del m
        hs = torch.cat(hs).numpy()
        labels = torch.cat(logits).argmax(-1).numpy()
        tgt, mask = keypoint_targets(data, labels, seed=7)
        w, err = fit_point_head(w, hs, tgt, mask, device=dev, prefix=prefix,
                                offset=None if rcfg is None else torch.cat(off).numpy())
        fit = {"fit_err_max_norm": float(err.max()), "fit_err_mean_norm": float(err.mean()),
               "fit_queries": int(mask.sum()), "fit_set": f"bench pool images 0..{BENCH_POOL - 1} (exact-f32 hs)"}
    if world > 1:
        for k in keys:
            t = torch.from_numpy(w[k]).to(dev) if rank == 0 else torch.empty(w[k].shape, device=dev)
            dist.broadcast(t, 0)
            w[k] = t.cpu().numpy()
    return w, fit


def keypoint_error_px(points_px, probs, data):
    """Per foreground query (argmax label < 11): pixel distance to its label's landmark."""
    import numpy as np
    pts, lab = points_px.cpu().numpy(), probs.argmax(-1).cpu().numpy()
    lm = data["landmarks"]
    e = [np.linalg.norm(pts[i, q] - lm[i, lab[i, q]]) for i in range(pts.shape[0]) for q in range(pts.shape[1])
         if lab[i, q] < lm.shape[1]]
    return np.asarray(e)


def image_areas(data, solver):
    """EPnPCeresSolver only (else None): each image's UNC SpeedEval "area" from its landmark box
    (bbox_xxyy, src/data/speed/speed_dataset.py:370-373, precedence kept), the threshold input."""
    import numpy as np
    from spe import _lib
    if getattr(solver, "mode", None) != _lib.SPE_PNP_EPNP_CERES:
        return None
    if "bbox_xxyy" in data:
        b = np.asarray(data["bbox_xxyy"], np.float64)
    else:
        lm = np.asarray(data["landmarks"], np.float64)
        b = np.stack([lm[..., 0].min(1), lm[..., 1].min(1), lm[..., 0].max(1), lm[..., 1].max(1)], 1)
    return [float(np.sqrt((x2 - x1) * y2 - y1)) for x1, y1, x2, y2 in b]


class Fp32Reference:
    """The exact-f32 parity mode's outputs on the timed batch (that mode is pinned to the reference
    at <= 1e-4 by tests/test_gpu_parity.py on every golden case), computed once and compared with
    every timed mode: forward outputs, hs, and its poses / SPEED scores through the same solver.
    `cond` [B]: the score's float32 conditioning -- per image, the largest SPEED-score change over
    ULP_DRAWS re-solves of the same keypoints each moved by one float32 ulp per coordinate in a
    random direction (the resolution of the reference's own float32 PostProcess output).  An image
    whose score moves by more than 1e-4 under such a perturbation cannot be matched to 1e-4 by any
    implementation that is not bit-identical to the reference."""
    ULP_DRAWS = 16

    def __init__(self, cfg, w, data, solver, dev):
        import numpy as np
        import torch
        from spe.models import DETR
        from spe.speed_eval import device_speed_score
        ref = DETR(cfg, dtype="fp32")
        ref.load_state_dict(w)
        self.images = torch.from_numpy(data["images"]).to(dev)
        self.clip = torch.from_numpy(data["clip_bbox"]).float().to(dev)
        self.r = ref(self.images, clip_bbox=self.clip, return_hs=True)
        area = image_areas(data, solver)
        kw = {} if area is None else {"area": area}
        self.pr = solver.solve_batch(self.r["points_px"], self.r["probs"], self.r.get("sigmas"), **kw)
        self.q_gt = torch.from_numpy(data["quat"]).to(dev)
        self.t_gt = torch.from_numpy(data["tvec"]).to(dev)
        st, sq = device_speed_score(self.pr["quat"], self.pr["tvec"], self.q_gt, self.t_gt)
        self.score = (st + sq).cpu().numpy()
        # the self-assessment filter's flag (sigma head, BASELINE config 4)
        self.reliable = (solver.self_assess(self.r["probs"], self.r["sigmas"], self.pr)["reliable"].bool()
                         if self.r.get("sigmas") is not None else None)
        # float32 conditioning of each image's score (same HIP solver, one batch of B * ULP_DRAWS)
        B = self.score.shape[0]
        M = self.ULP_DRAWS
        p = self.r["points_px"].cpu().numpy().astype(np.float32)
        rng = np.random.Generator(np.random.PCG64(11))
        sgn = rng.choice(np.array([-np.inf, np.inf], np.float32), size=(M,) + p.shape)
        pp = np.nextafter(np.broadcast_to(p, (M,) + p.shape), sgn).astype(np.float32).reshape((M * B,) + p.shape[1:])
        rep = lambda t: t.repeat((M,) + (1,) * (t.dim() - 1)) if t is not None else None  # noqa: E731
        kw = {} if area is None else {"area": list(area) * M}
        pert = solver.solve_batch(torch.from_numpy(pp).to(dev), rep(self.r["probs"]), rep(self.r.get("sigmas")), **kw)
        st, sq = device_speed_score(pert["quat"], pert["tvec"], rep(self.q_gt), rep(self.t_gt))
        sc = (st + sq).cpu().numpy().reshape(M, B)
        diff = np.abs(sc - self.score[None])            # NaN where either score is NaN
        diff = np.where(np.isnan(sc) != np.isnan(self.score[None]), np.inf, diff)
        self.cond = np.nan_to_num(diff, nan=0.0).max(0)
        torch.cuda.synchronize()
        del ref


def accuracy_raw(model, ref, out):
    """Per-row / per-image raw deltas of a timed mode against the fp32 parity mode on the timed
    batch (gathered over ranks before accuracy_summary)."""
    import numpy as np
    r = ref.r
    hb = model(ref.images, return_hs=True)["hs"]
    hs_rel = ((hb - r["hs"]).norm(dim=-1) / r["hs"].norm(dim=-1)).flatten()
    fo = out["forward"]
    lab_b, lab_r = fo["probs"].argmax(-1), r["probs"].argmax(-1)
    fg = (lab_r < 11) & (lab_b == lab_r)
    wcrop = (ref.clip[:, 2] - ref.clip[:, 0])[:, None].expand_as(lab_r)
    d = (fo["points_px"] - r["points_px"]).norm(dim=-1)[fg]
    dn = (fo["pred_points"] - r["pred_points"]).abs().amax(-1)[fg]
    return {"hs_rel": hs_rel.cpu().numpy(), "label_agree": (lab_b == lab_r).cpu().numpy().ravel(),
            "d_px": d.cpu().numpy(), "d_norm": dn.cpu().numpy(), "d_per_crop": (d / wcrop[fg]).cpu().numpy(),
            "score_ref": ref.score, "score": (out["s_t"] + out["s_q"]).cpu().numpy(), "cond": ref.cond,
            "status_agree": (ref.pr["status"] == out["poses"]["status"]).cpu().numpy(),
            **({"reliable": (out["assess"]["reliable"].bool() == ref.reliable).cpu().numpy()}
               if ref.reliable is not None and "assess" in out else {})}


# The fp32 implementation spread of the per-image SPEED score:
# the reference's own torch-CPU execution and the torch-GPU one against this repo's exact-f32 mode,
# all through the same HIP solver, on the config-2 batch (pool images 0..63, the bench fixture
# weights); written by tests/test_gpu_precision.py.
SCORE_SPREAD_FILE = os.path.join(REPO, "profiles", "r5f_precision_score.json")
# the same study on the whole 256-image pool (the north star's global batch; SPE_PRECISION_IMAGES=256)
SCORE_SPREAD_FILE_256 = os.path.join(REPO, "profiles", "r5f_precision_score_256.json")


# configs 4 and 5 (tests/test_gpu_precision.py::test_fp32h3_within_fp32_spread_config, their own
# solvers and shapes: sigma-weighted EPnP-RANSAC / 640x640 Q40 with P3P-RANSAC + LM)
SCORE_SPREAD_FILE_CFG = {4: os.path.join(REPO, "profiles", "r6_precision_score_c4.json"),
                         5: os.path.join(REPO, "profiles", "r6_precision_score_c5.json")}


def spread_file(images, config=2):
    """The committed spread study matching a batch of `images` pool images of BASELINE config
    `config` (the extreme-value max grows with the batch, so a 256-image batch is held to the
    256-image study when it exists)."""
    if config in SCORE_SPREAD_FILE_CFG:
        return SCORE_SPREAD_FILE_CFG[config]
    return SCORE_SPREAD_FILE_256 if images >= 256 and os.path.exists(SCORE_SPREAD_FILE_256) else SCORE_SPREAD_FILE


def score_spread(solver, images=64, config=2):
    """{'frac', 'median', 'max'} of torch-CPU vs ours-fp32 (max: the largest disagreement of any two fp32
    implementations -- torch-CPU, torch-GPU, ours) for `solver` on config `config`'s shape, or None."""
    try:
        st = json.load(open(spread_file(images, config)))["score"][solver]
    except Exception:
        return None
    per = st.get("per_image")
    if per is not None and len(per["torch_cpu_vs_fp32"]) >= images:
        # the study's per-image deltas on exactly the bench's images (pool images 0..images-1)
        import numpy as np
        d = {k: np.asarray(v[:images], np.float64) for k, v in per.items()}
        cpu = d["torch_cpu_vs_fp32"][np.isfinite(d["torch_cpu_vs_fp32"])]
        mx = max(float(np.nanmax(v)) for v in d.values())
        return {"frac": float((cpu <= 1e-4).mean()), "median": float(np.median(cpu)), "max": mx, "images": images}
    d = st["pairs"]
    cpu, gpu, cg = d["torch_cpu_vs_fp32"], d["torch_gpu_vs_fp32"], d["torch_cpu_vs_torch_gpu"]
    return {"frac": cpu["frac_le_1e-4"], "median": cpu["median"], "max": max(cpu["max"], gpu["max"], cg["max"])}


def reliable_spread(config, images=64):
    """torch-CPU's agreement with the exact-f32 mode on the self-assessment `reliable` flag (config 4's
    study; over its first `images` images when it holds them per image), or None."""
    try:
        r = json.load(open(spread_file(images, config)))["reliable"]
    except Exception:
        return None
    per = r.get("per_image_torch_cpu_vs_fp32")
    if per is not None and len(per) >= images:
        return float(sum(per[:images]) / images)
    return r["torch_cpu_vs_fp32"]


def accuracy_summary(raw, solver=None, config=2):
    """Accuracy of a timed mode against the fp32 parity mode: keypoint deltas of the foreground
    queries both label alike, label agreement, hs relative error, and the SPEED-score delta of the
    two modes' poses through the same solver -- overall, and over the images whose score is
    well-conditioned at float32 resolution (Fp32Reference.cond <= 1e-4).
    `score_within_fp32_spread`: the score half of the contract held to the spread of two fp32
    implementations of the reference instead of the strict 1e-4 (score_spread; the gates of
    tests/test_gpu_precision.py) -- the strict per-image `meets_1e-4_score` stays reported beside it;
    `meets_1e-4_within_fp32_spread` = `meets_1e-4_kpt` and `score_within_fp32_spread`.  With the sigma
    head: `reliable_agreement`, the share of images whose self-assessment flag equals the exact-f32
    mode's (config 4)."""
    import numpy as np
    sc_r, sc_b, cond = raw["score_ref"], raw["score"], raw["cond"]
    both = np.isfinite(sc_r) & np.isfinite(sc_b)
    ds = np.abs(sc_b - sc_r)[both]
    wc = (cond <= 1e-4)[both]
    dn = raw["d_norm"]
    res = {"reference_mode": "fp32 parity mode (<= 1e-4 of the reference on its goldens)",
           "hs_rel_err_mean": float(raw["hs_rel"].mean()), "hs_rel_err_max": float(raw["hs_rel"].max()),
           "label_agreement": float(raw["label_agree"].mean()),
           "kpt_px_max": float(raw["d_px"].max()), "kpt_px_mean": float(raw["d_px"].mean()),
           "kpt_norm_max": float(dn.max()), "kpt_norm_mean": float(dn.mean()),
           "frac_kpt_norm_le_1e-4": float((dn <= 1e-4).mean()),
           "kpt_px_per_crop_px": float(raw["d_per_crop"].max()),
           "score_delta_max": float(ds.max()) if ds.size else None,
           "score_delta_mean": float(ds.mean()) if ds.size else None,
           "frac_score_delta_le_1e-4": float((ds <= 1e-4).mean()) if ds.size else None,
           "score_mean_fp32": float(np.nanmean(sc_r)), "score_mean_timed": float(np.nanmean(sc_b)),
           "status_agreement": float(raw["status_agree"].mean()),
           "images": int(len(sc_r)),
           # float32 conditioning of the reference poses (Fp32Reference.cond)
           "images_ill_conditioned_at_f32_ulp": int((cond > 1e-4).sum()),
           "score_cond_ulp_median": float(np.median(cond)),
           "images_well_conditioned": int(wc.sum()),
           "score_delta_max_well_conditioned": float(ds[wc].max()) if wc.any() else None,
           "frac_score_delta_le_1e-4_well_conditioned": float((ds[wc] <= 1e-4).mean()) if wc.any() else None}
    res["score_delta_median"] = float(np.median(ds)) if ds.size else None
    res["meets_1e-4_kpt"] = bool(res["kpt_norm_max"] <= 1e-4)
    res["meets_1e-4_score"] = bool((res["score_delta_max"] or 0.0) <= 1e-4)
    res["meets_1e-4"] = res["meets_1e-4_kpt"] and res["meets_1e-4_score"]
    if "reliable" in raw:
        res["reliable_agreement"] = float(raw["reliable"].mean())
        rs = reliable_spread(config, len(raw["reliable"]))
        if rs is not None:
            res["reliable_agreement_torch_cpu_vs_fp32"] = rs
            res["reliable_within_fp32_spread"] = bool(res["reliable_agreement"] >= rs - 0.05)
    sp = score_spread(solver, len(sc_r), config) if solver else None
    if sp is not None and ds.size:
        res["score_fp32_spread"] = {
            "definition": "per-image |SPEED score - exact-f32 score| <= 1e-4 on at least the fraction of images the "
                          "reference's own fp32 CPU execution reaches - 0.05, median <= 2x its median, max <= the largest "
                          "disagreement of two fp32 implementations (torch-CPU / torch-GPU restatements and the exact-f32 "
                          "mode, same HIP solver)",
            "source": os.path.relpath(spread_file(len(sc_r), config), REPO) + " (pool images 0.."
                      + str(sp["images"] - 1 if "images" in sp else
                            255 if spread_file(len(sc_r), config) == SCORE_SPREAD_FILE_256 else 63) + ", " + solver + ")",
            "spread_frac_le_1e-4": sp["frac"], "spread_median": sp["median"], "spread_max": sp["max"],
            **({"spread_images": sp["images"]} if "images" in sp else {})}
        res["score_within_fp32_spread"] = bool(
            res["frac_score_delta_le_1e-4"] >= sp["frac"] - 0.05 and res["score_delta_median"] <= 2 * sp["median"]
            and res["score_delta_max"] <= sp["max"])
        res["meets_1e-4_within_fp32_spread"] = res["meets_1e-4_kpt"] and res["score_within_fp32_spread"]
    return res


def accuracy_vs_fp32(model, ref, out, world=1, solver=None, config=2):
    """accuracy_summary over all ranks' images (one all_gather_object of the raw deltas)."""
    import numpy as np
    raw = accuracy_raw(model, ref, out)
    if world > 1:
        import torch.distributed as dist
        parts = [None] * world
        dist.all_gather_object(parts, raw)
        raw = {k: np.concatenate([p[k] for p in parts]) for k in raw}
    return accuracy_summary(raw, solver, config)


def traffic_for(kind, grid, attn_dtype):
    """HBM bytes per launch of `kind` from a committed PMC summary (profiles/pmc_*.json), or None.
    Only a summary measured on the same launch (kind, grid size in threads, operand type) counts."""
    best = None
    for f in sorted(glob.glob(os.path.join(REPO, "profiles", "pmc_*.json"))):
        try:
            d = json.load(open(f))
        except Exception:
            continue
        if not isinstance(d, dict):            # per-kernel counter tables (scripts/pmc_summary.py --json)
            continue
        if (d.get("kind") == kind and "hbm_bytes_per_launch" in d and grid is not None and d.get("grid") == grid
                and d.get("attn_dtype", "bf16") == attn_dtype):
            best = d["hbm_bytes_per_launch"]
    return best


def launch_grid(kind, B, cfg):
    """rocprofv3 Grid_Size (threads) of one launch of `kind` at this workload, where known."""
    if kind == "attn.enc":
        return B * cfg.nheads * ((cfg.tokens + 127) // 128) * 256
    return None


def launch_ranks(args):
    """`bench.py --gpus N` outside a torchrun environment: start N ranks (one process per GPU,
    python -m torch.distributed.run, rendezvous on 127.0.0.1) BEFORE this process touches the GPU,
    and return the launcher's exit status.  Rank 0 prints the JSON line.  Mirrors the reference's
    one-process-per-GPU launch (REV/main.py:213-217, REV/utils/misc.py:415-440)."""
    import socket
    import subprocess
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("OMP_NUM_THREADS", "1")
    return subprocess.call(cmd, env=env)


def result_header(args, world, elapsed, B, dtype):
    """The contract fields of the JSON line (whole-job img/s over all ranks, max-over-ranks time)."""
    return {
        "metric": f"images/sec end-to-end (backbone->kpts->PnP) at {args.size}x{args.size}; SPEED pose score",
        "value": B * world * args.steps / elapsed,
        "unit": "images/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": 1e3 * elapsed / args.steps,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": dtype,
    }


def stub_worker(args):
    """SPE_BENCH_STUB=1 (CPU tests of the launcher, tests/test_host.py): the rank bookkeeping of a
    real run -- env:// rendezvous over gloo, world == --gpus check, barrier-bracketed timing, max
    over ranks, one pose-record all-gather -- with no GPU work; rank 0 prints the line."""
    import torch
    import torch.distributed as dist
    from spe import dist as sd
    rank, world, _ = sd.init_distributed_mode(backend="gloo")
    if world != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but world size {world}", file=sys.stderr)
        return 2
    B = args.batch
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        rec = sd.all_gather_records(sd.pack_records(torch.zeros(B, 4), torch.zeros(B, 3), torch.zeros(B, dtype=torch.float64),
                                                    torch.zeros(B, dtype=torch.float64), torch.zeros(B, dtype=torch.int32)))
    if world > 1:
        dist.barrier()
    el = torch.tensor([time.perf_counter() - t0], dtype=torch.float64)
    if world > 1:
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
    # the weights a real run of this shape would time (CPU-side: random init + the head fixture) and
    # the north-star shard of every rank (pool images), gathered like the real line's accuracy
    from spe.config import SpeConfig
    from spe.synthetic import fixed_bench_weights, weights_checksum
    cfg = SpeConfig(input_size=args.size, num_queries=args.queries, enc_layers=args.layers, dec_layers=args.layers)
    w, _ = fixed_bench_weights(cfg, 0)
    nb = NORTH_STAR_GLOBAL_BATCH // world
    shard = list(range(rank * nb, rank * nb + nb))
    shards = [None] * world
    if world > 1:
        dist.all_gather_object(shards, shard)
    else:
        shards = [shard]
    if rank == 0:
        r = result_header(args, world, float(el.item()), B, args.dtype)
        r["config"] = {"workload": "launcher stub (no GPU work)", "global_batch": B * world, "per_gpu_batch": B,
                       "parallelism": f"dp{world} (image sharding)"}
        r["records_gathered_per_step"] = int(rec.shape[0])
        r["weights_sha256_16"] = weights_checksum(w) if w is not None else None
        r["north_star"] = {"global_batch": NORTH_STAR_GLOBAL_BATCH, "per_gpu_batch": nb, "n_gpus": world,
                           "solver": "ransac_p3p_lm", "pool_images": sorted(i for sh in shards for i in sh)}
        print(json.dumps(r))
    if dist.is_initialized():
        dist.destroy_process_group()
    return 0


def time_mode(pipe, model, args, world, dev, dtype, attn_dtype, cfg, B, launch_table=None):
    """Warm-up, one per-launch-profiled step (dominant kernel class), then EXACTLY args.steps timed
    steps between barriers + synchronize, the dominant class's launches bracketed by HIP events on
    their stream; elapsed = max over ranks.  Returns the timing, the roofline object and the last
    step's outputs."""
    import ctypes
    import torch
    import torch.distributed as dist
    from spe import _lib
    from spe import dist as sd

    def step():
        out = pipe.run()
        if world > 1:
            # on the solver's stream: the record exchange waits for this batch's poses only
            sd.exchange_pose_records(out["poses"], out["s_t"], out["s_q"],
                                     stream=out.get("stream") or torch.cuda.current_stream())
        return out

    for _ in range(max(args.warmup, 1)):
        step()
    torch.cuda.synchronize()

    # dominant kernel class: one fully profiled step after warm-up
    L = _lib.lib()
    L.spe_model_profile_begin(model._h, b"")
    step()
    n = L.spe_model_profile_end(model._h)
    tot = {}
    kb = ctypes.create_string_buffer(64)
    ms, fl, by = ctypes.c_double(), ctypes.c_double(), ctypes.c_double()
    table = []
    for i in range(n):
        L.spe_model_profile_get(model._h, i, kb, 64, ctypes.byref(ms), ctypes.byref(fl), ctypes.byref(by))
        k = kb.value.decode()
        t = tot.setdefault(k, [0.0, 0])
        t[0] += ms.value
        t[1] += 1
        floor_ms = 1e3 * max(fl.value / (peak_for(dtype, k, cfg.num_queries) * 1e12), by.value / (PEAK["hbm"] * 1e9))
        table.append({"i": i, "kind": k, "ms": ms.value, "flops": fl.value, "bytes": by.value,
                      "floor_ms": floor_ms, "frac": floor_ms / max(ms.value, 1e-9)})
    dominant = max(tot, key=lambda k: tot[k][0])
    if launch_table and int(os.environ.get("RANK", "0")) == 0:
        with open(launch_table, "w") as f:
            json.dump(table, f, indent=0)

    # ---- timed region: K steps, dominant kernel bracketed with HIP events on its stream
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    L.spe_model_profile_begin(model._h, dominant.encode())
    t0 = time.perf_counter()
    for _ in range(args.steps):
        out = step()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    if world > 1:
        dist.barrier()
    n = L.spe_model_profile_end(model._h)
    k_ms, k_fl, k_by, k_n = 0.0, 0.0, 0.0, 0
    for i in range(n):
        L.spe_model_profile_get(model._h, i, kb, 64, ctypes.byref(ms), ctypes.byref(fl), ctypes.byref(by))
        if kb.value.decode() == dominant:
            k_ms += ms.value; k_fl += fl.value; k_by += by.value; k_n += 1
    elapsed = torch.tensor([t1 - t0], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(elapsed, op=dist.ReduceOp.MAX)
    elapsed = float(elapsed.item())

    avg_ms = k_ms / max(k_n, 1)
    # bound by the class's own arithmetic intensity against the ridge point (2500 TF/s / 8 TB/s
    # = 312 flop/B): the K <= 256 1x1 convs are HBM-bound, attention / FFN / 3x3 convs MFMA-bound
    mfma_bound = k_fl * PEAK["hbm"] * 1e9 > k_by * peak_for(dtype, dominant, cfg.num_queries) * 1e12
    if mfma_bound:
        achieved = (k_fl / max(k_n, 1)) / (avg_ms * 1e-3) / 1e12
        peak, unit = peak_for(dtype, dominant, cfg.num_queries), "TFLOP/s"
    else:
        achieved = (k_by / max(k_n, 1)) / (avg_ms * 1e-3) / 1e9
        peak, unit = PEAK["hbm"], "GB/s"
    prof_ms = tot[dominant][0] / max(tot[dominant][1], 1)
    # (fp32x3 / fp32x6 / fp32h3: K / V^T pre-split by the projections in the 16-bit key order -> the
    # LDS-DMA split kernel attn_split.hip, fp16 V planes in fp32h3; SPE_ATTN_PRESPLIT=0: attn_x3_kernel)
    split = os.environ.get("SPE_ATTN_PRESPLIT", "1") != "0" and cfg.tokens % 16 == 0
    sym3 = "attn_split_kernel<false>" if split else "attn_x3_kernel<false>"
    symbol = ({"fp32": "attn_f32_kernel", "fp32x3": sym3, "fp32x6": sym3,
               "fp32h3": "attn_split_kernel<true>" if split else "attn_x3_kernel<false>"}[dtype]
              if dominant == "attn.enc" and dtype != "bf16" else
              KIND_SYMBOL.get(dominant, dominant).replace("DF16b", "DF16_" if attn_dtype == "fp16" else "DF16b"))
    roofline = {"kernel": dominant, "kernel_symbol": symbol,
                "bound": "mfma" if mfma_bound else "hbm", "achieved": achieved,
                "peak": peak, "unit": unit, "frac": achieved / peak,
                "traffic": traffic_for(dominant, launch_grid(dominant, B, cfg), attn_dtype),
                "launches": k_n, "avg_launch_ms": avg_ms,
                # the timed-region launches share the CUs with the next batch's backbone (stream
                # overlap); the per-launch profiled step times each launch between events on its
                # stream, the kernel's own rate
                "avg_launch_ms_profiled_step": prof_ms,
                "frac_profiled_step": ((k_fl if mfma_bound else k_by) / max(k_n, 1)) / (prof_ms * 1e-3) /
                                      (1e12 if mfma_bound else 1e9) / peak,
                "algorithmic_flops_per_launch": k_fl / max(k_n, 1),
                "algorithmic_bytes_per_launch": k_by / max(k_n, 1)}
    return {"elapsed": elapsed, "out": out, "roofline": roofline,
            "kernel_time_ms_per_step": {k: v[0] for k, v in sorted(tot.items(), key=lambda kv: -kv[1][0])}}


def _lib_mode_ceres():
    from spe import _lib
    return _lib.SPE_PNP_EPNP_CERES


def host_input_line(args, model, solver, cfg, world, rank, dev, overlap, B):
    """The timed step fed the way the reference's evaluate() loop is (REV/engine.py:92,
    samples.to(device)): every step's batch -- the 8-bit grayscale crops [B,S,S] that to_tensor +
    Normalize turn into the model input (spe_forward_stages_u8 normalises them in the stem's input
    pack), boxes and ground truth -- comes from pinned host memory through an H2D copy on a copy
    stream, overlapped with the previous batch's compute.  Two pool batches alternate."""
    import torch
    from spe.pipeline import PosePipeline
    from spe.synthetic import bench_images
    pool = bench_images(cfg, rank * B, 2 * B)
    pipe = PosePipeline(model, solver, B, device=dev, host_input=True, **overlap)
    pipe.load_host(torch.from_numpy(pool["crops_u8"]), torch.from_numpy(pool["clip_bbox"]),
                   torch.from_numpy(pool["quat"]), torch.from_numpy(pool["tvec"]))
    torch.cuda.synchronize()
    tm = time_mode(pipe, model, args, world, dev, args.dtype, args.attn_dtype, cfg, B)
    # the PCIe rate of one batch's crops alone (pinned -> device, no compute beside it)
    h, d = pipe.host["crops"][:B], pipe.dev_crops[0]
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10):
        d.copy_(h, non_blocking=True)
    e1.record()
    torch.cuda.synchronize()
    copy_ms = e0.elapsed_time(e1) / 10
    res = {"value": B * world * args.steps / tm["elapsed"], "unit": "images/s",
           "ms_per_step": 1e3 * tm["elapsed"] / args.steps,
           "input": f"8-bit grayscale crops [B,{cfg.input_size},{cfg.input_size}] + boxes + ground truth in pinned "
                    "host memory, copied H2D every step on a copy stream (REV/engine.py:92); normalised on the "
                    "device in the stem's input pack (bit-identical to the fp32 batch)",
           "h2d_bytes_per_step": pipe.h2d_bytes,
           "fp32_batch_bytes_per_step": B * 3 * cfg.input_size ** 2 * 4,
           "h2d_copy_ms_alone": copy_ms, "h2d_GBps_alone": pipe.dev_crops[0].numel() / copy_ms / 1e6,
           "kernel_time_ms_per_step": tm["kernel_time_ms_per_step"],
           "dominant_avg_launch_ms": tm["roofline"]["avg_launch_ms"]}
    del pipe
    torch.cuda.synchronize()
    return res


def bench_weights_for(args, cfg, rcfg, rank, world, dev):
    """(weights, fit info, provenance) of a bench run.  DETR pose-consistent weights come from the
    committed head fixture when one exists for the shape (spe.synthetic.fixed_bench_weights:
    computed once from the torch-fp32 CPU restatement, independent of every kernel, device and rank
    count); other shapes calibrate the class head and fit the point head with the exact-f32 mode on
    the fixed bench pool (pose_consistent_weights)."""
    import numpy as np
    import torch
    from spe.models import DETR
    from spe.synthetic import (CALIB_SEED, bench_images, bench_weights, diversify_class_head, fixed_bench_weights,
                               random_weights, synthetic_batch)
    fit = None
    if rcfg is not None:
        from spe.rtdetr import RTDETR
        from spe.rtdetr_spec import random_rtdetr_weights
        w = random_rtdetr_weights(rcfg, 0)
        if args.weights in ("label-diverse", "pose-consistent"):
            # RT-DETR's queries are distinct encoder tokens already; only the last score head is
            # drawn in the principal subspace of its input (spe.synthetic.diversify_class_head),
            # calibrated by the exact-f32 mode on the first 64 pool images (identical on every rank)
            m = RTDETR(rcfg, dtype="fp32", aux_outputs=False)
            m.load_state_dict(w)
            x = torch.from_numpy(bench_images(cfg, 0, 64)["images"]).to(dev)
            hs = m(x, return_hs=True)["hs"].cpu().numpy()
            del m
            # the selected queries of one image sit close together (top-k encoder tokens of a
            # random-init encoder): the head's directions come from the within-image spread, off
            # the span of the image means, or every query of an image gets the same one to three
            # labels and the solver stops at its fewer-than-4-correspondences check
            w = diversify_class_head(w, hs, head=f"decoder.dec_score_head.{rcfg.dec_layers - 1}", within_image=True)
        if args.weights == "pose-consistent":
            w, fit = pose_consistent_weights(w, cfg, rank, world, dev, rcfg=rcfg)
        return w, fit, "exact-f32 calibration on the bench pool"
    if args.weights == "random":
        return random_weights(cfg, 0), None, "random init"
    if args.weights == "pose-consistent":
        w, meta = fixed_bench_weights(cfg, 0)
        if w is not None:
            fit = {k: meta[k] for k in ("fit_err_max_norm", "fit_err_mean_norm", "fg_queries")}
            fit["fit_set"] = f"bench pool images 0..{meta['pool'] - 1}"
            return w, fit, "committed head fixture (" + meta["generator"] + ")"

    def hs_fn(ww, images):
        m = DETR(cfg, dtype="fp32")
        m.load_state_dict(ww)
        hs = m(torch.from_numpy(images).to(dev), return_hs=True)["hs"].cpu().numpy()
        del m
        return hs
    w = bench_weights(cfg, 0, hs_fn)
    if args.weights == "pose-consistent":
        w, fit = pose_consistent_weights(w, cfg, rank, world, dev)
    _ = (np, synthetic_batch, CALIB_SEED)
    return w, fit, "exact-f32 calibration on the bench pool"


def north_star_line(args, cfg, w, world, rank, dev, overlap):
    """BASELINE north_star: "bs=256 over 8 GPUs, RANSAC-PnP + GN refinement, within 1e-4".  The
    global batch of 256 pool images is sharded 256/N per rank (same images at every N), solved
    with P3P-RANSAC + LM (SimplePoseSolver, REV/utils/speed_eval.py:209-230), timed in bf16 and in
    the accuracy-contract mode, each with its accuracy against the exact-f32 mode over all 256
    images (REV/main.py:213-217,239-244 launch one process per GPU the same way)."""
    import argparse as ap
    import torch
    from spe.models import DETR
    from spe.pipeline import PosePipeline
    from spe.solver import build_solver
    G = NORTH_STAR_GLOBAL_BATCH
    if G % world:
        return {"skipped": f"global batch {G} does not split over {world} ranks"}
    nb = G // world
    data = bench_data(cfg, nb, rank)
    solver = build_solver(ap.Namespace(solver="ransac_p3p_lm", repro=20))
    ref = Fp32Reference(cfg, w, data, solver, dev)
    sargs = ap.Namespace(**vars(args))
    sargs.steps = min(args.steps, 10)
    res = {"global_batch": G, "per_gpu_batch": nb, "n_gpus": world, "input_size": cfg.input_size,
           "num_queries": cfg.num_queries, "solver": "ransac_p3p_lm", "steps": sargs.steps, "modes": {}}
    for dt in ("bf16", args.parity_dtype):
        m = DETR(cfg, dtype=dt, attn_dtype=dt)
        m.load_state_dict(w)
        pipe = PosePipeline(m, solver, nb, device=dev, **overlap)
        pipe.load(torch.from_numpy(data["images"]).to(dev), torch.from_numpy(data["clip_bbox"]).float().to(dev),
                  torch.from_numpy(data["quat"]).to(dev), torch.from_numpy(data["tvec"]).to(dev))
        torch.cuda.synchronize()
        t = time_mode(pipe, m, sargs, world, dev, dt, dt, cfg, nb)
        hdr = result_header(sargs, world, t["elapsed"], nb, dt)
        st = t["out"]["poses"]["status"]
        counts = torch.stack([(st == s).sum() for s in range(5)])
        if world > 1:
            torch.distributed.all_reduce(counts)
        res["modes"][dt] = {"value": hdr["value"], "unit": "images/s", "value_per_gpu": hdr["value"] / world,
                            "ms_per_step": hdr["ms_per_step"], "roofline_frac": t["roofline"]["frac"],
                            "roofline_kernel": t["roofline"]["kernel"],
                            "solver_status_counts": {str(s): int(c) for s, c in enumerate(counts.tolist())},
                            "accuracy_vs_fp32": accuracy_vs_fp32(m, ref, t["out"], world, "ransac_p3p_lm")}
        del pipe, m
        torch.cuda.synchronize()
        torch.cuda.empty_cache()
    del ref
    torch.cuda.empty_cache()
    return res


def main():
    args = parse()
    if os.environ.get("SPE_BENCH_STUB"):
        if args.gpus > 1 and "RANK" not in os.environ:
            return launch_ranks(args)
        return stub_worker(args)
    if args.gpus > 1 and "RANK" not in os.environ:
        return launch_ranks(args)
    import torch
    import torch.distributed as dist
    from spe import dist as sd
    from spe.config import SpeConfig
    from spe.models import DETR
    from spe.pipeline import PosePipeline
    from spe.solver import build_solver
    import numpy as np
    from spe.synthetic import weights_checksum

    rank, world, local = sd.init_distributed_mode()
    if world != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but the launch has world size {world}", file=sys.stderr)
        return 2
    if os.environ.get("SPE_BENCH_SHARE_GPU") == "1":
        # rehearsal of the N-rank path on fewer GPUs (with SPE_DIST_BACKEND=gloo): ranks share devices
        local = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    cfg = SpeConfig(input_size=args.size, num_queries=args.queries, enc_layers=args.layers, dec_layers=args.layers,
                    sigma_head=bool(args.sigma_head))
    B = args.batch

    rcfg = None
    if args.model != "detr":
        from spe.rtdetr import RTDETR
        from spe.rtdetr_spec import RtdetrConfig
        rcfg = RtdetrConfig(depth=18 if args.model == "rtdetr_r18" else 50, input_size=args.size,
                            num_queries=args.queries, dec_layers=args.layers)
    w, fit, wsource = bench_weights_for(args, cfg, rcfg, rank, world, dev)
    if rcfg is not None:
        model = RTDETR(rcfg, dtype=args.dtype, aux_outputs=False)
    else:
        model = DETR(cfg, dtype=args.dtype, attn_dtype=args.attn_dtype)
    model.load_state_dict(w)
    solver = build_solver(argparse.Namespace(solver=args.solver, repro=20))
    overlap = dict(overlap=not args.no_overlap,
                   overlap_decode=rcfg is None and not (args.no_overlap_decode or args.no_overlap),
                   overlap_backbone=rcfg is None and not (args.no_overlap_backbone or args.no_overlap_decode or args.no_overlap))
    jpeg_bytes = 0
    if args.raw_frames:
        from spe.synthetic import synthetic_frames
        data = synthetic_frames(B, seed=1000 + rank)
        H, W = data["frames"].shape[1:3]
        files = None
        if args.jpeg:
            import io
            from PIL import Image
            from spe.datasets import JpegDecoder

            def enc(a):
                bio = io.BytesIO()
                Image.fromarray(a).save(bio, "JPEG", quality=90)
                return bio.getvalue()
            files = [enc(f) for f in data["frames"]]
        pipe = PosePipeline(model, solver, B, device=dev, overlap=not args.no_overlap,
                            overlap_decode=not (args.no_overlap_decode or args.no_overlap), raw_frames=(H, W, 1),
                            overlap_backbone=not (args.no_overlap_backbone or args.no_overlap_decode or args.no_overlap),
                            jpeg_max_bytes=max(len(f) for f in files) if files else 0)
        if files:
            jpeg_bytes = sum(len(f) for f in files)
            pipe.load_jpeg(*JpegDecoder.pack(files, dev), torch.from_numpy(data["bbox_xxyy"]).to(dev),
                           torch.from_numpy(data["quat"]).to(dev), torch.from_numpy(data["tvec"]).to(dev),
                           area=image_areas(data, solver))
        else:
            pipe.load_frames(torch.from_numpy(data["frames"]).to(dev), torch.from_numpy(data["bbox_xxyy"]).to(dev),
                             torch.from_numpy(data["quat"]).to(dev), torch.from_numpy(data["tvec"]).to(dev),
                             area=image_areas(data, solver))
    else:
        pipe = PosePipeline(model, solver, B, device=dev, **overlap)
        data = bench_data(cfg, B, rank)
        pipe.load(torch.from_numpy(data["images"]).to(dev), torch.from_numpy(data["clip_bbox"]).float().to(dev),
                  torch.from_numpy(data["quat"]).to(dev), torch.from_numpy(data["tvec"]).to(dev),
                  area=image_areas(data, solver))
    torch.cuda.synchronize()

    host = None
    host_ok = (rcfg is None and not args.raw_frames and not args.no_host_input
               and getattr(solver, "mode", None) != _lib_mode_ceres())
    if host_ok and not args.host_input_last:
        host = host_input_line(args, model, solver, cfg, world, rank, dev, overlap, B)
    tm = time_mode(pipe, model, args, world, dev, args.dtype, args.attn_dtype, cfg, B, args.launch_table)
    out = tm["out"]
    score = float((out["s_t"] + out["s_q"]).mean().item())
    status = out["poses"]["status"].cpu()

    # ---- host input: the same step with every batch copied from pinned host memory
    if host_ok:
        if host is None:
            host = host_input_line(args, model, solver, cfg, world, rank, dev, overlap, B)
        host["value_vs_device_resident"] = host["value"] / (B * world * args.steps / tm["elapsed"])
        host["timed_before_device_resident"] = not args.host_input_last

    # ---- parity mode: the same weights, batch and pipeline in the fast parity dtype, timed the
    # same way (its own steps between barriers), with its accuracy against the exact-f32 mode
    parity = None
    want_parity = (rcfg is None and not args.raw_frames and not args.no_parity and args.parity_dtype != args.dtype)
    ref = None
    if rcfg is None and not args.raw_frames and not args.no_accuracy and (args.dtype != "fp32" or want_parity):
        ref = Fp32Reference(cfg, w, data, solver, dev)
    acc = (accuracy_vs_fp32(model, ref, out, world, args.solver, args.config)
           if (ref is not None and args.dtype != "fp32") else None)
    if want_parity:
        del pipe
        pm = DETR(cfg, dtype=args.parity_dtype)
        pm.load_state_dict(w)
        ppipe = PosePipeline(pm, solver, B, device=dev, **overlap)
        ppipe.load(torch.from_numpy(data["images"]).to(dev), torch.from_numpy(data["clip_bbox"]).float().to(dev),
                   torch.from_numpy(data["quat"]).to(dev), torch.from_numpy(data["tvec"]).to(dev),
                   area=image_areas(data, solver))
        torch.cuda.synchronize()
        pt = time_mode(ppipe, pm, args, world, dev, args.parity_dtype, args.parity_dtype, cfg, B)
        parity = {k: v for k, v in result_header(args, world, pt["elapsed"], B, args.parity_dtype).items()
                  if k in ("value", "unit", "ms_per_step", "dtype")}
        parity["value_per_gpu"] = parity["value"] / world
        parity["mode"] = PARITY_MODE_TEXT.get(args.parity_dtype, args.parity_dtype)
        parity["roofline"] = pt["roofline"]
        parity["kernel_time_ms_per_step"] = pt["kernel_time_ms_per_step"]
        if ref is not None:
            parity["accuracy_vs_fp32"] = accuracy_vs_fp32(pm, ref, pt["out"], world, args.solver, args.config)
        del ppipe, pm
        torch.cuda.synchronize()
        torch.cuda.empty_cache()

    # ---- the north-star shape (global bs 256, RANSAC-P3P + LM) for multi-GPU runs
    ns = None
    if (rcfg is None and not args.raw_frames and not args.no_north_star and (world > 1 or args.north_star)
            and (cfg.input_size, cfg.num_queries, cfg.enc_layers) == (416, 11, 6)):
        ns = north_star_line(args, cfg, w, world, rank, dev, overlap)

    if rank != 0:
        if dist.is_initialized():
            dist.destroy_process_group()
        return 0
    result = result_header(args, world, tm["elapsed"], B, args.dtype)
    result.update({
        "data": f"synthetic (seeded SPEED-shaped {('1920x1200 grayscale JPEG files (q90) + detector boxes, on-device decode + val transform' if args.jpeg else '1920x1200 8-bit frames + detector boxes, on-device val transform') if args.raw_frames else 'crops from a fixed 256-image pool'}; "
                f"{args.weights} random-init weights, no checkpoint exists in the reference)",
        "config": {"workload": (CONFIG_NAME[args.config].format(L=args.layers, Q=args.queries, S=args.size,
                                                                 solver=args.solver, A=args.attn_dtype) if rcfg is None else
                                f"UNC RT-DETR r{rcfg.depth}vd + HybridEncoder + {args.layers}-layer deformable decoder "
                                f"with sigma head, {args.queries} queries, {args.size}x{args.size}, sigma-weighted "
                                f"EPnP-RANSAC + self-assessment (solver={args.solver}; SURVEY 8f.4, not a BASELINE config)"),
                   "global_batch": B * world, "per_gpu_batch": B, "input_size": args.size,
                   **({"jpeg_bytes_per_step": jpeg_bytes} if args.raw_frames and args.jpeg else {}),
                   "num_queries": args.queries,
                   # bf16 models' encoder attention keeps q/k bf16 and runs V^T and P in fp16 (finer
                   # mantissa than bf16; attention.hip TV)
                   "attention_dtype": ("bf16 q/k, fp16 V/P" if args.attn_dtype == "bf16" and args.dtype == "bf16"
                                       and os.environ.get("SPE_ATTN_F16V", "1") != "0" else args.attn_dtype),
                   "parallelism": f"dp{world} (image sharding)"},
        "weights_sha256_16": weights_checksum(w),
        "weights_source": wsource,
        "roofline": tm["roofline"],
        "kernel_time_ms_per_step": tm["kernel_time_ms_per_step"],
        "speed_score_mean_random_weights": score,
        "solver_status_counts": {str(s): int((status == s).sum()) for s in range(5)},
    })
    if "assess" in out:
        result["self_assessment_reliable"] = int(out["assess"]["reliable"].sum().item())
    if not args.raw_frames and "points_px" in out["forward"] and "probs" in out["forward"]:
        e = keypoint_error_px(out["forward"]["points_px"], out["forward"]["probs"], data)
        result["keypoints_vs_gt_px"] = {"median": float(np.median(e)), "p90": float(np.percentile(e, 90)),
                                        "fg_queries": int(e.size), "weights": args.weights}
        if fit is not None:
            # the point head is fitted on the bench pool, which holds the timed images: these are
            # fit-set (training-set) errors, not held-out accuracy
            result["keypoints_vs_gt_px"].update(fit)
        if acc is not None:
            result["accuracy_vs_fp32"] = acc
    if host is not None:
        result["value_host_input"] = host["value"]
        result["host_input"] = host
    if parity is not None:
        result["parity_mode"] = parity
    if ns is not None:
        result["north_star"] = ns
    if world == 1 and not args.no_cpu_baseline:
        result["cpu_baseline"] = (cpu_baseline(cfg, args.cpu_seconds, args.solver) if rcfg is None
                                  else cpu_baseline_rtdetr(rcfg, args.cpu_seconds))
    print(json.dumps(result))
    if dist.is_initialized():
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
