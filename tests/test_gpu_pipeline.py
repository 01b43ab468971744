"""GPU: end-to-end evaluate() path (model -> fused PostProcess -> batched solver -> score) and
its agreement with the reference-style per-image path and the CPU oracles."""
import argparse

import numpy as np
import pytest
import torch

from spe.config import SpeConfig, Camera, world_points
from spe.synthetic import bench_weights, synthetic_batch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def small_model(gpu_device):
    from spe.models import DETR
    cfg = SpeConfig(input_size=128, num_queries=11, enc_layers=2, dec_layers=2)

    def hs_fn(w, images):
        m = DETR(cfg, dtype="fp32")
        m.load_state_dict(w)
        return m(torch.from_numpy(images).to(gpu_device), return_hs=True)["hs"].cpu().numpy()

    w = bench_weights(cfg, 3, hs_fn)
    m = DETR(cfg, dtype="fp32")
    m.load_state_dict(w)
    return cfg, w, m


def test_label_diverse_weights_feed_the_solver(gpu_device, small_model):
    cfg, w, m = small_model
    b = synthetic_batch(cfg, 16, 21)
    o = m(torch.from_numpy(b["images"]).to(gpu_device), clip_bbox=torch.from_numpy(b["clip_bbox"]).float().to(gpu_device))
    labels = o["probs"].argmax(-1).cpu().numpy()
    n_fg = np.array([len(set(l.tolist()) - {11}) for l in labels])
    assert (n_fg >= 4).mean() >= 0.5


def test_batched_solver_equals_per_image_solver(gpu_device, small_model):
    """solve_batch over the fused PostProcess outputs == reference-style per-image solver calls
    on PostProcess's numpy dicts == CPU oracle."""
    import pnp_ref
    from spe.models import PostProcess
    from spe.solver import SimplePoseSolver, SolverError
    cfg, w, m = small_model
    b = synthetic_batch(cfg, 12, 22)
    img = torch.from_numpy(b["images"]).to(gpu_device)
    clip = torch.from_numpy(b["clip_bbox"]).float().to(gpu_device)
    o = m(img, clip_bbox=clip)
    solver = SimplePoseSolver(argparse.Namespace(repro=20))
    batched = solver.solve_batch(o["points_px"], o["probs"])
    pp = PostProcess()(o, [c for c in b["clip_bbox"]])
    ref = pnp_ref.pnp_batch(np.stack([r["points"] for r in pp]), np.stack([r["logits"] for r in pp]), Camera.K,
                            world_points(), mode=pnp_ref.MODE_RANSAC_P3P_LM)
    st = batched["status"].cpu().numpy()
    np.testing.assert_array_equal(st, ref["status"])
    for i, r in enumerate(pp):
        try:
            q, t = solver(r["points"], r["logits"])
        except (IndexError, SolverError):
            assert st[i] in (1, 2, 4)
            continue
        np.testing.assert_allclose(q, batched["quat"][i].double().cpu().numpy(), atol=1e-7)
        np.testing.assert_allclose(t, batched["tvec"][i].cpu().numpy(), rtol=1e-9, atol=1e-9)
        np.testing.assert_allclose(t, ref["tvec"][i], rtol=1e-6, atol=1e-6)


def test_evaluate_matches_reference_style_speedeval(gpu_device, small_model):
    from spe.engine import evaluate
    from spe.misc import NestedTensor
    from spe.models import PostProcess
    from spe.solver import build_solver
    from spe.speed_eval import SpeedEval
    cfg, w, m = small_model
    b = synthetic_batch(cfg, 10, 23)
    names = [f"img{i:03d}.jpg" for i in range(10)]
    gt = [{"filename": n, "q_vbs2tango": b["quat"][i].tolist(), "r_Vo2To_vbs_true": b["tvec"][i].tolist()}
          for i, n in enumerate(names)]
    loader = []
    for s in range(0, 10, 4):
        x = torch.from_numpy(b["images"][s:s + 4])
        tg = [{"filename": names[i], "clip_bbox": torch.as_tensor(b["clip_bbox"][i])} for i in range(s, min(s + 4, 10))]
        loader.append((NestedTensor(x, torch.zeros(x.shape[0], 128, 128, dtype=torch.bool)), tg))
    solver = build_solver(argparse.Namespace(repro=20, solver="ransac_p3p_lm"))
    stats, ev = evaluate(m, None, {"points": PostProcess()}, loader, gt, solver, gpu_device, None)
    # reference-style path: PostProcess dicts -> per-image solver -> SpeedEval.update
    ev2 = SpeedEval(gt, solver)
    for x, tg in loader:
        out = m(x.tensors.to(gpu_device))
        pp = PostProcess()(out, [t["clip_bbox"] for t in tg])
        ev2.update({t["filename"]: r for t, r in zip(tg, pp)})
    ev2.summarize()
    for n in names:
        a, c = ev.log[n], ev2.log[n]
        assert a["quat_pr"] == c["quat_pr"] and a["tvec_pr"] == c["tvec_pr"]
        assert abs(a["score"] - c["score"]) < 1e-7
    assert stats["speed_eval_pose"] == ev2.stats


@pytest.mark.parametrize("solver_name", ["epnp", "ransac_p3p_lm"])
def test_overlapped_pipeline_equals_serial(gpu_device, small_model, solver_name):
    """Solver of batch i on the second stream while the forward of batch i+1 runs: after wait(),
    every batch's poses / scores equal the single-stream pipeline's (same inputs, same kernels;
    each batch loads its own ground truth, which the next load() overwrites while the previous
    batch's score may still be queued)."""
    from spe.pipeline import PosePipeline
    from spe.solver import build_solver
    cfg, w, m = small_model
    B = 8
    solver = build_solver(argparse.Namespace(solver=solver_name, repro=20))
    batches = [synthetic_batch(cfg, B, 40 + i) for i in range(3)]
    res = {}
    for ov in (False, True):
        pipe = PosePipeline(m, solver, B, device=gpu_device, overlap=ov)
        outs = []
        for b in batches:
            pipe.load(torch.from_numpy(b["images"]).to(gpu_device), torch.from_numpy(b["clip_bbox"]).float().to(gpu_device),
                      torch.from_numpy(b["quat"]).to(gpu_device), torch.from_numpy(b["tvec"]).to(gpu_device))
            outs.append(pipe.run())
        for o in outs:
            pipe.wait(o)
        res[ov] = [(o["poses"]["status"].cpu().numpy(), o["poses"]["tvec"].cpu().numpy(), o["s_t"].cpu().numpy(),
                    o["s_q"].cpu().numpy()) for o in outs]
    for r0, r1 in zip(res[False], res[True]):
        for x0, x1 in zip(r0, r1):
            np.testing.assert_array_equal(x0, x1)


def test_pipeline_from_raw_frames(gpu_device, small_model):
    """Raw-frame mode (device validation transform -> model -> solver) == the same pipeline fed
    with the oracle's preprocessed images and clip boxes: identical poses and statuses."""
    import preprocess_ref as pr
    from spe.pipeline import PosePipeline
    from spe.solver import build_solver
    from spe.synthetic import synthetic_frames
    cfg, w, m = small_model
    B = 6
    d = synthetic_frames(B, seed=31)
    solver = build_solver(argparse.Namespace(solver="ransac_p3p_lm", repro=20))
    raw = PosePipeline(m, solver, B, device=gpu_device, raw_frames=d["frames"].shape[1:3] + (1,))
    raw.load_frames(torch.from_numpy(d["frames"]).to(gpu_device), torch.from_numpy(d["bbox_xxyy"]).to(gpu_device))
    a = raw.run()
    torch.cuda.synchronize()
    ref = pr.preprocess(d["frames"], d["bbox_xxyy"], cfg.input_size)
    assert np.array_equal(raw.images.cpu().numpy(), ref["images"])
    pre = PosePipeline(m, solver, B, device=gpu_device)
    pre.load(torch.from_numpy(ref["images"]).to(gpu_device), torch.from_numpy(ref["clip_bbox"]).float().to(gpu_device))
    b = pre.run()
    torch.cuda.synchronize()
    for k in ("status", "quat", "tvec"):
        assert torch.equal(a["poses"][k], b["poses"][k]), k


def test_encode_parts_match_forward(gpu_device, small_model):
    """BACKBONE then TRANSFORMER (spe_forward_stages bits 4, 8) then DECODE in one workspace
    equals the one-call forward bit for bit."""
    cfg, w, m = small_model
    B = 4
    b = synthetic_batch(cfg, B, 77)
    x = torch.from_numpy(b["images"]).to(gpu_device)
    clip = torch.from_numpy(b["clip_bbox"]).float().to(gpu_device)
    ref = m(x, clip_bbox=clip)
    ws = m.new_workspace(B, gpu_device)
    m.encode(x, ws, part="backbone")
    m.encode(None, ws, part="transformer", B=B)
    out = m.decode(B, ws, clip_bbox=clip)
    torch.cuda.synchronize()
    for k in ("pred_logits", "pred_points", "probs", "points_px"):
        assert torch.equal(out[k], ref[k]), k


@pytest.mark.parametrize("backbone", [False, True])
def test_pipeline_overlap_decode_matches_serial(gpu_device, small_model, backbone):
    """Decoder of batch i on its own stream beside the encoder of batch i+1 (two workspaces,
    per-slot snapshots of clip boxes / ground truth) -- and with `backbone`, batch i's encoder
    layers on a fourth stream beside batch i+1's backbone (three workspaces): every batch's poses
    and scores equal the serial
    pipeline's, over consecutive batches that reuse every slot."""
    from spe.pipeline import PosePipeline
    from spe.solver import build_solver
    cfg, w, m = small_model
    B = 8
    solver = build_solver(argparse.Namespace(solver="ransac_p3p_lm", repro=20))
    serial = PosePipeline(m, solver, B, device=gpu_device)
    staged = PosePipeline(m, solver, B, device=gpu_device, overlap_decode=True, overlap_backbone=backbone)
    batches = [synthetic_batch(cfg, B, 500 + k) for k in range(7 if backbone else 4)]
    dev = gpu_device

    def load(p, b):
        p.load(torch.from_numpy(b["images"]).to(dev), torch.from_numpy(b["clip_bbox"]).float().to(dev),
               torch.from_numpy(b["quat"]).to(dev), torch.from_numpy(b["tvec"]).to(dev))

    outs = []
    for b in batches:                    # enqueue all batches back to back, no host sync between
        load(staged, b)
        outs.append(staged.run())
    torch.cuda.synchronize()
    for b, o in zip(batches, outs):
        load(serial, b)
        r = serial.run()
        torch.cuda.synchronize()
        for k in ("status", "quat", "tvec"):
            assert torch.equal(o["poses"][k], r["poses"][k]), k
        assert torch.equal(o["s_t"], r["s_t"]) and torch.equal(o["s_q"], r["s_q"])


def test_pipeline_graph_sigma_matches_eager(gpu_device):
    """use_graph=True with the sigma head and the sigma-weighted EPnP-RANSAC solver (whose
    hypothesis scratch lives in per-stream device memory): warm-up and capture share one stream,
    so the replayed graph reuses the warmed-up workspace / scratch, and every replay over new
    inputs equals the eager pipeline."""
    from spe.models import DETR
    from spe.pipeline import PosePipeline
    from spe.solver import build_solver
    cfg = SpeConfig(input_size=128, num_queries=11, enc_layers=2, dec_layers=2, sigma_head=True)

    def hs_fn(w, images):
        mm = DETR(cfg, dtype="bf16")
        mm.load_state_dict(w)
        return mm(torch.from_numpy(images).to(gpu_device), return_hs=True)["hs"].cpu().numpy()

    w = bench_weights(cfg, 5, hs_fn)
    m = DETR(cfg, dtype="bf16")
    m.load_state_dict(w)
    B = 8
    solver = build_solver(argparse.Namespace(solver="epnp_ransac_sigma", repro=25))
    eager = PosePipeline(m, solver, B, device=gpu_device)
    graph = PosePipeline(m, solver, B, device=gpu_device, use_graph=True)
    dev = gpu_device
    for k in range(3):
        b = synthetic_batch(cfg, B, 700 + k)
        res = []
        for p in (eager, graph):
            p.load(torch.from_numpy(b["images"]).to(dev), torch.from_numpy(b["clip_bbox"]).float().to(dev),
                   torch.from_numpy(b["quat"]).to(dev), torch.from_numpy(b["tvec"]).to(dev))
            o = p.run()
            torch.cuda.synchronize()
            res.append({"status": o["poses"]["status"].clone(), "quat": o["poses"]["quat"].clone(),
                        "tvec": o["poses"]["tvec"].clone(), "s_t": o["s_t"].clone(),
                        "reliable": o["assess"]["reliable"].clone()})
        for key in res[0]:
            assert torch.equal(res[0][key], res[1][key]), (k, key)
    assert graph.graph is not None


def test_pipeline_from_jpeg_matches_raw_frames(gpu_device, small_model):
    """JPEG mode (device decode -> validation transform -> model -> solver) == the raw-frame
    pipeline fed with Pillow's decode of the same files."""
    import io
    from PIL import Image
    from spe.datasets import JpegDecoder
    from spe.pipeline import PosePipeline
    from spe.solver import build_solver
    from spe.synthetic import synthetic_frames
    cfg, w, m = small_model
    B = 4
    d = synthetic_frames(B, seed=41)
    files = []
    for f in d["frames"]:
        bio = io.BytesIO()
        Image.fromarray(f).save(bio, "JPEG", quality=90)
        files.append(bio.getvalue())
    dec = np.stack([np.asarray(Image.open(io.BytesIO(f))) for f in files])
    solver = build_solver(argparse.Namespace(solver="ransac_p3p_lm", repro=20))
    hw = d["frames"].shape[1:3]
    jp = PosePipeline(m, solver, B, device=gpu_device, raw_frames=hw + (1,), jpeg_max_bytes=max(map(len, files)))
    jp.load_jpeg(*JpegDecoder.pack(files, gpu_device), torch.from_numpy(d["bbox_xxyy"]).to(gpu_device))
    a = jp.run()
    raw = PosePipeline(m, solver, B, device=gpu_device, raw_frames=hw + (1,))
    raw.load_frames(torch.from_numpy(dec).to(gpu_device), torch.from_numpy(d["bbox_xxyy"]).to(gpu_device))
    b = raw.run()
    torch.cuda.synchronize()
    assert torch.equal(jp.frames, raw.frames)
    for k in ("status", "quat", "tvec"):
        assert torch.equal(a["poses"][k], b["poses"][k]), k


@pytest.mark.parametrize("dtype", ["bf16", "fp32", "fp32h3"])
def test_u8_crops_equal_normalised_batch(gpu_device, small_model, dtype):
    """spe_forward_stages_u8: the 8-bit crops (grayscale [B,S,S] and RGB [B,S,S,3]) normalised in the
    stem's input pack give bit-identical outputs to the fp32 batch to_tensor + Normalize makes of
    them (REV/datasets/speed.py:25-41; numpy float32, the reference's operation order)."""
    from spe.models import DETR
    cfg, w, _ = small_model
    m = DETR(cfg, dtype=dtype)
    m.load_state_dict(w)
    b = synthetic_batch(cfg, 6, 77)
    dev = gpu_device
    clip = torch.from_numpy(b["clip_bbox"]).float().to(dev)
    mean = np.array([0.485, 0.456, 0.406], np.float32)
    std = np.array([0.229, 0.224, 0.225], np.float32)
    rgb = np.random.Generator(np.random.PCG64(5)).integers(0, 256, (6, cfg.input_size, cfg.input_size, 3), np.uint8)
    for crops in (b["crops_u8"], rgb):
        u = crops.astype(np.float32)
        if u.ndim == 3:
            u = u[..., None].repeat(3, -1)
        x = np.stack([(u[..., c] / np.float32(255) - mean[c]) / std[c] for c in range(3)], 1)
        if crops is b["crops_u8"]:
            assert np.array_equal(x, b["images"])
        ref = m(torch.from_numpy(x).to(dev), clip_bbox=clip)
        got = m(torch.from_numpy(crops).to(dev), clip_bbox=clip)
        torch.cuda.synchronize()
        for k in ("pred_logits", "pred_points", "points_px", "probs"):
            assert torch.equal(got[k], ref[k]), (dtype, crops.ndim, k)


@pytest.mark.parametrize("staged", [False, True])
def test_pipeline_host_input_matches_device_resident(gpu_device, small_model, staged):
    """Host-input pipeline (every run() copies the next pool batch's 8-bit crops, boxes and ground
    truth from pinned host memory on a copy stream; REV/engine.py:92) over consecutive batches that
    cycle the pool and reuse every slot: poses and scores bit for bit those of the device-resident
    pipeline fed each batch's fp32 images."""
    from spe.models import DETR
    from spe.pipeline import PosePipeline
    from spe.solver import build_solver
    cfg, w, _ = small_model
    m = DETR(cfg, dtype="bf16")
    m.load_state_dict(w)
    B, dev = 8, gpu_device
    solver = build_solver(argparse.Namespace(solver="ransac_p3p_lm", repro=20))
    kw = dict(overlap_decode=True, overlap_backbone=True) if staged else dict(overlap=True)
    host = PosePipeline(m, solver, B, device=dev, host_input=True, **kw)
    batches = [synthetic_batch(cfg, B, 900 + k) for k in range(3)]
    cat = {k: np.concatenate([bb[k] for bb in batches]) for k in ("crops_u8", "clip_bbox", "quat", "tvec")}
    host.load_host(torch.from_numpy(cat["crops_u8"]), torch.from_numpy(cat["clip_bbox"]),
                   torch.from_numpy(cat["quat"]), torch.from_numpy(cat["tvec"]))
    order = [0, 1, 2, 0, 1, 2, 0]                     # the pool cycles; 7 runs reuse all three slots
    outs = [host.run() for _ in order]
    torch.cuda.synchronize()
    ref = PosePipeline(m, solver, B, device=dev)
    for k, o in zip(order, outs):
        bb = batches[k]
        ref.load(torch.from_numpy(bb["images"]).to(dev), torch.from_numpy(bb["clip_bbox"]).float().to(dev),
                 torch.from_numpy(bb["quat"]).to(dev), torch.from_numpy(bb["tvec"]).to(dev))
        r = ref.run()
        torch.cuda.synchronize()
        for f in ("points_px", "probs"):
            assert torch.equal(o["forward"][f], r["forward"][f]), f
        for f in ("status", "quat", "tvec"):
            assert torch.equal(o["poses"][f], r["poses"][f]), f
        assert torch.equal(o["s_t"], r["s_t"]) and torch.equal(o["s_q"], r["s_q"])
    assert host.h2d_bytes == B * cfg.input_size ** 2 + B * 4 * 4 + B * 7 * 8
