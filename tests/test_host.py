"""CPU: host-side logic of the drop-in surface (no GPU compute).

SpeedEval log schema / rounding / failure mapping (REV/datasets/speed.py:337-421),
speed_score (REV/utils/speed_eval.py:245-262), NestedTensor batching (REV/utils/misc.py:287-333),
and the data-parallel record exchange over a world_size-2 gloo group.
"""
import json
import os

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

import pnp_ref
from spe import dist as sd
from spe.misc import NestedTensor, nested_tensor_from_tensor_list, collate_fn
from spe.speed_eval import SpeedEval, speed_score
from spe.solver import SolverError


class _StubSolver:
    """Returns a fixed pose, or raises what the reference's cv2 / indexing raises."""

    def __init__(self):
        self.calls = 0

    def __call__(self, points, logits):
        self.calls += 1
        if logits.shape[0] == 1:
            raise IndexError("no fg")
        if logits.shape[0] == 2:
            raise SolverError("cv2")
        return np.array([1.0, 0, 0, 0]), np.array([0.0, 0.0, 10.0])


def _gt():
    return [{"filename": f"img{i}.jpg", "q_vbs2tango": [1.0, 0, 0, 0], "r_Vo2To_vbs_true": [0.0, 0.0, 10.0 + i]}
            for i in range(3)]


def test_speed_score_matches_oracle():
    rng = np.random.default_rng(0)
    for _ in range(50):
        q, qg = rng.normal(size=4), rng.normal(size=4)
        t, tg = rng.normal(size=3), rng.normal(size=3) + 5
        assert np.allclose(speed_score(q, t, qg / np.linalg.norm(qg), tg),
                           pnp_ref.speed_score(q, t, qg / np.linalg.norm(qg), tg))


def test_speedeval_update_and_summary_format():
    ev = SpeedEval(_gt(), _StubSolver())
    ev.update({"img0.jpg": {"points": np.full((11, 2), 1.234567, np.float32), "logits": np.full((11, 12), 0.1234567)},
               "img1.jpg": {"points": np.zeros((1, 2)), "logits": np.zeros((1, 12))},
               "img2.jpg": {"points": np.zeros((2, 2)), "logits": np.zeros((2, 12))}})
    rec = ev.log["img0.jpg"]
    # float32 points round in float32 exactly as np.around does in the reference
    assert rec["points"][0] == [float(np.float32(1.23))] * 2 and rec["logits"][0][0] == 0.123457
    assert rec["score"] == 0.0
    # failures -> zero pose -> s_t = 1, s_q = pi
    for fn in ("img1.jpg", "img2.jpg"):
        assert ev.log[fn]["quat_pr"] == [0.0] * 4 and ev.log[fn]["score_tvec"] == 1.0
        assert ev.log[fn]["score_quat"] == pytest.approx(np.pi, abs=1e-7)
    s = ev.summarize()
    mean_t = np.mean([r["score_tvec"] for r in ev.log.values()])
    assert s.startswith("tvec score: {:.6f}, quat score: ".format(mean_t))
    # reference quirk: "median" of the already-averaged scalar equals the mean
    assert "median tvec: {:.6f},".format(mean_t) in s
    assert "median tvec abs:[" in s


def test_nested_tensor_contract():
    a, b = torch.ones(3, 4, 5), torch.ones(3, 6, 2)
    nt = nested_tensor_from_tensor_list([a, b])
    assert nt.tensors.shape == (2, 3, 6, 5)
    assert not nt.mask[0, :4, :5].any() and nt.mask[0, 4:, :].all() and nt.mask[1, :, 2:].all()
    x, targets = collate_fn([(a, {"f": 1}), (a, {"f": 2})])
    assert isinstance(x, NestedTensor) and not x.mask.any() and len(targets) == 2


def test_shard_covers_everything():
    for n in (1, 7, 64, 256):
        for w in (1, 2, 3, 8):
            parts = [sd.shard(n, r, w) for r in range(w)]
            assert parts[0][0] == 0 and parts[-1][1] == n
            assert all(parts[i][1] == parts[i + 1][0] for i in range(w - 1))


def _worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    r, w, _ = sd.init_distributed_mode(backend="gloo")
    B = 4
    quat = torch.full((B, 4), float(r))
    tvec = torch.full((B, 3), 10.0 * r, dtype=torch.float64)
    s_t = torch.full((B,), 0.1 * r, dtype=torch.float64)
    s_q = torch.full((B,), 0.2 * r, dtype=torch.float64)
    status = torch.full((B,), r, dtype=torch.int32)
    rec = sd.all_gather_records(sd.pack_records(quat, tvec, s_t, s_q, status))
    log = sd.all_gather_log({f"img{r}_{i}": {"score": float(r)} for i in range(2)})
    if r == 0:
        out.put((rec.numpy().tolist(), sorted(log)))
    torch.distributed.destroy_process_group()


def test_gloo_world2_record_exchange():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29500 + os.getpid() % 1000
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    rec, keys = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    rec = np.asarray(rec)
    assert rec.shape == (8, sd.RECORD_LEN)
    assert (rec[:4, 0] == 0).all() and (rec[4:, 0] == 1).all() and (rec[4:, 9] == 1).all()
    assert keys == ["img0_0", "img0_1", "img1_0", "img1_1"]


def _eval_records(n, seed=3):
    """n images' worth of device-style solver outputs (CPU tensors) + ground truth."""
    rng = np.random.default_rng(seed)
    q = rng.normal(size=(n, 4)).astype(np.float32)
    q /= np.linalg.norm(q, axis=1, keepdims=True)
    t = rng.normal(size=(n, 3)) + [0, 0, 10]
    status = rng.integers(0, 4, n).astype(np.int32)
    q[status == 1] = 0
    t[status == 1] = 0
    gt = [{"filename": f"img{i:04d}.jpg", "q_vbs2tango": (q[i] + rng.normal(0, 0.05, 4)).tolist(),
           "r_Vo2To_vbs_true": (t[i] + rng.normal(0, 0.3, 3)).tolist()} for i in range(n)]
    return {"gt": gt, "points": rng.uniform(0, 1900, (n, 11, 2)).astype(np.float32),
            "probs": rng.dirichlet(np.ones(12), (n, 11)).astype(np.float32), "quat": q, "tvec": t, "status": status,
            "sigmas": rng.uniform(0.5, 9, (n, 11, 2)).astype(np.float32),
            "mean_sigma": rng.uniform(0.5, 9, n).astype(np.float32), "reliable": rng.integers(0, 2, n).astype(bool)}


def _eval_shard(d, lo, hi):
    ev = SpeedEval(d["gt"], _StubSolver())
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a[lo:hi]))
    poses = {"quat": t(d["quat"]), "tvec": t(d["tvec"]), "status": t(d["status"])}
    ev.update_batch([g["filename"] for g in d["gt"][lo:hi]], t(d["points"]), t(d["probs"]), poses, sigmas=t(d["sigmas"]),
                    assess={"mean_sigma": t(d["mean_sigma"]), "reliable": t(d["reliable"])})
    return ev


def _eval_worker(rank, world, port, n, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    r, w, _ = sd.init_distributed_mode(backend="gloo")
    d = _eval_records(n)
    lo, hi = sd.shard(n, r, w)
    ev = _eval_shard(d, lo, hi)
    # evaluate()'s end of loop (spe/engine.py): merge every rank's log, then summarize
    ev.log = sd.all_gather_log(ev.log)
    ev.summarize()
    # the bench's per-batch record exchange (bench.py step(): pack -> all-gather)
    from spe.speed_eval import speed_score as host_score
    # (equal per-rank blocks, as the bench's fixed per-GPU batch gives)
    hi = lo + n // w
    st = torch.tensor([host_score(d["quat"][i], d["tvec"][i], d["gt"][i]["q_vbs2tango"], d["gt"][i]["r_Vo2To_vbs_true"])[0]
                       for i in range(lo, hi)], dtype=torch.float64)
    rec = sd.exchange_pose_records({"quat": torch.from_numpy(d["quat"][lo:hi]), "tvec": torch.from_numpy(d["tvec"][lo:hi]),
                                    "status": torch.from_numpy(d["status"][lo:hi])}, st, st * 2)
    out.put((r, ev.stats, json.dumps(ev.log, sort_keys=False), rec.numpy().tolist()))
    torch.distributed.destroy_process_group()


def test_gloo_world2_speedeval_equals_world1():
    """with the one log all-gather, the N-rank evaluate() summary equals the 1-rank
    summary (the reference's summarize() is rank-local, REV/engine.py:122-128), and the bench's
    record exchange returns every rank's records in rank order."""
    n = 37                                   # ragged: shards of 19 and 18 images
    d = _eval_records(n)
    one = _eval_shard(d, 0, n)
    one.summarize()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 30500 + os.getpid() % 1000
    procs = [ctx.Process(target=_eval_worker, args=(r, 2, port, n, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=180) for _ in range(2)])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r, stats, log, rec in res:
        assert stats == one.stats, r
        assert log == json.dumps(one.log, sort_keys=False)
    assert "self-assessment" in one.stats
    for _, _, _, rec in res:
        rec = np.asarray(rec)
        assert rec.shape == (2 * 18, sd.RECORD_LEN)
        idx = np.r_[0:18, 19:37]                     # rank 0's block, then rank 1's
        np.testing.assert_array_equal(rec[:, :4], d["quat"][idx].astype(np.float64))
        np.testing.assert_array_equal(rec[:, 4:7], d["tvec"][idx])
        np.testing.assert_array_equal(rec[:, 9], d["status"][idx])
        np.testing.assert_allclose(rec[:, 8], 2 * rec[:, 7])


def _bench_line(stdout):
    lines = [l for l in stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, stdout
    return json.loads(lines[0])


def test_bench_launcher_spawns_ranks():
    """`python bench.py --gpus 2` (the driver's command form, no torchrun env) starts two ranks
    through the launcher; rank 0's single line reports the whole job.  The
    SPE_BENCH_STUB worker runs the rank bookkeeping over gloo with no GPU work."""
    import subprocess
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, SPE_BENCH_STUB="1", OMP_NUM_THREADS="1")
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    lines = {}
    for n in (2, 1):
        r = subprocess.run([sys.executable, os.path.join(repo, "bench.py"), "--gpus", str(n), "--batch", "4", "--steps",
                            "3", "--warmup", "1"], env=env, capture_output=True, text=True, timeout=180)
        assert r.returncode == 0, r.stderr[-2000:]
        lines[n] = _bench_line(r.stdout)
    d = lines[2]
    assert d["n_gpus"] == 2 and d["config"]["global_batch"] == 8 and d["config"]["per_gpu_batch"] == 4
    assert d["records_gathered_per_step"] == 8
    assert d["value"] > 0 and d["steps"] == 3
    # the north-star shape: global batch 256 split 128 per rank over the fixed
    # pool, and the same weights at world 1 and world 2 (committed head fixture, no fit per run)
    ns = d["north_star"]
    assert ns["global_batch"] == 256 and ns["per_gpu_batch"] == 128 and ns["solver"] == "ransac_p3p_lm"
    assert ns["pool_images"] == list(range(256))
    assert lines[1]["north_star"]["per_gpu_batch"] == 256
    assert d["weights_sha256_16"] is not None and d["weights_sha256_16"] == lines[1]["weights_sha256_16"]


def test_bench_rejects_world_mismatch():
    """A rank whose world size differs from --gpus exits non-zero instead of reporting n_gpus 1."""
    import subprocess
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, SPE_BENCH_STUB="1", RANK="0", WORLD_SIZE="1", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1",
               MASTER_PORT=str(29400 + os.getpid() % 500))
    r = subprocess.run([sys.executable, os.path.join(repo, "bench.py"), "--gpus", "2", "--batch", "4", "--steps", "1"],
                       env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode == 2 and "world size" in r.stderr


def test_diversify_within_image_labels_ignore_the_image():
    """RT-DETR bench weights (spe.synthetic.diversify_class_head, within_image): when the image
    means dominate the query features, the head still gives each image's queries several labels
    and does not see the image-mean differences."""
    from spe.synthetic import diversify_class_head
    rng = np.random.Generator(np.random.PCG64(3))
    B, Q, d = 16, 30, 64
    means = rng.normal(0, 10.0, (B, d))
    hs = means[:, None, :] + rng.normal(0, 0.05, (B, Q, d))
    w = {"h.weight": np.zeros((12, d), np.float32), "h.bias": np.zeros(12, np.float32)}
    w = diversify_class_head(w, hs, head="h", within_image=True)
    lab = (hs @ w["h.weight"].T + w["h.bias"]).argmax(-1)
    assert min(len(set(lab[i].tolist()) - {11}) for i in range(B)) >= 4
    # the head's rows are orthogonal to the image-mean differences (to float32 storage precision)
    W = w["h.weight"].astype(np.float64)
    diff = means[3] - means[5]
    assert np.abs(W @ diff).max() <= 1e-3 * np.linalg.norm(W, axis=1).max() * np.linalg.norm(diff)


def test_fit_point_head_with_logit_offset():
    """RT-DETR's refined points are sigmoid(head(hs) + inverse_sigmoid(reference)): the fit with
    that offset reproduces its targets through the same formula."""
    from spe.synthetic import fit_point_head
    rng = np.random.Generator(np.random.PCG64(5))
    N, d = 200, 32
    hs = rng.normal(0, 1.0, (N, d)).astype(np.float32)
    tgt = rng.uniform(0.1, 0.9, (N, 2)).astype(np.float32)
    off = rng.normal(0, 1.0, (N, 2)).astype(np.float32)
    mask = np.ones(N, bool)
    w, err = fit_point_head({}, hs, tgt, mask, steps=1500, lr=3e-3, prefix="p", noise_rel=0.0, offset=off)
    z = np.maximum(hs @ w["p.layers.0.weight"].T + w["p.layers.0.bias"], 0)
    z = np.maximum(z @ w["p.layers.1.weight"].T + w["p.layers.1.bias"], 0)
    pts = 1 / (1 + np.exp(-(z @ w["p.layers.2.weight"].T + w["p.layers.2.bias"] + off)))
    assert np.abs(pts - tgt).max() < 0.05 and err.max() < 0.05, (np.abs(pts - tgt).max(), err.max())


@pytest.mark.parametrize("decode,backbone", [(False, False), (True, False), (True, True)])
def test_pipeline_staged_state_without_gpu(monkeypatch, decode, backbone):
    """PosePipeline's constructor on the CPU (HIP streams stubbed): the staged forms own their
    slot workspaces, snapshots and counters (a regression once left them under an unrelated
    branch, and only the GPU pipeline tests noticed)."""
    from types import SimpleNamespace
    import spe.pipeline as pp

    class _Stream:
        def __init__(self, device=None):
            self.device = device
    monkeypatch.setattr(pp.torch.cuda, "Stream", _Stream)

    class _Model:
        cfg = SimpleNamespace(input_size=32, num_queries=11)

        def workspace(self, B, dev):
            pass

        def new_workspace(self, B, dev):
            return torch.zeros(1)
    p = pp.PosePipeline(_Model(), None, 2, device="cpu", overlap_decode=decode, overlap_backbone=backbone)
    assert not p.per_image_th and p.repro.shape == (2,)
    if decode:
        n = 3 if backbone else 2
        assert p.nslot == n and p.calls == 0 and len(p.ws2) == n and len(p.slot_clip) == n
        assert (p.enc_stream is not None) == backbone and p.dec_stream is not None
    else:
        assert not hasattr(p, "ws2")


def test_epnp_ceres_batch_needs_areas_and_keeps_state():
    """EPnPCeresSolver.solve_batch derives every image's threshold from its own box area
    (UNC/utils/speed_eval_ceres.py:53-58,90); a batch without areas is refused instead of running
    at the constructor's 20 px, and batch thresholds leave reprojectionError (the reference's
    per-image __call__ state) untouched."""
    import torch
    from spe.solver import EPnPCeresSolver
    s = EPnPCeresSolver(input_size=256)
    s.get_repro_th(100.0)                       # the per-image path: int(100/256*10) = 3
    assert s.reprojectionError == 3.0
    assert [s.repro_th(a) for a in (10.0, 100.0, 1e5)] == [1.5, 3.0, 20.0]
    assert s.reprojectionError == 3.0
    pts, probs = torch.zeros(2, 11, 2), torch.zeros(2, 11, 12)
    with pytest.raises(ValueError, match="area"):
        s.solve_batch(pts, probs)


def test_ground_truth_area_keeps_reference_precedence():
    """UNC SpeedEval's area = sqrt((x2 - x1) * y2 - y1) (src/data/speed/speed_dataset.py:370-373)."""
    from spe.speed_eval import load_ground_truth
    g = load_ground_truth([{"filename": "a.jpg", "q_vbs2tango": [1, 0, 0, 0], "r_Vo2To_vbs_true": [0, 0, 10],
                            "bbox_xxyy": [100.0, 200.0, 300.0, 400.0]}])
    assert g["a.jpg"]["area"] == pytest.approx(np.sqrt(200.0 * 400.0 - 200.0))


def test_bench_score_contract_against_fp32_spread():
    """bench.accuracy_summary's score half of the contract: measured against the
    committed spread of two fp32 implementations (profiles/r5b_precision_score.json) -- met by deltas
    inside that spread, not met by a wider fraction of misses or a larger worst case."""
    import importlib.util
    import numpy as np
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(repo, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    sp = bench.score_spread("epnp")
    assert sp is not None and 0.5 < sp["frac"] < 1.0 and sp["max"] > 0.0
    n = 64
    rng = np.random.default_rng(3)
    ref = rng.uniform(0.1, 2.0, n)

    def raw(delta):
        return {"score_ref": ref, "score": ref + delta, "cond": np.full(n, 1e-6), "d_norm": np.full(10, 3e-5),
                "d_px": np.full(10, 0.02), "d_per_crop": np.full(10, 3e-5), "hs_rel": np.full(4, 1e-6),
                "label_agree": np.ones(4), "status_agree": np.ones(n)}
    good = np.full(n, 1e-5)
    good[:4] = 2e-3                                    # 94 % within 1e-4, small worst case
    a = bench.accuracy_summary(raw(good), "epnp")
    assert a["meets_1e-4_kpt"] and not a["meets_1e-4_score"]
    assert a["score_within_fp32_spread"] and a["meets_1e-4_within_fp32_spread"]
    bad = np.full(n, 1e-5)
    bad[: n // 2] = 1e-3                               # half the images outside 1e-4
    assert not bench.accuracy_summary(raw(bad), "epnp")["score_within_fp32_spread"]
    worst = good.copy()
    worst[0] = 10.0 * sp["max"]
    assert not bench.accuracy_summary(raw(worst), "epnp")["score_within_fp32_spread"]
    assert "score_within_fp32_spread" not in bench.accuracy_summary(raw(good), None)


def test_evaluate_ceres_refuses_ground_truth_without_areas():
    """evaluate() with the EPnPCeresSolver checks up front that every ground-truth entry
    carries the box area its per-image threshold comes from, instead of a KeyError mid-evaluation."""
    from spe.engine import evaluate
    from spe.solver import EPnPCeresSolver
    gt = [{"filename": "img000001.jpg", "q_vbs2tango": [1, 0, 0, 0], "r_Vo2To_vbs_true": [0, 0, 10]},
          {"filename": "img000002.jpg", "q_vbs2tango": [1, 0, 0, 0], "r_Vo2To_vbs_true": [0, 0, 9],
           "bbox_xxyy": [10, 20, 110, 140]}]
    with pytest.raises(ValueError, match="box areas"):
        evaluate(None, None, None, [], gt, EPnPCeresSolver(input_size=256), "cpu")
