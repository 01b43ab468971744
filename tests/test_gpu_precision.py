"""GPU: the accuracy contract on the bench's own weights (BASELINE north_star "keypoint L2 and SPEED
pose-score within 1e-4 of reference").

The bench's pose-consistent weights (spe.synthetic.fixed_bench_weights: label-diverse random init
with a 64x-sharpened decoder cross-attention and a point head fitted to the decoder outputs of the
256-image bench pool) amplify perturbations of the decoder output hs ~20x into the keypoints.  This
test measures, on the config-2 timed batch (pool images 0..63), how far apart INDEPENDENT fp32
implementations of the same model land -- at the keypoints and at the SPEED score, both solvers:

  * ours-fp32     the exact-f32 parity mode (this repo; <= 1e-4 of the reference on its goldens)
  * torch-gpu     the oracle's torch restatement (oracle/model_ref.py, pinned to the reference at
                  <= 2e-7 on the goldens) in fp32 on the GPU (hipBLASLt / MIOpen, TF32 off)
  * torch-cpu     the same restatement on the CPU, all 64 images (the reference's own execution
                  model: REV main.py --eval on CPU, BASELINE config 1)

and where the fast modes land against them (fp32x6 / fp32h3 = the accuracy-contract candidates, fp32x3,
bf16).
Every implementation's keypoints go through the SAME HIP solver (EPnP = config 2, P3P-RANSAC + LM
= configs 3 / north star), so the score deltas isolate the keypoints.  Per image the test also
records the score's float32 conditioning (the largest score change when the ours-fp32 keypoints
move by one float32 ulp per coordinate, 16 random directions; bench.Fp32Reference.cond) and, for
every image where fp32x6 and ours-fp32 differ by more than 1e-4, the solver decision behind it
(oracle/pnp_ref.c trace: EPnP beta-candidate errors / pick, RANSAC best iteration / inlier mask /
the point nearest the threshold).

Gates (written here):
  keypoints  fp32x6 within 2x the ours-fp32 / torch-gpu spread + 1e-5 of ours-fp32, and <= 1e-4
             normalised of torch-cpu on all 64 images;
  score      per solver, fp32x6's per-image score deltas against ours-fp32 lie inside the fp32
             implementation spread (torch-cpu's deltas against ours-fp32): its fraction of images
             within 1e-4 is at least torch-cpu's minus 0.05 (64-image sampling slack), its median
             delta at most 2x torch-cpu's, and its largest delta no larger than the largest of the
             two torch implementations'.  The images fp32x6 misses are listed with their
             conditioning and the solver decision behind them (informational).

Measured (profiles/r5_precision_score.json, config-2 batch): EPnP -- fp32x6 84 % within 1e-4 of
ours-fp32, torch-cpu 80 %, torch-gpu 81 %, torch-cpu vs torch-gpu 88 %; P3P-RANSAC + LM -- fp32x6
98 % (max 1.09e-4), torch-cpu 92 %, torch-gpu 97 %.  Every fp32x6 miss is a continuous move of an
EPnP pose fitted through an outlier (mean reprojection errors of 20-176 px), no beta-candidate or
RANSAC flip.
"""
import argparse
import json
import os
import sys

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# pool images 0..B-1: 64 = the config-2 batch (the suite's case); SPE_PRECISION_IMAGES=256 repeats the
# study on the north star's global batch (the whole pool; gpurun_out/precision_score_256.json)
B = int(os.environ.get("SPE_PRECISION_IMAGES", "64"))


def _progress(msg):
    """A progress line on stdout and, when a gpurun_out/ scratch directory exists, appended to a file
    there: the CPU restatement passes run for minutes with pytest capturing stdout."""
    print(msg, flush=True)
    out = os.path.join(REPO, "gpurun_out")
    if os.path.isdir(out):
        with open(os.path.join(out, "precision_progress.log"), "a") as f:
            f.write(msg + "\n")


def _kpt(a, b, fg):
    return float((a - b).abs().amax(-1)[fg].max())


def _decision(tr_a, tr_b, mode):
    """Name the discrete solver choice that differs between two traces (or 'continuous')."""
    if mode == 0:
        if tr_a["epnp_pick"] != tr_b["epnp_pick"]:
            return f"epnp_beta_pick {tr_a['epnp_pick']}->{tr_b['epnp_pick']}"
        return "continuous"
    for k in ("ransac_mask", "ransac_best_iter", "ransac_iters", "epnp_pick"):
        if tr_a[k] != tr_b[k]:
            return f"{k} {tr_a[k]}->{tr_b[k]}"
    return "continuous"


@pytest.mark.timeout(900)
def test_fp32x6_within_fp32_implementation_spread(gpu_device):
    sys.path.insert(0, REPO)
    import model_ref
    import pnp_ref
    from spe.config import Camera, SpeConfig, world_points
    from spe.models import DETR
    from spe.solver import build_solver
    from spe.speed_eval import device_speed_score
    from spe.synthetic import bench_images, fixed_bench_weights

    dev = gpu_device
    cfg = SpeConfig(input_size=416, num_queries=11, enc_layers=6, dec_layers=6)
    w, meta = fixed_bench_weights(cfg, 0)
    assert w is not None, "committed head fixture missing (oracle/gen_bench_heads.py)"
    data = bench_images(cfg, 0, B)
    x = torch.from_numpy(data["images"]).to(dev)
    clip = torch.from_numpy(data["clip_bbox"]).float().to(dev)
    q_gt = torch.from_numpy(data["quat"]).to(dev)
    t_gt = torch.from_numpy(data["tvec"]).to(dev)

    impl = {}                                      # name -> (pred_points, points_px, probs)

    def ours(dtype):
        m = DETR(cfg, dtype=dtype, attn_dtype=dtype)
        m.load_state_dict(w)
        o = m(x, clip_bbox=clip)
        torch.cuda.synchronize()
        impl[dtype] = (o["pred_points"].clone(), o["points_px"].clone(), o["probs"].clone())
        del m

    for dt in ("fp32", "fp32x6", "fp32h3", "fp32x3", "bf16"):
        ours(dt)

    def torch_impl(images, device):
        mm, cv = torch.backends.cuda.matmul.allow_tf32, torch.backends.cudnn.allow_tf32
        torch.backends.cuda.matmul.allow_tf32 = torch.backends.cudnn.allow_tf32 = False
        try:
            with torch.no_grad():
                outs = []
                for i in range(0, len(images), 16):       # (progress lines: a long CPU pass stays visible)
                    outs.append(model_ref.forward(images[i:i + 16], w, cfg))
                    _progress(f"torch {device}: {i + 16}/{len(images)} images")
        finally:
            torch.backends.cuda.matmul.allow_tf32, torch.backends.cudnn.allow_tf32 = mm, cv
        lg = torch.cat([o["pred_logits"] for o in outs]).float().cpu()
        pn = torch.cat([o["pred_points"] for o in outs]).float().cpu()
        pp = model_ref.postprocess(lg, pn, data["clip_bbox"])
        px = torch.from_numpy(np.stack([r["points"] for r in pp])).to(dev)
        pr = torch.from_numpy(np.stack([r["logits"] for r in pp])).to(dev)
        return pn.to(dev), px, pr

    impl["torch_gpu"] = torch_impl(x, dev)
    torch.set_num_threads(max(1, min(16, os.cpu_count() or 1)))
    impl["torch_cpu"] = torch_impl(data["images"], "cpu")

    lab = {k: v[2].argmax(-1) for k, v in impl.items()}
    fg = (lab["fp32"] < 11)
    for k in ("fp32x6", "fp32h3", "fp32x3", "torch_gpu", "torch_cpu"):
        fg &= lab[k] == lab["fp32"]
    kp = {k: v[0] for k, v in impl.items()}
    r = {"config": "config 2 shape, pool images 0..63, bench fixture weights " + meta["generator"],
         "fg_queries": int(fg.sum()),
         "kpt": {"ours_fp32_vs_torch_gpu": _kpt(kp["fp32"], kp["torch_gpu"], fg),
                 "ours_fp32_vs_torch_cpu": _kpt(kp["fp32"], kp["torch_cpu"], fg),
                 "torch_cpu_vs_torch_gpu": _kpt(kp["torch_cpu"], kp["torch_gpu"], fg),
                 "fp32x6_vs_ours_fp32": _kpt(kp["fp32x6"], kp["fp32"], fg),
                 "fp32x6_vs_torch_gpu": _kpt(kp["fp32x6"], kp["torch_gpu"], fg),
                 "fp32x6_vs_torch_cpu": _kpt(kp["fp32x6"], kp["torch_cpu"], fg),
                 "fp32h3_vs_ours_fp32": _kpt(kp["fp32h3"], kp["fp32"], fg),
                 "fp32h3_vs_torch_gpu": _kpt(kp["fp32h3"], kp["torch_gpu"], fg),
                 "fp32h3_vs_torch_cpu": _kpt(kp["fp32h3"], kp["torch_cpu"], fg),
                 "fp32x3_vs_ours_fp32": _kpt(kp["fp32x3"], kp["fp32"], fg),
                 "label_agreement_bf16": float((lab["bf16"] == lab["fp32"]).float().mean())}}

    # ---- the same HIP solver on every implementation's keypoints
    K, Wd = Camera.K, world_points()
    trace_pairs = {}
    r["score"] = {}
    for name, mode in (("epnp", 0), ("ransac_p3p_lm", 1)):
        solver = build_solver(argparse.Namespace(solver=name, repro=20))
        sc = {}
        for k, (_, px, pr) in impl.items():
            po = solver.solve_batch(px, pr)
            st, sq = device_speed_score(po["quat"], po["tvec"], q_gt, t_gt)
            sc[k] = (st + sq).cpu().numpy()
        # float32 conditioning of the ours-fp32 scores (bench.Fp32Reference's rule)
        cond = _ulp_conditioning(solver, impl["fp32"][1], impl["fp32"][2], q_gt, t_gt, sc["fp32"], dev)
        pairs = [("fp32x6", "fp32"), ("fp32h3", "fp32"), ("torch_cpu", "fp32"), ("torch_gpu", "fp32"),
                 ("torch_cpu", "torch_gpu"), ("fp32x6", "torch_cpu"), ("fp32h3", "torch_cpu"), ("fp32x3", "fp32"),
                 ("bf16", "fp32")]
        tab = {}
        for a, b in pairs:
            d = np.abs(sc[a] - sc[b])
            ok = np.isfinite(d)
            tab[f"{a}_vs_{b}"] = {"frac_le_1e-4": float((d[ok] <= 1e-4).mean()), "max": float(d[ok].max()),
                                  "median": float(np.median(d[ok]))}
        dc = np.abs(sc["torch_cpu"] - sc["fp32"])
        dg = np.abs(sc["torch_gpu"] - sc["fp32"])
        wc = cond <= 1e-4
        r["score"][name] = {"pairs": tab, "images_ill_conditioned_at_f32_ulp": int((~wc).sum()),
                            "cond_median": float(np.median(cond)),
                            "frac_torch_cpu_le_1e-4_well_conditioned": float((dc[wc] <= 1e-4).mean()) if wc.any() else None,
                            "decisions": {}}
        for cand in ("fp32x6", "fp32h3"):
            d6 = np.abs(sc[cand] - sc["fp32"])
            miss = np.where(d6 > 1e-4)[0]
            # the decision behind every miss: oracle traces of the two keypoint sets
            _, tr32 = pnp_ref.pnp_trace(impl["fp32"][1][miss].cpu().numpy(), impl["fp32"][2][miss].cpu().numpy(), K,
                                        Wd, mode=mode, repro=20.0)
            _, tr6 = pnp_ref.pnp_trace(impl[cand][1][miss].cpu().numpy(), impl[cand][2][miss].cpu().numpy(), K,
                                       Wd, mode=mode, repro=20.0)
            per = []
            for j, i in enumerate(miss):
                per.append({"image": int(i), "score_fp32": float(sc["fp32"][i]), f"delta_{cand}": float(d6[i]),
                            "delta_torch_cpu": float(dc[i]), "delta_torch_gpu": float(dg[i]),
                            "cond_f32_ulp": float(cond[i]), "decision": _decision(tr32[j], tr6[j], mode),
                            "epnp_err_fp32": [round(tr32[j][f"epnp_err{c}"], 6) for c in (1, 2, 3)],
                            f"epnp_err_{cand}": [round(tr6[j][f"epnp_err{c}"], 6) for c in (1, 2, 3)],
                            "epnp_pick": [tr32[j]["epnp_pick"], tr6[j]["epnp_pick"]],
                            **({"ransac_inliers": [tr32[j]["ransac_inliers"], tr6[j]["ransac_inliers"]],
                                "ransac_margin_px": round(tr32[j]["ransac_margin_px"], 4)} if mode == 1 else {})})
            r["score"][name][f"frac_{cand}_le_1e-4_well_conditioned"] = \
                float((d6[wc] <= 1e-4).mean()) if wc.any() else None
            r["score"][name][f"{cand}_misses"] = per
            r["score"][name]["decisions"][cand] = {k: sum(1 for p in per if p["decision"].split(" ")[0] == k)
                                                   for k in sorted({p["decision"].split(" ")[0] for p in per})}
        trace_pairs[name] = cond

    out = os.path.join(REPO, "gpurun_out")
    if os.path.isdir(out):
        sfx = "" if B == 64 else f"_{B}"
        with open(os.path.join(out, f"precision_score{sfx}.json"), "w") as f:
            json.dump(r, f, indent=1)
        np.savez(os.path.join(out, f"precision_keypoints{sfx}.npz"),
                 **{f"{k}_{j}": v[j].cpu().numpy() for k, v in impl.items() for j in range(3)})
    print(json.dumps({k: v for k, v in r.items() if k != "score"}))
    for name, s in r["score"].items():
        print(name, json.dumps(s["pairs"]), s["decisions"])

    # ---- gates
    k = r["kpt"]
    assert fg.sum() > 300
    assert k["ours_fp32_vs_torch_gpu"] <= 1e-3
    for mode in ("fp32x6", "fp32h3"):                   # both accuracy-contract candidates
        assert k[f"{mode}_vs_ours_fp32"] <= 2 * k["ours_fp32_vs_torch_gpu"] + 1e-5, (mode, k)
        assert k[f"{mode}_vs_torch_cpu"] <= 1e-4, (mode, k)
        for name in trace_pairs:
            tab = r["score"][name]["pairs"]
            x6, cpu, gpu = tab[f"{mode}_vs_fp32"], tab["torch_cpu_vs_fp32"], tab["torch_gpu_vs_fp32"]
            cg = tab["torch_cpu_vs_torch_gpu"]
            assert x6["frac_le_1e-4"] >= cpu["frac_le_1e-4"] - 0.05, (mode, name, tab)
            assert x6["median"] <= 2 * cpu["median"], (mode, name, tab)
            # the worst image: within the largest disagreement of two fp32 implementations (the maxima
            # are single ill-conditioned images, so every fp32 pair counts)
            assert x6["max"] <= max(cpu["max"], gpu["max"], cg["max"]), (mode, name, tab)


def _ulp_conditioning(solver, px, probs, q_gt, t_gt, score, dev, draws=16):
    """Per image: the largest SPEED-score change over `draws` re-solves of the keypoints each moved
    by one float32 ulp per coordinate in a random direction (bench.Fp32Reference.cond)."""
    from spe.speed_eval import device_speed_score
    p = px.cpu().numpy().astype(np.float32)
    n = p.shape[0]
    rng = np.random.Generator(np.random.PCG64(11))
    sgn = rng.choice(np.array([-np.inf, np.inf], np.float32), size=(draws,) + p.shape)
    pp = np.nextafter(np.broadcast_to(p, (draws,) + p.shape), sgn).astype(np.float32).reshape((draws * n,) + p.shape[1:])
    po = solver.solve_batch(torch.from_numpy(pp).to(dev), probs.repeat(draws, 1, 1))
    st, sq = device_speed_score(po["quat"], po["tvec"], q_gt.repeat(draws, 1), t_gt.repeat(draws, 1))
    sc = (st + sq).cpu().numpy().reshape(draws, n)
    diff = np.abs(sc - score[None])
    diff = np.where(np.isnan(sc) != np.isnan(score[None]), np.inf, diff)
    return np.nan_to_num(diff, nan=0.0).max(0)


# BASELINE configs 4 and 5 (the contract mode on their shapes): the model, solver and weights the
# bench's --config 4 / 5 lines time (bench.PRESETS, bench.bench_weights_for)
CONFIG_CASES = {
    4: dict(size=416, queries=11, layers=6, sigma_head=True, solver="epnp_ransac_sigma"),
    5: dict(size=640, queries=40, layers=6, sigma_head=False, solver="ransac_p3p_lm"),
}


@pytest.mark.timeout(1200)
@pytest.mark.parametrize("config", [4, 5])
def test_fp32h3_within_fp32_spread_config(gpu_device, config):
    """The accuracy contract on BASELINE configs 4 (sigma head, sigma-weighted EPnP-RANSAC,
    self-assessment filter; UNC/utils/speed_eval.py:322-420) and 5 (640x640, 40 queries;
    REV/train_resnet50s8_query40.sh:24-43): fp32h3 against the exact-f32 mode, inside the spread of
    two fp32 implementations of the reference (torch-CPU / torch-GPU restatements) on the same batch,
    with the same gates as config 2 -- keypoints within 2x the ours-fp32 / torch-GPU spread + 1e-5 and
    <= 1e-4 of torch-CPU (or within the largest fp32-pair disagreement where that is larger); per-image score fraction within 1e-4 >= torch-CPU's - 0.05, median <= 2x,
    max <= the largest fp32-pair disagreement.  Config 4 also compares the self-assessment `reliable`
    flag: fp32h3's agreement with exact f32 at least torch-CPU's - 0.05.  Writes
    gpurun_out/precision_score_c<config>.json (the spread the bench lines are held to)."""
    sys.path.insert(0, REPO)
    import bench
    import model_ref
    from spe.config import SpeConfig
    from spe.models import DETR
    from spe.solver import build_solver
    from spe.speed_eval import device_speed_score
    from spe.synthetic import bench_images

    dev = gpu_device
    cc = CONFIG_CASES[config]
    cfg = SpeConfig(input_size=cc["size"], num_queries=cc["queries"], enc_layers=cc["layers"],
                    dec_layers=cc["layers"], sigma_head=cc["sigma_head"])
    args = argparse.Namespace(weights="pose-consistent")
    _progress(f"config {config}: bench weights")
    w, _, wsource = bench.bench_weights_for(args, cfg, None, 0, 1, dev)
    _progress(f"config {config}: weights ready ({wsource})")
    # (config 5: the 32 images of its bench line -- the 640 x 640 CPU restatement is the long pole)
    nb = int(os.environ.get("SPE_PRECISION_IMAGES_CFG", "64" if config == 4 else "32"))
    data = bench_images(cfg, 0, nb)
    x = torch.from_numpy(data["images"]).to(dev)
    clip = torch.from_numpy(data["clip_bbox"]).float().to(dev)
    q_gt = torch.from_numpy(data["quat"]).to(dev)
    t_gt = torch.from_numpy(data["tvec"]).to(dev)
    impl = {}                                      # name -> (pred_points, points_px, probs, sigmas)
    for dt in ("fp32", "fp32h3", "bf16"):
        _progress(f"config {config}: {dt} forward")
        m = DETR(cfg, dtype=dt, attn_dtype="fp16" if (dt == "bf16" and config == 5) else dt)
        m.load_state_dict(w)
        outs = [m(x[i:i + 16], clip_bbox=clip[i:i + 16]) for i in range(0, nb, 16)]
        torch.cuda.synchronize()
        impl[dt] = tuple(torch.cat([o[k] for o in outs]).clone() if k in outs[0] else None
                         for k in ("pred_points", "points_px", "probs", "sigmas"))
        del m, outs

    def torch_impl(images, device):
        mm, cv = torch.backends.cuda.matmul.allow_tf32, torch.backends.cudnn.allow_tf32
        torch.backends.cuda.matmul.allow_tf32 = torch.backends.cudnn.allow_tf32 = False
        try:
            with torch.no_grad():
                outs = []
                for i in range(0, len(images), 8):
                    outs.append(model_ref.forward(images[i:i + 8], w, cfg))
                    _progress(f"config {config} torch {device}: {i + 8}/{len(images)} images")
        finally:
            torch.backends.cuda.matmul.allow_tf32, torch.backends.cudnn.allow_tf32 = mm, cv
        lg = torch.cat([o["pred_logits"] for o in outs]).float().cpu()
        pn = torch.cat([o["pred_points"] for o in outs]).float().cpu()
        ls = torch.cat([o["pred_sigmas"] for o in outs]).float().cpu() if cfg.sigma_head else None
        pp = model_ref.postprocess(lg, pn, data["clip_bbox"], ls)
        px = torch.from_numpy(np.stack([r["points"] for r in pp])).to(dev)
        pr = torch.from_numpy(np.stack([r["logits"] for r in pp])).to(dev)
        sg = torch.from_numpy(np.stack([r["sigmas"] for r in pp])).to(dev) if cfg.sigma_head else None
        return pn.to(dev), px, pr, sg

    impl["torch_gpu"] = torch_impl(x, dev)
    torch.set_num_threads(max(1, min(16, os.cpu_count() or 1)))
    impl["torch_cpu"] = torch_impl(data["images"], "cpu")

    lab = {k: v[2].argmax(-1) for k, v in impl.items()}
    fg = lab["fp32"] < 11
    for k in ("fp32h3", "torch_gpu", "torch_cpu"):
        fg &= lab[k] == lab["fp32"]
    kp = {k: v[0] for k, v in impl.items()}
    r = {"config": f"BASELINE config {config} shape, pool images 0..{nb - 1}, bench weights ({wsource})",
         "fg_queries": int(fg.sum()),
         "kpt": {"ours_fp32_vs_torch_gpu": _kpt(kp["fp32"], kp["torch_gpu"], fg),
                 "ours_fp32_vs_torch_cpu": _kpt(kp["fp32"], kp["torch_cpu"], fg),
                 "torch_cpu_vs_torch_gpu": _kpt(kp["torch_cpu"], kp["torch_gpu"], fg),
                 "fp32h3_vs_ours_fp32": _kpt(kp["fp32h3"], kp["fp32"], fg),
                 "fp32h3_vs_torch_gpu": _kpt(kp["fp32h3"], kp["torch_gpu"], fg),
                 "fp32h3_vs_torch_cpu": _kpt(kp["fp32h3"], kp["torch_cpu"], fg),
                 "label_agreement_bf16": float((lab["bf16"] == lab["fp32"]).float().mean()),
                 "label_agreement_fp32h3": float((lab["fp32h3"] == lab["fp32"]).float().mean())}}
    solver = build_solver(argparse.Namespace(solver=cc["solver"], repro=20))
    sc, rel = {}, {}
    for k, (_, px, pr, sg) in impl.items():
        po = solver.solve_batch(px, pr, sg)
        st, sq = device_speed_score(po["quat"], po["tvec"], q_gt, t_gt)
        sc[k] = (st + sq).cpu().numpy()
        if sg is not None:
            rel[k] = solver.self_assess(pr, sg, po)["reliable"].cpu().numpy().astype(bool)
    tab = {}
    for a, b in (("fp32h3", "fp32"), ("torch_cpu", "fp32"), ("torch_gpu", "fp32"), ("torch_cpu", "torch_gpu"),
                 ("fp32h3", "torch_cpu"), ("bf16", "fp32")):
        d = np.abs(sc[a] - sc[b])
        ok = np.isfinite(d)
        tab[f"{a}_vs_{b}"] = {"frac_le_1e-4": float((d[ok] <= 1e-4).mean()), "max": float(d[ok].max()),
                              "median": float(np.median(d[ok]))}
    # per-image deltas of the fp32 pairs (pool image order): a bench line over the first n images
    # is held to the spread on exactly those images (bench.score_spread)
    per = {f"{a}_vs_{b}": [float(v) for v in np.abs(sc[a] - sc[b])]
           for a, b in (("torch_cpu", "fp32"), ("torch_gpu", "fp32"), ("torch_cpu", "torch_gpu"))}
    # (fp32h3's own per-image deltas, for the record; bench.score_spread reads the fp32 pairs only)
    r["fp32h3_per_image"] = {f"fp32h3_vs_{b}": [float(v) for v in np.abs(sc["fp32h3"] - sc[b])]
                             for b in ("fp32", "torch_cpu", "torch_gpu")}
    r["score"] = {cc["solver"]: {"pairs": tab, "per_image": per}}
    if rel:
        r["reliable"] = {f"{a}_vs_fp32": float((rel[a] == rel["fp32"]).mean()) for a in rel if a != "fp32"}
        r["reliable"]["fp32_reliable_images"] = int(rel["fp32"].sum())
        r["reliable"]["per_image_torch_cpu_vs_fp32"] = [bool(v) for v in rel["torch_cpu"] == rel["fp32"]]
    out = os.path.join(REPO, "gpurun_out")
    if os.path.isdir(out):
        with open(os.path.join(out, f"precision_score_c{config}.json"), "w") as f:
            json.dump(r, f, indent=1)
    print(json.dumps(r))

    k = r["kpt"]
    assert fg.sum() > 50
    assert k["fp32h3_vs_ours_fp32"] <= 2 * k["ours_fp32_vs_torch_gpu"] + 1e-5, k
    # 1e-4 of torch-CPU, or -- where two fp32 implementations already disagree by more (config 5's
    # 640 / Q40 shape: ours-fp32 vs torch-CPU 1.4e-4, profiles/r6_precision_score_c5.json) -- within
    # their largest disagreement
    spread = max(k["ours_fp32_vs_torch_cpu"], k["ours_fp32_vs_torch_gpu"], k["torch_cpu_vs_torch_gpu"])
    assert k["fp32h3_vs_torch_cpu"] <= max(1e-4, spread), k
    h3, cpu, gpu, cg = (tab["fp32h3_vs_fp32"], tab["torch_cpu_vs_fp32"], tab["torch_gpu_vs_fp32"],
                        tab["torch_cpu_vs_torch_gpu"])
    assert h3["frac_le_1e-4"] >= cpu["frac_le_1e-4"] - 0.05, tab
    assert h3["median"] <= 2 * max(cpu["median"], 1e-7), tab
    assert h3["max"] <= max(cpu["max"], gpu["max"], cg["max"]), tab
    if rel:
        assert r["reliable"]["fp32h3_vs_fp32"] >= r["reliable"]["torch_cpu_vs_fp32"] - 0.05, r["reliable"]
