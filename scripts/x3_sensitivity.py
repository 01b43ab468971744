"""Per-stage precision study of the fp32x3 parity mode.

Builds the bench's pose-consistent weights (bench.py, config 2, B = 64), runs the exact-f32 model
as the reference, then the fp32x3 model with chosen launch kinds forced to the exact-f32 kernels
(SPE_X3_EXACT, read at model creation) and reports the keypoint / hs deviation of each variant:

  * "only G split": every stage exact except group G (the error G contributes alone)
  * "G exact":      every stage split except group G

    python scripts/x3_sensitivity.py [--out gpurun_out/x3_sensitivity.json]
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "satellite-pose-estimation_amd"))

GROUPS = {
    "backbone": "conv.,gemm.input_proj",
    "enc_proj": "gemm.enc.qk,gemm.enc.v,gemm.enc.o",
    "enc_attn": "attn.enc",
    "enc_ffn": "gemm.enc.ffn",
    "dec_cross": "gemm.cross_kv,attn.dec_cross",
    "dec_rest": "gemm.dec,attn.dec_self",
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=os.path.join(REPO, "gpurun_out", "x3_sensitivity.json"))
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--variants", default="all")
    a = ap.parse_args()
    import numpy as np
    import torch
    import bench
    from spe.config import SpeConfig
    from spe.models import DETR
    from spe.synthetic import bench_weights

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    B = a.batch
    cfg = SpeConfig(input_size=416, num_queries=11, enc_layers=6, dec_layers=6)
    # weights built exactly as the default (bf16) bench line builds them
    args = argparse.Namespace(dtype="bf16", attn_dtype="bf16")

    def hs_fn(w, images):
        m = DETR(cfg, dtype="bf16")
        m.load_state_dict(w)
        n = len(images)
        x = torch.from_numpy(np.concatenate([images] * ((B + n - 1) // n))[:B]).to(dev)
        return m(x, return_hs=True)["hs"].cpu().numpy()[:n]

    t0 = time.time()
    w = bench_weights(cfg, 0, hs_fn)
    w, fit = bench.pose_consistent_weights(w, cfg, args, B, 0, 1, dev)
    data = bench.bench_data(cfg, B, 0)
    x = torch.from_numpy(data["images"]).to(dev)
    clip = torch.from_numpy(data["clip_bbox"]).float().to(dev)
    print(f"weights ready in {time.time() - t0:.1f}s fit={fit}", flush=True)

    def run(dtype, exact=None):
        if not exact:
            os.environ.pop("SPE_X3_EXACT", None)
        else:
            os.environ["SPE_X3_EXACT"] = exact
        m = DETR(cfg, dtype=dtype)
        m.load_state_dict(w)
        o = m(x, clip_bbox=clip, return_hs=True)
        torch.cuda.synchronize()
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ev0.record()
        for _ in range(3):
            m(x, clip_bbox=clip, return_hs=True)
        ev1.record()
        torch.cuda.synchronize()
        o = {k: v for k, v in o.items() if torch.is_tensor(v)}
        o["ms"] = ev0.elapsed_time(ev1) / 3
        del m
        return o

    ref = run("fp32")
    print(f"fp32 forward {ref['ms']:.2f} ms", flush=True)
    lab_r = ref["probs"].argmax(-1)

    def cmp(o):
        lab = o["probs"].argmax(-1)
        fg = (lab_r < 11) & (lab == lab_r)
        dn = (o["pred_points"] - ref["pred_points"]).abs().amax(-1)[fg]
        hs = ((o["hs"] - ref["hs"]).norm(dim=-1) / ref["hs"].norm(dim=-1)).flatten()
        dl = (o["pred_logits"] - ref["pred_logits"]).abs().max().item()
        return {"kpt_norm_max": float(dn.max()), "kpt_norm_mean": float(dn.mean()),
                "kpt_norm_p99": float(torch.quantile(dn, 0.99)),
                "frac_kpt_le_1e-4": float((dn <= 1e-4).float().mean()),
                "hs_rel_max": float(hs.max()), "hs_rel_mean": float(hs.mean()), "logit_abs_max": dl,
                "label_agreement": float((lab == lab_r).float().mean()), "ms": o["ms"]}

    allk = ",".join(GROUPS.values())
    variants = [("x3 (all split)", None), ("all exact", allk)]
    for g in GROUPS:
        variants.append((f"only {g} split", ",".join(v for k, v in GROUPS.items() if k != g)))
    for g, v in GROUPS.items():
        variants.append((f"{g} exact", v))
    if a.variants != "all":
        keep = a.variants.split(";")
        variants = [(n, e) for n, e in variants if n in keep]
    res = {"config": "config 2, B=%d, bench pose-consistent weights" % B, "fp32_ms": ref["ms"], "fit": fit, "rows": []}
    if a.variants == "all" or "fp32x6" in a.variants.split(";"):
        variants.insert(0, ("fp32x6", "__x6__"))
    if a.variants == "x6":            # the fp32x6 mode with one group at a time on the exact-f32 kernels
        variants = [("fp32x6", "__x6__")] + [(f"x6, {g} exact", "__x6__" + v) for g, v in GROUPS.items()]
    for name, exact in variants:
        if exact is not None and exact.startswith("__x6__"):
            r = cmp(run("fp32x6", exact[6:] or None))
        else:
            r = cmp(run("fp32x3", exact))
        r["variant"], r["exact_kinds"] = name, exact
        res["rows"].append(r)
        print(json.dumps(r), flush=True)
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    with open(a.out, "w") as f:
        json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
