"""Per-class roofline summary of one profiled bench step (bench.py --launch-table FILE):
for every launch class, the algorithmic flops and bytes, the HIP-event time, achieved TFLOP/s
and HBM GB/s, and the fraction of the binding gfx950 peak (MI355X_MICROARCH.md: 2500 TFLOP/s
dense bf16, 8000 GB/s HBM).

usage: python scripts/launch_summary.py gpurun_out/<tag>_launch_table.json [--out profiles/<tag>_class_roofline.json]
"""
import argparse
import json

PEAK_TF, PEAK_GBS = 2500.0, 8000.0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("table")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    rows = json.load(open(a.table))
    cls = {}
    for r in rows:
        c = cls.setdefault(r["kind"], {"launches": 0, "ms": 0.0, "flops": 0.0, "bytes": 0.0, "floor_ms": 0.0})
        c["launches"] += 1
        c["ms"] += r["ms"]
        c["flops"] += r["flops"]
        c["bytes"] += r["bytes"]
        c["floor_ms"] += r["floor_ms"]
    out = []
    for k, c in sorted(cls.items(), key=lambda kv: -kv[1]["ms"]):
        s = c["ms"] * 1e-3
        tf = c["flops"] / s / 1e12 if s > 0 else 0.0
        gbs = c["bytes"] / s / 1e9 if s > 0 else 0.0
        bound = "mfma" if c["flops"] / PEAK_TF / 1e12 >= c["bytes"] / PEAK_GBS / 1e9 else "hbm"
        out.append({"kind": k, "launches": c["launches"], "ms": round(c["ms"], 4),
                    "achieved_tflops": round(tf, 1), "achieved_hbm_gbs": round(gbs, 1), "bound": bound,
                    "frac_of_bound_peak": round(c["floor_ms"] / c["ms"], 3) if c["ms"] > 0 else None})
    tot = sum(c["ms"] for c in cls.values())
    for o in out:
        print(f"{o['kind']:18s} {o['launches']:4d} {o['ms']:8.3f} ms ({100 * o['ms'] / tot:5.1f} %) "
              f"{o['achieved_tflops']:7.1f} TF/s {o['achieved_hbm_gbs']:7.1f} GB/s  {o['bound']:4s} "
              f"frac {o['frac_of_bound_peak']}")
    if a.out:
        json.dump({"peaks": {"bf16_tflops": PEAK_TF, "hbm_gbs": PEAK_GBS},
                   "note": "algorithmic flops/bytes per launch (bench.py run_gemm/run_attn accounting) over "
                           "HIP-event launch time of one profiled step; bytes = operands read once + "
                           "outputs written once",
                   "classes": out}, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
