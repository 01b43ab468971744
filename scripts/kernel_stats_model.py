"""Per-kernel statistics of the path's own kernels from a rocprofv3 kernel trace.

rocprofv3 --stats counts every dispatch of the process, so bench setup (the point-head fit's
hipBLASLt GEMMs and torch element-wise kernels) dominates its percentages.  This rewrites the
summary over libspe's kernels only (the anonymous-namespace symbols of csrc/), in the same
columns as rocprofv3's kernel_stats.csv, so "Percentage" is a share of the pipeline's kernel time.
    python scripts/kernel_stats_model.py <dir with *kernel_trace.csv> --out stats_model.csv
"""
import argparse
import csv
import glob
import os
from collections import defaultdict

EXCLUDE = ("Cijk_", "at::", "void at", "rocprim", "hipcub", "Memcpy", "__amd_rocclr")
# libspe's kernels (csrc/*.hip); torch's own anonymous-namespace kernels (e.g. the point-head
# fit's indexing_backward_kernel) match none of these stems
OURS = ("attn", "ffn_", "gemm", "lnproj", "pconv", "btail", "stempool", "layernorm", "heads", "pnp", "maxpool",
        "upconv", "upsample", "pack_input", "postprocess", "score", "xattn", "jpeg", "preprocess", "self_assess",
        "ensemble", "criterion", "msdeform", "query_select", "head_finish", "resample", "qpos", "ransac", "sigma",
        "speed", "fuse", "crop", "idct", "huff", "unstuff", "parse")


def main():
    p = argparse.ArgumentParser()
    p.add_argument("trace_dir")
    p.add_argument("--out", required=True)
    a = p.parse_args()
    dur = defaultdict(list)
    for f in glob.glob(os.path.join(a.trace_dir, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            n = r["Kernel_Name"]
            if any(x in n for x in EXCLUDE) or not any(x in n for x in OURS):
                continue
            dur[n].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    total = sum(sum(v) for v in dur.values()) or 1
    rows = sorted(dur.items(), key=lambda kv: -sum(kv[1]))
    with open(a.out, "w", newline="") as fo:
        w = csv.writer(fo)
        w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs"])
        for n, v in rows:
            w.writerow([n, len(v), sum(v), sum(v) / len(v), 100.0 * sum(v) / total, min(v), max(v)])
    print(f"{len(rows)} kernels, {sum(len(v) for v in dur.values())} dispatches, {total / 1e6:.1f} ms")


if __name__ == "__main__":
    main()
