"""Per launch-class HBM traffic of one bench step from rocprofv3 FETCH_SIZE / WRITE_SIZE passes.

Run the bench serialised on one stream with its launch table, once per counter (scripts/gpu_pmc_kinds.sh):
    rocprofv3 --kernel-trace --pmc FETCH_SIZE -- python3 bench.py --no-overlap --steps 1 ... --launch-table lt.json
then
    python scripts/pmc_kinds.py gpurun_out/pmc_kinds --table lt.json --out profiles/r4_pmc_kinds.json

The launch table lists the step's model launches in issue order (kind, algorithmic bytes); the
rocprofv3 dispatches of the LAST step are aligned to it backwards: every GEMM / conv / LayerNorm /
element-wise / heads record is one dispatch, an FFN or decoder cross-attention record is the run
of consecutive dispatches of its kernel family.  Solver, score and torch kernels are skipped.
Corrections (MI355X_MICROARCH.md, HBM): the counters are KiB; FETCH_SIZE is doubled on gfx950 for
16-B/lane streaming reads.  Memory-side L2 requests: an upper bound on HBM bytes.
"""
import argparse
import csv
import glob
import json
import os
from collections import defaultdict

SKIP = ("pnp_", "score_kernel", "self_assess", "at::", "void at", "rocprim", "hipcub", "__amd_rocclr", "Cijk")
FAMILY = {"attn.enc": ("attn16", "attn_x3", "attn_split", "attn_f32"), "attn.dec_self": ("attn16", "attn_f32"),
          "attn.dec_cross": ("xattn", "attn_f32"),
          "ffn.enc": ("ffn_",), "ffn.dec": ("ffn_",)}


def family(kind):
    for k, v in FAMILY.items():
        if kind == k:
            return v
    return None


def load(dirname, counter):
    rows = []
    for f in sorted(glob.glob(os.path.join(dirname, "**", "*counter_collection.csv"), recursive=True)):
        for r in csv.DictReader(open(f)):
            if r.get("Counter_Name") != counter:
                continue
            rows.append((int(r["Dispatch_Id"]), r["Kernel_Name"], float(r["Counter_Value"])))
    agg = defaultdict(float)
    names = {}
    for d, n, v in rows:                      # one row per dispatch (summed over XCD instances)
        agg[d] += v
        names[d] = n
    return [(d, names[d], agg[d]) for d in sorted(agg)]


def align(disp, table):
    """Backwards alignment of the last step's dispatches to the table's records."""
    disp = [x for x in disp if not any(s in x[1] for s in SKIP)]
    out = [None] * len(table)
    j = len(disp) - 1
    for i in range(len(table) - 1, -1, -1):
        fam = family(table[i]["kind"])
        if fam is None:
            out[i] = [disp[j]]
            j -= 1
        else:
            grp = []
            while j >= 0 and any(f in disp[j][1] for f in fam):
                grp.append(disp[j])
                j -= 1
            if not grp:
                raise SystemExit(f"alignment failed at record {i} ({table[i]['kind']}): {disp[j][1]}")
            out[i] = grp[::-1]
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--table", required=True)
    ap.add_argument("--out", default=None)
    ap.add_argument("--mode", default="bf16", help="the bench dtype the passes ran (recorded in the note)")
    a = ap.parse_args()
    table = json.load(open(a.table))
    res = defaultdict(lambda: {"launches": 0, "algorithmic_bytes": 0.0, "fetch_bytes": 0.0, "write_bytes": 0.0,
                               "kernels": set()})
    for counter, key, scale in (("FETCH_SIZE", "fetch_bytes", 2 * 1024.0), ("WRITE_SIZE", "write_bytes", 1024.0)):
        disp = load(os.path.join(a.dir, counter), counter)
        for rec, grp in zip(table, align(disp, table)):
            r = res[rec["kind"]]
            r[key] += sum(v for _, _, v in grp) * scale
            for _, n, _ in grp:
                r["kernels"].add(n.replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0][:80])
    for rec in table:
        r = res[rec["kind"]]
        r["launches"] += 1
        r["algorithmic_bytes"] += rec["bytes"]
    out = {}
    for k, r in res.items():
        tb = r["fetch_bytes"] + r["write_bytes"]
        out[k] = {"launches": r["launches"], "algorithmic_MB": r["algorithmic_bytes"] / 1e6,
                  "fetch_MB": r["fetch_bytes"] / 1e6, "write_MB": r["write_bytes"] / 1e6,
                  "counter_over_algorithmic": tb / r["algorithmic_bytes"] if r["algorithmic_bytes"] else None,
                  "kernels": sorted(r["kernels"])}
    s = json.dumps({"note": f"per bench step (B=64, config 2, {a.mode}, serialised --no-overlap); FETCH x2 (gfx950), KiB->B",
                    "classes": out}, indent=1)
    print(s)
    if a.out:
        open(a.out, "w").write(s)


if __name__ == "__main__":
    main()
