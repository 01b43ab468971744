"""Turn a FETCH_SIZE / WRITE_SIZE rocprofv3 PMC run (scripts/gpu_pmc.sh) into the per-launch
HBM traffic figure bench.py reports as roofline.traffic.

usage: python scripts/pmc_traffic.py gpurun_out/pmc_<tag> --kernel attn16_kernel --kind attn.enc \
           [--grid 2883584] [--out profiles/pmc_attn.enc.json]

Corrections (MI355X_MICROARCH.md, "HBM"): FETCH_SIZE and WRITE_SIZE are in KiB; on gfx950
FETCH_SIZE reports half of the bytes of 16-B/lane streaming reads, so it is doubled.  The
counters are memory-side L2 requests (Infinity-Cache hits included), i.e. an upper bound on
HBM bytes.
"""
import argparse
import csv
import glob
import json
import os


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--kernel", required=True)
    ap.add_argument("--kind", required=True)
    ap.add_argument("--grid", type=int, default=None, help="only dispatches with this grid size (the bench shape)")
    ap.add_argument("--out", default=None)
    ap.add_argument("--attn-dtype", default="bf16", help="operand type of the profiled attention launches")
    a = ap.parse_args()
    vals = {"FETCH_SIZE": [], "WRITE_SIZE": []}
    for f in glob.glob(os.path.join(a.dir, "set*", "*counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            if a.kernel not in r["Kernel_Name"]:
                continue
            if a.grid and int(r["Grid_Size"]) != a.grid:
                continue
            if r["Counter_Name"] in vals:
                vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
    if not vals["FETCH_SIZE"] or not vals["WRITE_SIZE"]:
        raise SystemExit("no matching dispatches with both counters")
    fetch = 2.0 * 1024 * sum(vals["FETCH_SIZE"]) / len(vals["FETCH_SIZE"])
    write = 1024.0 * sum(vals["WRITE_SIZE"]) / len(vals["WRITE_SIZE"])
    out = {"kind": a.kind, "kernel": a.kernel, "grid": a.grid, "attn_dtype": a.attn_dtype,
           "dispatches": len(vals["FETCH_SIZE"]),
           "fetch_bytes_per_launch": fetch, "write_bytes_per_launch": write,
           "hbm_bytes_per_launch": fetch + write,
           "note": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE in separate passes; FETCH_SIZE x2 (gfx950 "
                   "16-B/lane read correction); KiB -> bytes; memory-side L2 requests (MALL hits included)"}
    print(json.dumps(out, indent=1))
    if a.out:
        json.dump(out, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
