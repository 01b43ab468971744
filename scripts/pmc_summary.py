"""Summarise rocprofv3 --pmc CSVs (scripts/gpu_pmc.sh output) per (kernel, grid size).

usage: python scripts/pmc_summary.py gpurun_out/pmc_<tag> [--min-us 20] [--json out.json]
FETCH_SIZE is doubled (gfx950 reports half of the bytes of 16-B/lane streaming reads,
MI355X_MICROARCH.md "HBM"); SQ cycle counters are quad-cycles.
"""
import argparse
import collections
import csv
import glob
import json
import os


def short(name):
    n = name.replace("(anonymous namespace)::", "")
    for key in ("attn_split_kernel", "ffn_h3_kernel", "gemm_h3d", "gemm_x6d_kernel", "gemm_x6_kernel", "attn_x3_kernel", "sgemm_kernel", "gemm2_kernel", "gemm_kernel", "ffn_pipe_kernel", "attn_bf16", "attn_f32", "ffn_ln", "layernorm", "heads", "pnp_kernel",
                "maxpool", "upsample", "pack_input", "postprocess", "score"):
        if key in n:
            return n[n.find(key):].replace("(GemmArgs", "(").split("(")[0][:64]
    return n[-40:]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--min-us", type=float, default=20.0)
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    rows = collections.defaultdict(lambda: collections.defaultdict(list))
    dur = collections.defaultdict(list)
    for f in sorted(glob.glob(os.path.join(a.dir, "set*", "*counter_collection.csv"))):
        for r in csv.DictReader(open(f)):
            key = (short(r["Kernel_Name"]), int(r["Grid_Size"]))
            v = float(r["Counter_Value"])
            if r["Counter_Name"] == "FETCH_SIZE":
                v *= 2.0
            rows[key][r["Counter_Name"]].append(v)
            dur[key].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    out = []
    for key, cs in rows.items():
        us = sum(dur[key]) / len(dur[key])
        if us < a.min_us:
            continue
        avg = {c: sum(v) / len(v) for c, v in cs.items()}
        out.append({"kernel": key[0], "grid": key[1], "us": us, **avg})
    out.sort(key=lambda d: -d["us"])
    for d in out:
        line = f"{d['kernel']:32s} grid={d['grid']:9d} {d['us']:8.1f}us"
        if "FETCH_SIZE" in d:
            line += f" fetch={d['FETCH_SIZE'] / 1e3 / max(d['us'], 1e-9):6.2f}TB/s"
        if "WRITE_SIZE" in d:
            line += f" write={d['WRITE_SIZE'] / 1e3 / max(d['us'], 1e-9):6.2f}TB/s"
        wc = d.get("SQ_WAVE_CYCLES")
        if wc:
            for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU"):
                if c in d:
                    line += f" {c[3:]}={d[c] / wc:.2f}"
        if "SQ_VALU_MFMA_BUSY_CYCLES" in d and "GRBM_GUI_ACTIVE" in d:
            # MFMA-busy cycles per SIMD over the dispatch: GRBM_GUI_ACTIVE sums the 8 XCDs' clocks,
            # the chip has 1024 SIMDs (MI355X_MICROARCH.md PMC notes)
            line += f" mfma_busy={d['SQ_VALU_MFMA_BUSY_CYCLES'] / (d['GRBM_GUI_ACTIVE'] / 8 * 1024):.2f}"
            line += f" clk={d['GRBM_GUI_ACTIVE'] / 8 / d['us'] / 1e3:.2f}GHz"
        if "SQ_INSTS_MFMA" in d and d["SQ_INSTS_MFMA"]:
            line += f" valu/mfma={d.get('SQ_INSTS_VALU', 0) / d['SQ_INSTS_MFMA']:.2f}"
            if "SQ_VALU_MFMA_COEXEC_CYCLES" in d and "SQ_VALU_MFMA_BUSY_CYCLES" in d:
                line += f" coexec={d['SQ_VALU_MFMA_COEXEC_CYCLES'] / max(d['SQ_VALU_MFMA_BUSY_CYCLES'], 1):.2f}"
        if "SQ_LDS_BANK_CONFLICT" in d and "SQ_LDS_IDX_ACTIVE" in d:
            line += f" lds_conf={d['SQ_LDS_BANK_CONFLICT'] / max(d['SQ_LDS_IDX_ACTIVE'], 1):.2f}"
        print(line)
    if a.json:
        json.dump(out, open(a.json, "w"), indent=1)


if __name__ == "__main__":
    main()
