"""Per-kernel PMC summary of scripts/lab/pmc_lab.sh output: clock, busy fractions, per-dispatch
VALU / MFMA figures.  usage: python scripts/lab/pmc_lab_summary.py gpurun_out/pmc_lab"""
import collections
import csv
import glob
import os
import sys

d = sys.argv[1]
rows = collections.defaultdict(lambda: collections.defaultdict(list))
durs = collections.defaultdict(list)
for f in sorted(glob.glob(os.path.join(d, "set*", "*counter_collection.csv"))):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].replace("(anonymous namespace)::", "")[:60]
        rows[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
        durs[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for k, c in rows.items():
    a = {n: sum(v) / len(v) for n, v in c.items()}
    us = sum(durs[k]) / len(durs[k])
    line = f"{k:60s} {us:8.1f}us"
    if "GRBM_GUI_ACTIVE" in a:
        clk = a["GRBM_GUI_ACTIVE"] / 8 / (us * 1e-6) / 1e9
        cyc = a["GRBM_GUI_ACTIVE"] / 8
        line += f" clk={clk:.2f}GHz"
        if "SQ_VALU_MFMA_BUSY_CYCLES" in a:
            line += f" mfma={a['SQ_VALU_MFMA_BUSY_CYCLES'] / (cyc * 1024):.2f}"
        if "SQ_ACTIVE_INST_VALU" in a:
            line += f" valu={a['SQ_ACTIVE_INST_VALU'] * 4 / (cyc * 1024):.2f}"
        if "SQ_ACTIVE_INST_ANY" in a:
            line += f" any={a['SQ_ACTIVE_INST_ANY'] * 4 / (cyc * 1024):.2f}"
        if "SQ_WAVE_CYCLES" in a:
            line += f" waves/simd={a['SQ_WAVE_CYCLES'] * 4 / (cyc * 1024):.2f}"
        if "SQ_WAIT_INST_ANY" in a:
            line += f" waitinst={a['SQ_WAIT_INST_ANY'] * 4 / (cyc * 1024):.2f}"
        if "SQ_WAIT_ANY" in a:
            line += f" wait={a['SQ_WAIT_ANY'] * 4 / (cyc * 1024):.2f}"
    if "SQ_INSTS_VALU" in a:
        line += f" valu_insts={a['SQ_INSTS_VALU'] / 1e6:.1f}M"
    print(line)
