#!/bin/bash
# Round 6 final snapshot (tag r6z): rocprofv3 kernel stats (bf16 and fp32h3), per-class FETCH / WRITE
# passes (bf16 and fp32h3) and the fp32h3 attention's per-launch HBM bytes, then the default bench line
# (host_input, parity_mode fp32h3 with accuracy, CPU baseline, launch table), config 3 and the
# north-star line at N = 1.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
T=${PROF_TAG:-r6z}
mkdir -p gpurun_out
PROF_TAG=$T bash scripts/gpu_profile.sh > gpurun_out/${T}_prof_bf16.out 2>&1 || { tail -5 gpurun_out/${T}_prof_bf16.out; exit 1; }
echo "prof bf16 done"
BENCH_ARGS="--dtype fp32h3" PROF_TAG=${T}_fp32h3 bash scripts/gpu_profile.sh > gpurun_out/${T}_prof_h3.out 2>&1 || { tail -5 gpurun_out/${T}_prof_h3.out; exit 2; }
echo "prof fp32h3 done"
PMC_SUFFIX=_$T bash scripts/gpu_pmc_kinds.sh > gpurun_out/${T}_pmc_bf16.out 2>&1 || { tail -5 gpurun_out/${T}_pmc_bf16.out; exit 3; }
echo "pmc bf16 done"
BENCH_ARGS="--dtype fp32h3" PMC_SUFFIX=_${T}_h3 PMC_MODE=fp32h3 bash scripts/gpu_pmc_kinds.sh > gpurun_out/${T}_pmc_h3.out 2>&1 \
  || { tail -5 gpurun_out/${T}_pmc_h3.out; exit 4; }
echo "pmc fp32h3 done"
python3 - <<PY || exit 5
import json
c = json.load(open("gpurun_out/pmc_kinds_${T}_h3/pmc_kinds.json"))["classes"]["attn.enc"]
n = c["launches"]
d = {"kind": "attn.enc", "kernel": "attn_split_kernel<true>", "grid": 2883584, "attn_dtype": "fp32h3", "dispatches": n,
     "fetch_bytes_per_launch": c["fetch_MB"] * 1e6 / n, "write_bytes_per_launch": c["write_MB"] * 1e6 / n,
     "hbm_bytes_per_launch": (c["fetch_MB"] + c["write_MB"]) * 1e6 / n,
     "algorithmic_bytes_per_launch": c["algorithmic_MB"] * 1e6 / n,
     "note": "fp32h3 bench step serialised (--no-overlap), rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE in separate passes "
             "(scripts/gpu_pmc_kinds.sh); FETCH_SIZE x2 (gfx950); KiB -> bytes; memory-side L2 requests"}
json.dump(d, open("profiles/pmc_attn.enc_fp32h3.json", "w"), indent=1)
json.dump(d, open("gpurun_out/pmc_attn.enc_fp32h3.json", "w"), indent=1)
print("traffic", d["hbm_bytes_per_launch"] / 1e6, "MB per launch")
PY
timeout -k 10 900 python bench.py --steps 20 --warmup 3 --cpu-seconds 12 --launch-table gpurun_out/${T}_launch_table.json \
  > gpurun_out/${T}_bench.log 2>&1 || { tail -20 gpurun_out/${T}_bench.log; exit 6; }
tail -1 gpurun_out/${T}_bench.log | cut -c1-300
timeout -k 10 600 python bench.py --config 3 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/${T}_bench_c3.log 2>&1 \
  || { tail -20 gpurun_out/${T}_bench_c3.log; exit 7; }
tail -1 gpurun_out/${T}_bench_c3.log | cut -c1-200
timeout -k 10 800 python bench.py --north-star --no-cpu-baseline --no-host-input > gpurun_out/${T}_ns1.log 2>&1 \
  || { tail -20 gpurun_out/${T}_ns1.log; exit 8; }
tail -1 gpurun_out/${T}_ns1.log | cut -c1-200
echo final done
