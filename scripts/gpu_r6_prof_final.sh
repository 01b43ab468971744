#!/bin/bash
# Round 6, the final tree's profiles (tag r6j): rocprofv3 kernel stats of the default (bf16) and the
# fp32h3 bench runs, and the fp32h3 per-class FETCH / WRITE passes.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
PROF_TAG=r6j bash scripts/gpu_profile.sh || exit 1
PROF_TAG=r6j_fp32h3 BENCH_ARGS="--dtype fp32h3" bash scripts/gpu_profile.sh || exit 2
PMC_SUFFIX=_r6j_fp32h3 PMC_MODE=fp32h3 BENCH_ARGS="--dtype fp32h3" bash scripts/gpu_pmc_kinds.sh || exit 3
python3 - <<'PY'
import json
d = json.load(open("gpurun_out/pmc_kinds_r6j_fp32h3/pmc_kinds.json"))
for k, v in d["classes"].items():
    if "dec" in k:
        print(k, v["launches"], round(v["algorithmic_MB"], 1), round(v["fetch_MB"], 1), round(v["write_MB"], 1), v["counter_over_algorithmic"])
PY
echo done
