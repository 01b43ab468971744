#!/bin/bash
# Round 6: rocprofv3 kernel stats of the fp32h3 bench (current tree) + an un-profiled fp32h3 line.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${PROF_TAG:-r6f}
mkdir -p gpurun_out
BENCH_ARGS="--dtype fp32h3" PROF_TAG=${TAG}_fp32h3 bash scripts/gpu_profile.sh || exit 3
head -12 gpurun_out/prof_${TAG}_fp32h3/bench_kernel_stats_model.csv | cut -c1-150
timeout -k 10 600 python bench.py --dtype fp32h3 --steps 20 --warmup 3 --no-cpu-baseline --no-parity \
  --launch-table gpurun_out/${TAG}_lt_h3.json > gpurun_out/${TAG}_bench_h3.log 2>&1 || { tail -20 gpurun_out/${TAG}_bench_h3.log; exit 5; }
tail -1 gpurun_out/${TAG}_bench_h3.log | cut -c1-200
python3 scripts/launch_summary.py gpurun_out/${TAG}_lt_h3.json --out gpurun_out/${TAG}_class_roofline_h3.json > /dev/null
