#!/bin/bash
# Round 6: the fp32h3 decoder fold -- kernel stats of the fp32h3 line, then the config-2 precision
# study (fp32 implementation spread) and the per-config fp32h3 spread tests.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
PROF_TAG=r6r_h3 BENCH_ARGS="--dtype fp32h3" bash scripts/gpu_profile.sh || exit 1
grep -E "xattn|gemm_h3|Name" gpurun_out/prof_r6r_h3/bench_kernel_stats.csv | cut -d, -f1-8 | head -20
timeout -k 10 1000 python -u -m pytest tests/test_gpu_precision.py -m gpu -x -q --timeout 900 --timeout-method thread > gpurun_out/r6r_precision.log 2>&1 \
  || { grep -E "^E |FAILED|Error|assert" gpurun_out/r6r_precision.log | head -30; tail -5 gpurun_out/r6r_precision.log; exit 2; }
tail -3 gpurun_out/r6r_precision.log
