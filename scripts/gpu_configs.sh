#!/bin/bash
# BASELINE configs 3-5 at their per-GPU shapes (1 GPU), after the GPU test suite.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 \
  || { echo "pytest failed"; tail -30 gpurun_out/pytest_gpu.log; exit 2; }
tail -2 gpurun_out/pytest_gpu.log
for c in ${CONFIGS:-3 4 5}; do
  timeout -k 10 600 python bench.py --config $c --steps ${BENCH_STEPS:-10} --warmup 2 --cpu-seconds 10 > gpurun_out/bench_c$c.log 2>&1 \
    || { echo "bench config $c failed"; tail -30 gpurun_out/bench_c$c.log; exit 3; }
  tail -1 gpurun_out/bench_c$c.log | cut -c1-600
done
