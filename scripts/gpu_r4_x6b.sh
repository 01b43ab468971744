#!/bin/bash
# x6 tile A/B: kernel precision tests + the GEMM microbenchmark at both tile geometries
set -o pipefail
mkdir -p gpurun_out
T="timeout -k 10"
for tile in 256 128; do
  SPE_X6_TILE=$tile $T 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_kernels.py -k "x3_close" > gpurun_out/x6b_tests_$tile.log 2>&1; rc=$?; tail -1 gpurun_out/x6b_tests_$tile.log; [ $rc = 0 ] || exit $rc
  SPE_X6_TILE=$tile $T 300 python -u scripts/x6_bench.py > gpurun_out/x6b_bench_$tile.log 2>&1; rc=$?; echo "tile $tile"; grep -v amdgpu.ids gpurun_out/x6b_bench_$tile.log; [ $rc = 0 ] || exit $rc
done
