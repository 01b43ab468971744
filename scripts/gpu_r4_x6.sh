#!/bin/bash
# fp32x6 iteration: kernel precision tests, the parity-GEMM microbenchmark, the x6 precision row
set -o pipefail
mkdir -p gpurun_out
T="timeout -k 10"
$T 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_kernels.py -k "x3_close" > gpurun_out/x6_tests.log 2>&1; rc=$?; tail -2 gpurun_out/x6_tests.log; [ $rc = 0 ] || exit $rc
$T 300 python -u scripts/x6_bench.py > gpurun_out/x6_bench.log 2>&1; rc=$?; cat gpurun_out/x6_bench.log | grep -v amdgpu.ids; [ $rc = 0 ] || exit $rc
$T 400 python -u scripts/x3_sensitivity.py --variants "fp32x6;only enc_attn split" --out gpurun_out/x6_sens.json > gpurun_out/x6_sens.log 2>&1; rc=$?; grep -o '"kpt_norm_max": [0-9.e-]*\|"hs_rel_max": [0-9.e-]*\|"ms": [0-9.]*\|"variant": "[^"]*"' gpurun_out/x6_sens.log; exit $rc
