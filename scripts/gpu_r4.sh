#!/bin/bash
# Round-4 GPU session steps: targeted parity tests, the parity-GEMM microbenchmark, the x3/x6
# precision study, one bench line.  Every GPU step has its own time limit; the chain stops at the
# first failure.
set -o pipefail
mkdir -p gpurun_out
T="timeout -k 10"
step() { echo "== $1"; }
step tests && $T 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_capi.py \
    tests/test_gpu_kernels.py -k "x3_close or gemm_linear or capi" > gpurun_out/r4_tests.log 2>&1; rc=$?; tail -3 gpurun_out/r4_tests.log; [ $rc = 0 ] || exit $rc
step parity && $T 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py \
    tests/test_reference_front.py tests/test_jpeg.py tests/test_gpu_kernels.py -m gpu -k "forward_fp32 or ceres or pnp or sigma or selection or jpeg or stempool" \
    > gpurun_out/r4_parity.log 2>&1; rc=$?; tail -3 gpurun_out/r4_parity.log; [ $rc = 0 ] || exit $rc
step x6bench && $T 300 python -u scripts/x6_bench.py > gpurun_out/r4_x6bench.log 2>&1; rc=$?; cat gpurun_out/r4_x6bench.log; [ $rc = 0 ] || exit $rc
step sens && $T 400 python -u scripts/x3_sensitivity.py --variants "fp32x6;x3 (all split);only enc_attn split" --out gpurun_out/r4_sens.json > gpurun_out/r4_sens.log 2>&1; rc=$?; tail -4 gpurun_out/r4_sens.log; [ $rc = 0 ] || exit $rc
step bench && $T 600 python -u bench.py --steps 10 --warmup 3 > gpurun_out/r4_bench.json 2> gpurun_out/r4_bench.err; rc=$?; tail -c 3000 gpurun_out/r4_bench.json; exit $rc
