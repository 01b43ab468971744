#!/bin/bash
# fp32x6 LDS-DMA GEMM iteration: x6 kernel tests (register-staged + DMA), forward parity and the
# precision floor, the x6 GEMM microbenchmark (fp32x6bp = pre-split weights = the DMA kernel), the bench line.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
T="timeout -k 10"
$T 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_parity.py \
   tests/test_gpu_precision.py -k "x3_close or x6_dma or forward_fp32 or precision or linear_epilogue or vt or attention" > gpurun_out/f_tests.log 2>&1; rc=$?
tail -2 gpurun_out/f_tests.log; [ $rc = 0 ] || { grep -E "^E |FAILED" gpurun_out/f_tests.log | head -20; exit $rc; }
grep x6 gpurun_out/precision_floor.json
$T 300 python -u scripts/x6_bench.py > gpurun_out/f_x6bench.log 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/f_x6bench.log; [ $rc = 0 ] || exit $rc
$T 600 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/f_bench.json 2> gpurun_out/f_bench.err; rc=$?; python -c "
import json; d=json.loads(open('gpurun_out/f_bench.json').read().strip().splitlines()[-1]); p=d['parity_mode']
print('bf16', round(d['value']), 'parity', round(p['value']), p['ms_per_step'], {k: p['accuracy_vs_fp32'][k] for k in ('kpt_norm_max','frac_kpt_norm_le_1e-4','frac_score_delta_le_1e-4','meets_1e-4_kpt')})
print({k: round(v,2) for k,v in p['kernel_time_ms_per_step'].items()})"; exit $rc
