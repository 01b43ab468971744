#!/bin/bash
# precision gate + one bench line
set -o pipefail
mkdir -p gpurun_out
T="timeout -k 10"
$T 600 python -u -m pytest -x -q -s --timeout 500 --timeout-method thread tests/test_gpu_precision.py > gpurun_out/precision.log 2>&1; rc=$?; tail -3 gpurun_out/precision.log; cat gpurun_out/precision_floor.json; [ $rc = 0 ] || exit $rc
$T 600 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r4c_bench.json 2> gpurun_out/r4c_bench.err; rc=$?; python -c "
import json; d=json.loads(open('gpurun_out/r4c_bench.json').read().strip().splitlines()[-1]); p=d['parity_mode']
print('bf16', round(d['value']), 'parity', round(p['value']), p['ms_per_step'], {k: p['accuracy_vs_fp32'][k] for k in ('kpt_norm_max','frac_kpt_norm_le_1e-4','score_delta_max','frac_score_delta_le_1e-4','meets_1e-4_kpt')})"; exit $rc
