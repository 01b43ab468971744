#!/bin/bash
# Round 5: the one-pass fp32h3 FFN kernel test, the score-spread study with fp32h3 (tests/test_gpu_precision.py)
# and the default bench line (parity mode fp32h3)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
T="timeout -k 10"
$T 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_kernels.py -k "ffn_h3 or h3_close" \
  > gpurun_out/o_k.log 2>&1 || { grep -E "^E |FAILED|Error" gpurun_out/o_k.log | head -20; tail -3 gpurun_out/o_k.log; exit 2; }
tail -1 gpurun_out/o_k.log
$T 1000 python -u -m pytest -x -v --timeout 950 --timeout-method thread tests/test_gpu_precision.py \
  > gpurun_out/o_precision.log 2>&1 || { grep -E "^E |FAILED|Error" gpurun_out/o_precision.log | head -20; tail -5 gpurun_out/o_precision.log; exit 3; }
tail -2 gpurun_out/o_precision.log
$T 600 python bench.py > gpurun_out/o_bench.json 2> gpurun_out/o_bench.err || { tail -20 gpurun_out/o_bench.err; exit 4; }
python -c "
import json; d=json.loads(open('gpurun_out/o_bench.json').read().strip().splitlines()[-1]); p=d['parity_mode']; a=p['accuracy_vs_fp32']
print('bf16', round(d['value']), round(d['ms_per_step'],2), 'frac', round(d['roofline']['frac'],3), '| parity', p['dtype'], round(p['value']), round(p['ms_per_step'],2), 'kpt', a['kpt_norm_max'], 'score<=1e-4', a['frac_score_delta_le_1e-4'], 'wc', a['frac_score_delta_le_1e-4_well_conditioned'], '| cpu', d['cpu_baseline']['value'])"
