#!/bin/bash
# split-N bottleneck tail: kernel tests + bf16 forward tests, then the bench with the split tail
# off / on (SPE_BTAIL_SPLIT), interleaved.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
T="timeout -k 10"
$T 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_parity.py \
   -k "btail or forward_bf16 or batch_independence or forward_fp32" > gpurun_out/h_tests.log 2>&1; rc=$?
tail -2 gpurun_out/h_tests.log; [ $rc = 0 ] || { grep -E "^E |FAILED" gpurun_out/h_tests.log | head -20; exit $rc; }
for v in 0 1 0 1; do
  SPE_BTAIL_SPLIT=$v $T 400 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-parity > gpurun_out/h_b$v.json 2> gpurun_out/h_b$v.err \
    || { tail -20 gpurun_out/h_b$v.err; exit 3; }
  python -c "
import json; d=json.loads(open('gpurun_out/h_b$v.json').read().strip().splitlines()[-1]); k=d['kernel_time_ms_per_step']
print('split=$v', round(d['value']), round(d['ms_per_step'],3), {x: round(k[x],3) for x in ('conv.1x1','conv.3x3','attn.enc','ffn.enc') if x in k}, d['accuracy_vs_fp32']['kpt_norm_max'] if 'accuracy_vs_fp32' in d else '')"
done
