#!/bin/bash
# decoder: xattn with the shared pos table + out-projection/norm through lnproj.  Kernel tests and
# bf16 forward tests, kbench decsa, then the bench with the per-image out-projection + norm off / on.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
T="timeout -k 10"
$T 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_parity.py tests/test_gpu_pipeline.py \
   -k "decoder_out_projection or decoder_self_attention or cross_attention or lnproj or forward or batch_independence or golden or pipeline or sigma" > gpurun_out/dec_tests.log 2>&1; rc=$?
tail -2 gpurun_out/dec_tests.log; [ $rc = 0 ] || { grep -E "^E |FAILED" gpurun_out/dec_tests.log | head -20; exit $rc; }
{ $T 200 python scripts/kbench.py decsa --iters 50; } > gpurun_out/dec_kbench.log 2>&1 || { tail -20 gpurun_out/dec_kbench.log; exit 4; }
cat gpurun_out/dec_kbench.log
for v in 0 1 0 1; do
  SPE_DECPROJ=$v $T 400 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-parity > gpurun_out/dec_b$v.json 2> gpurun_out/dec_b$v.err \
    || { tail -20 gpurun_out/dec_b$v.err; exit 3; }
  python -c "
import json; d=json.loads(open('gpurun_out/dec_b$v.json').read().strip().splitlines()[-1]); k=d['kernel_time_ms_per_step']
print('decproj=$v', round(d['value']), round(d['ms_per_step'],3), {x: round(k[x],3) for x in k if 'dec' in x or x in ('heads','attn.enc')}, d['accuracy_vs_fp32']['kpt_norm_max'] if 'accuracy_vs_fp32' in d else '')"
done
