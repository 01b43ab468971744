#!/bin/bash
# fp32x3 / fp32 attention iteration: attention + forward parity tests, kbench A/B of the x3 and
# fp32 attention kernels over ablate/{old,x3u0} and the tree's library, pconv (3x3) old vs tree,
# then the bench line.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
T="timeout -k 10"
$T 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_parity.py \
   tests/test_gpu_precision.py -k "attention or forward_fp32 or precision or patch_conv" > gpurun_out/e_tests.log 2>&1; rc=$?
tail -2 gpurun_out/e_tests.log; grep x6 gpurun_out/precision_floor.json; [ $rc = 0 ] || exit $rc
for rep in 1 2; do
  for v in old x3u0 main; do
    if [ "$v" = main ]; then unset SPE_LIB_PATH; else export SPE_LIB_PATH=ablate/$v/libspe.so; fi
    echo "== $v $($T 120 python scripts/kbench.py attn --attn-dtype 4 --iters 20 2>&1 | grep attn.enc) | fp32 $($T 120 python scripts/kbench.py attn --attn-dtype 1 --iters 10 2>&1 | grep attn.enc)" || exit 2
  done
done
unset SPE_LIB_PATH
LIBS="old main" KB="gemm --only 3x3" bash scripts/ab_libs.sh 2>&1 | grep -v amdgpu.ids || exit 3
$T 600 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/e_bench.json 2> gpurun_out/e_bench.err; rc=$?; python -c "
import json; d=json.loads(open('gpurun_out/e_bench.json').read().strip().splitlines()[-1]); p=d['parity_mode']
print('bf16', round(d['value']), 'parity', round(p['value']), p['ms_per_step'], {k: p['accuracy_vs_fp32'][k] for k in ('kpt_norm_max','frac_kpt_norm_le_1e-4','frac_score_delta_le_1e-4','meets_1e-4_kpt')})
print({k: round(v,2) for k,v in p['kernel_time_ms_per_step'].items()})
print({k: round(v,3) for k,v in d['kernel_time_ms_per_step'].items()})"; exit $rc
