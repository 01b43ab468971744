#!/bin/bash
# full-bank weight swizzle (btail / sgemm / lnproj): kernel + bf16 forward tests, kbench and bench A/B
# against ablate/pre (the tree before the change)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
T="timeout -k 10"
$T 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_parity.py \
   -k "btail or gemm or bf16 or ln or stream or vt" > gpurun_out/swz_tests.log 2>&1; rc=$?
tail -2 gpurun_out/swz_tests.log; [ $rc = 0 ] || { grep -E "^E |FAILED" gpurun_out/swz_tests.log | head -20; exit $rc; }
for v in pre main pre main; do
  if [ "$v" = main ]; then unset SPE_LIB_PATH; else export SPE_LIB_PATH=ablate/$v/libspe.so; fi
  echo "== $v"; $T 120 python scripts/kbench.py btail --iters 20 2>&1 | grep btail
  $T 120 python scripts/kbench.py gemm --iters 20 2>&1 | grep -E "l1.c|enc|l2|l3" | head -12
done
for v in pre main pre main; do
  if [ "$v" = main ]; then unset SPE_LIB_PATH; else export SPE_LIB_PATH=ablate/$v/libspe.so; fi
  $T 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-accuracy --no-parity > gpurun_out/swz_b_$v.json 2> gpurun_out/swz_b_$v.err || { tail -20 gpurun_out/swz_b_$v.err; exit 3; }
  python -c "
import json; d=json.loads(open('gpurun_out/swz_b_$v.json').read().strip().splitlines()[-1]); k=d['kernel_time_ms_per_step']
print('$v', round(d['value']), round(d['ms_per_step'],3), {x: round(k[x],3) for x in ('conv.1x1','gemm.enc.qk','gemm.enc.o','gemm.enc.v','conv.neck','attn.enc') if x in k})"
done
