#!/bin/bash
# A/B of the tree's libspe.so against ablate/old/libspe.so: affected kernel tests ($TESTK), kbench
# ($KB) and the default bench, interleaved.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
if [ -n "$TESTK" ]; then
  timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -m gpu -k "$TESTK" > gpurun_out/ab_t.log 2>&1 || { tail -30 gpurun_out/ab_t.log; exit 1; }
  tail -1 gpurun_out/ab_t.log
fi
if [ -n "$KB" ]; then
  LIBS="old main" KB="$KB" bash scripts/ab_libs.sh 2>&1 | grep -v amdgpu.ids || exit 2
fi
for v in old main old main; do
  if [ "$v" = main ]; then unset SPE_LIB_PATH; else export SPE_LIB_PATH=ablate/$v/libspe.so; fi
  timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-accuracy $BENCH_ARGS > gpurun_out/ab_b_$v.log 2>&1 || { tail -20 gpurun_out/ab_b_$v.log; exit 3; }
  echo "$v $(tail -1 gpurun_out/ab_b_$v.log | grep -o '"value": [0-9.]*') $(tail -1 gpurun_out/ab_b_$v.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['kernel_time_ms_per_step']; print({x: round(k[x],3) for x in ('attn.enc','ffn.enc','conv.1x1','conv.3x3','gemm.enc.qk','gemm.enc.o','gemm.enc.v','conv.neck') if x in k})")"
done
