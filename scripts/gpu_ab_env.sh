#!/bin/bash
# A/B of one environment knob on the tree's libspe.so: kernel tests ($TESTK, knob at its default),
# then the bench with $VAR=$A and $VAR=$B interleaved.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
if [ -n "$TESTK" ]; then
  timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_parity.py tests/test_gpu_pipeline.py -x -q --timeout 120 --timeout-method thread -m gpu -k "$TESTK" > gpurun_out/ab_t.log 2>&1 || { tail -30 gpurun_out/ab_t.log; exit 1; }
  tail -1 gpurun_out/ab_t.log
fi
for v in $A $B $A $B; do
  env $VAR=$v timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-accuracy $BENCH_ARGS > gpurun_out/ab_e_$v.log 2>&1 || { tail -20 gpurun_out/ab_e_$v.log; exit 3; }
  echo "$VAR=$v $(tail -1 gpurun_out/ab_e_$v.log | grep -o '"value": [0-9.]*') $(tail -1 gpurun_out/ab_e_$v.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['kernel_time_ms_per_step']; print({x: round(k[x],3) for x in ${KEYS:-('attn.enc','ffn.enc','conv.1x1','gemm.enc.qk','gemm.enc.o','conv.neck')} if x in k})")"
done
