#!/bin/bash
# Bench the tree's libspe.so against several ablate/<name>/libspe.so variants, two interleaved
# passes ($LIBS: the variant names; "main" = the tree's library).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for pass in 1 2; do
  for v in $LIBS; do
    if [ "$v" = main ]; then unset SPE_LIB_PATH; else export SPE_LIB_PATH=ablate/$v/libspe.so; fi
    timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-accuracy $BENCH_ARGS > gpurun_out/abm_$v.log 2>&1 || { tail -20 gpurun_out/abm_$v.log; exit 3; }
    echo "$v $(tail -1 gpurun_out/abm_$v.log | grep -o '"value": [0-9.]*') $(tail -1 gpurun_out/abm_$v.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['kernel_time_ms_per_step']; print({x: round(k[x],3) for x in ${KEYS:-('attn.enc','ffn.enc','conv.1x1','conv.3x3')} if x in k})")"
  done
done
