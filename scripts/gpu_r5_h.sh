#!/bin/bash
# fp32h3 parity step: fused LN GEMM (non-persistent 256-wide tile) vs persistent GEMM + LayerNorm kernel
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for v in 0 3 0 3; do
  SPE_H3_LNSPLIT=$v timeout -k 10 300 python bench.py --dtype fp32h3 --no-parity --no-cpu-baseline --no-accuracy --steps 10 --warmup 2 \
    > gpurun_out/h_bench_$v.json 2> gpurun_out/h_bench_$v.err || { tail -20 gpurun_out/h_bench_$v.err; exit 4; }
  python -c "
import json; d=json.loads(open('gpurun_out/h_bench_$v.json').read().strip().splitlines()[-1]); k=d['kernel_time_ms_per_step']
print('lnsplit=$v', round(d['value']), round(d['ms_per_step'],2), {x: round(k[x],3) for x in ('gemm.enc.o','gemm.enc.ffn2','ln.enc','gemm.enc.ffn1','conv.1x1') if x in k})"
done
