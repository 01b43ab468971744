#!/bin/bash
# decoder classes with the pipeline serialised (--no-overlap: no backbone beside the decoder),
# fused self-attention block off / on, plus the isolated kernels
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
T="timeout -k 10"
{ $T 200 python scripts/kbench.py decsa --iters 50 && $T 200 python scripts/kbench.py xattn --iters 20; } > gpurun_out/dec2_kbench.log 2>&1 || { tail -20 gpurun_out/dec2_kbench.log; exit 4; }
cat gpurun_out/dec2_kbench.log | grep -v amdgpu.ids
for v in 0 1; do
  SPE_DECSA=$v $T 400 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-parity --no-overlap --launch-table gpurun_out/dec2_lt$v.json > gpurun_out/dec2_b$v.json 2> gpurun_out/dec2_b$v.err \
    || { tail -20 gpurun_out/dec2_b$v.err; exit 3; }
  python -c "
import json; d=json.loads(open('gpurun_out/dec2_b$v.json').read().strip().splitlines()[-1]); k=d['kernel_time_ms_per_step']
dec={x: round(k[x],3) for x in k if 'dec' in x or x in ('heads',)}
print('serial decsa=$v', round(d['value']), round(d['ms_per_step'],3), dec, 'decoder total', round(sum(dec.values()),3))"
done
