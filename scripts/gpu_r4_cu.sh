#!/bin/bash
# CU partition between the backbone and encoder streams (SPE_CU_SPLIT = k eighths to the
# backbone): bench with k = 0 (off), 2, 3, 4, interleaved twice.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for rep in 1 2; do
  for k in 0 2 3 4; do
    SPE_CU_SPLIT=$k timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-parity --no-accuracy > gpurun_out/cu_$k.json 2> gpurun_out/cu_$k.err \
      || { tail -20 gpurun_out/cu_$k.err; exit 3; }
    python -c "
import json; d=json.loads(open('gpurun_out/cu_$k.json').read().strip().splitlines()[-1]); k=d['kernel_time_ms_per_step']
print('split=$k', round(d['value']), round(d['ms_per_step'],3), {x: round(k[x],3) for x in ('attn.enc','ffn.enc','conv.1x1','conv.3x3') if x in k})"
  done
done
