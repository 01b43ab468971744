#!/bin/bash
# Same-box A/B of the decoder's 16-row kernels (SPE_DECFFN) at 256 images per GPU (the one-GPU north-star shape).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for i in 1 2; do
  for v in 0 1; do
    SPE_DECFFN=$v timeout -k 10 300 python bench.py --config 3 --batch 256 --steps 10 --warmup 3 --no-cpu-baseline --no-accuracy --no-parity \
      > gpurun_out/ab256_${v}_$i.json 2> gpurun_out/ab256_${v}_$i.err || { tail -5 gpurun_out/ab256_${v}_$i.err; exit 3; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); k=d['kernel_time_ms_per_step']; print(sys.argv[2], round(d['value'],1), round(d['ms_per_step'],2), {x: round(k[x],3) for x in ('ffn.dec','gemm.dec','conv.1x1','attn.enc') if x in k})" gpurun_out/ab256_${v}_$i.json "decffn=$v run $i"
  done
done
