#!/bin/bash
# Round 6 A/B: HIP stream priorities of the pipeline's encoder / decoder streams (scheduling only:
# results bit-identical) on the fp32h3 and bf16 lines, alternating.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for rep in 1 2; do
for p in "" "encode:-1" "encode:-1,decode:-1" "decode:-1"; do
  for dt in fp32h3 bf16; do
    SPE_STREAM_PRIORITY="$p" timeout -k 10 400 python bench.py --dtype $dt --no-parity --no-accuracy --no-cpu-baseline --no-host-input --steps 10 --warmup 3 \
      > gpurun_out/r6pr.json 2> gpurun_out/r6pr.err || { tail -5 gpurun_out/r6pr.err; exit 3; }
    python3 -c "import json; r=json.loads(open('gpurun_out/r6pr.json').read().strip().splitlines()[-1]); print('$dt', '[$p]', round(r['value'],1), round(r['ms_per_step'],3))"
  done
done
done
