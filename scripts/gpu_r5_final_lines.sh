#!/bin/bash
# Round-5 final tree: BASELINE configs 3-5 and the north-star line on one GPU (global batch 256).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${PROF_TAG:-r5h}
mkdir -p gpurun_out
for c in 3 4 5; do
  np=--no-parity; [ $c = 3 ] && np=
  timeout -k 10 600 python bench.py --config $c --steps 10 --warmup 2 --no-cpu-baseline $np > gpurun_out/${TAG}_bench_c$c.log 2>&1 \
    || { tail -20 gpurun_out/${TAG}_bench_c$c.log; exit 5; }
  tail -1 gpurun_out/${TAG}_bench_c$c.log | cut -c1-120
done
timeout -k 10 800 python bench.py --north-star --no-cpu-baseline > gpurun_out/${TAG}_ns1.log 2>&1 || { tail -20 gpurun_out/${TAG}_ns1.log; exit 6; }
tail -1 gpurun_out/${TAG}_ns1.log | cut -c1-160
