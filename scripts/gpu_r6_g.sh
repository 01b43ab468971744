#!/bin/bash
# Round 6 experiment: the fp32h3 split attention with P as one fp16 term (SPE_ATTN_P16=1) -- kbench
# timing and the precision study with it, against the default (P split hi / lo).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${PROF_TAG:-r6g}
mkdir -p gpurun_out
for v in "" "--p16"; do
  timeout -k 10 120 python3 scripts/kbench.py attn --attn-dtype 4 --presplit --split-dma --f16v $v --iters 20 2>&1 | grep attn || exit 2
done
SPE_ATTN_P16=1 timeout -k 10 900 python -u -m pytest tests/test_gpu_precision.py -x -q -s --timeout 900 --timeout-method thread \
  > gpurun_out/${TAG}_precision_p16.log 2>&1
echo "precision p16 rc=$?"
cp gpurun_out/precision_score.json gpurun_out/${TAG}_precision_score_p16.json
grep -E "passed|failed" gpurun_out/${TAG}_precision_p16.log | tail -2
SPE_ATTN_P16=1 timeout -k 10 600 python bench.py --dtype fp32h3 --steps 20 --warmup 3 --no-cpu-baseline --no-parity \
  > gpurun_out/${TAG}_bench_h3_p16.log 2>&1 || { tail -20 gpurun_out/${TAG}_bench_h3_p16.log; exit 5; }
tail -1 gpurun_out/${TAG}_bench_h3_p16.log | cut -c1-200
