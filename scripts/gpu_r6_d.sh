#!/bin/bash
# Round 6: split attention kernel tests + kbench (old x3 / split bf16 V / split fp16 V).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${PROF_TAG:-r6d}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread \
  -k "split_dma or x3_presplit or x3_close" > gpurun_out/${TAG}_tests.log 2>&1 \
  || { grep -E "^E |FAILED|Error" gpurun_out/${TAG}_tests.log | head -20; tail -5 gpurun_out/${TAG}_tests.log; exit 1; }
tail -1 gpurun_out/${TAG}_tests.log
for v in "--split-dma" "--split-dma --f16v"; do
  timeout -k 10 120 python3 scripts/kbench.py attn --attn-dtype 4 --presplit $v --iters 20 2>&1 | grep attn || exit 2
done
