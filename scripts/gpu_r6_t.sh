#!/bin/bash
# Round 6: after gating the fp32h3 fold to Q <= 12 -- the config 4 / 5 spread tests, the fp32h3
# goldens and the config-2 precision study.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "fp32h3" --timeout 240 --timeout-method thread > gpurun_out/r6t_parity.log 2>&1 \
  || { grep -E "^E |FAILED" gpurun_out/r6t_parity.log | head; exit 1; }
tail -1 gpurun_out/r6t_parity.log
timeout -k 10 1100 python -u -m pytest tests/test_gpu_precision.py -m gpu -x -q --timeout 1000 --timeout-method thread > gpurun_out/r6t_precision.log 2>&1 \
  || { grep -E "^E |FAILED" gpurun_out/r6t_precision.log | head -20; exit 2; }
tail -1 gpurun_out/r6t_precision.log
for c in 4 5; do cp gpurun_out/precision_score_c$c.json gpurun_out/r6t_precision_score_c$c.json; done
