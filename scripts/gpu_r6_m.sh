#!/bin/bash
# Round 6: config 4 / 5 spread studies with per-image deltas, then the c4 / c5 lines held to them.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${PROF_TAG:-r6m}
mkdir -p gpurun_out
timeout -k 10 1500 python -u -m pytest tests/test_gpu_precision.py -x -q -s --timeout 1400 --timeout-method thread \
  -k "config" > gpurun_out/${TAG}_precision_cfg.log 2>&1
rc=$?
grep -E "passed|failed" gpurun_out/${TAG}_precision_cfg.log | tail -2
for c in 4 5; do [ -f gpurun_out/precision_score_c$c.json ] && cp gpurun_out/precision_score_c$c.json profiles/r6_precision_score_c$c.json; done
[ $rc = 0 ] || { grep -E "^E " gpurun_out/${TAG}_precision_cfg.log | head -20; exit 1; }
PROF_TAG=$TAG bash scripts/gpu_r6_l.sh
