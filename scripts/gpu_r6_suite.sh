#!/bin/bash
# Round 6: the whole GPU suite and smoke().
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${PROF_TAG:-r6s}
mkdir -p gpurun_out
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -q --timeout 1000 --timeout-method thread > gpurun_out/${TAG}_pytest_gpu.log 2>&1 \
  || { grep -E "^E |FAILED|Error" gpurun_out/${TAG}_pytest_gpu.log | head -20; tail -5 gpurun_out/${TAG}_pytest_gpu.log; exit 1; }
tail -1 gpurun_out/${TAG}_pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || { tail -10 gpurun_out/${TAG}_smoke.log; exit 2; }
tail -1 gpurun_out/${TAG}_smoke.log
