#!/bin/bash
# Round-5 snapshot, part 1: the GPU suite, rocprofv3 kernel stats of the default bench, the bench line
# (launch table, CPU baseline, parity mode fp32h3), FETCH/WRITE PMC passes of the dominant kernel.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${PROF_TAG:-r5}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest_gpu.log 2>&1 \
  || { grep -E "^E |FAILED" gpurun_out/${TAG}_pytest_gpu.log | head -20; tail -5 gpurun_out/${TAG}_pytest_gpu.log; exit 1; }
tail -1 gpurun_out/${TAG}_pytest_gpu.log
PROF_TAG=$TAG bash scripts/gpu_profile.sh || exit 2
timeout -k 10 600 python bench.py --steps 20 --warmup 3 --cpu-seconds 12 --launch-table gpurun_out/${TAG}_launch_table.json \
  > gpurun_out/${TAG}_bench.log 2>&1 || { tail -20 gpurun_out/${TAG}_bench.log; exit 3; }
tail -1 gpurun_out/${TAG}_bench.log | cut -c1-200
PROF_TAG=$TAG PMC_SETS="FETCH_SIZE;WRITE_SIZE" bash scripts/gpu_pmc.sh > /dev/null || exit 4
echo s1 done
