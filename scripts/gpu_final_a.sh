#!/bin/bash
# round-end snapshot, part A: GPU suite + smoke, rocprofv3 kernel stats of the default bench,
# the default bench line (launch table + CPU baseline), FETCH/WRITE per class
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${PROF_TAG:-r4f}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest_gpu.log 2>&1 \
  || { tail -30 gpurun_out/${TAG}_pytest_gpu.log; exit 1; }
tail -1 gpurun_out/${TAG}_pytest_gpu.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || { tail -20 gpurun_out/${TAG}_smoke.log; exit 2; }
tail -1 gpurun_out/${TAG}_smoke.log
timeout -k 10 600 python bench.py --steps 20 --warmup 3 --cpu-seconds 12 --launch-table gpurun_out/${TAG}_launch_table.json \
  > gpurun_out/${TAG}_bench.log 2>&1 || { tail -20 gpurun_out/${TAG}_bench.log; exit 3; }
tail -1 gpurun_out/${TAG}_bench.log | cut -c1-300
PROF_TAG=$TAG bash scripts/gpu_profile.sh > gpurun_out/${TAG}_profile.txt 2>&1 || { tail -20 gpurun_out/${TAG}_profile.txt; exit 4; }
bash scripts/gpu_pmc_kinds.sh > gpurun_out/${TAG}_pmc_kinds.log 2>&1 || { tail -20 gpurun_out/${TAG}_pmc_kinds.log; exit 5; }
echo done
