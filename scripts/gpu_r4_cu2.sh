#!/bin/bash
# pipeline tests (incl. the CU-masked streams), the CU-split sweep, the 2-rank gloo rehearsal
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_pipeline.py > gpurun_out/cu_tests.log 2>&1; rc=$?
tail -2 gpurun_out/cu_tests.log; [ $rc = 0 ] || { grep -E "^E |FAILED" gpurun_out/cu_tests.log | head; exit $rc; }
bash scripts/gpu_r4_cu.sh || exit $?
SPE_DIST_BACKEND=gloo SPE_BENCH_SHARE_GPU=1 timeout -k 10 600 python -u bench.py --gpus 2 --steps 5 --warmup 2 --no-cpu-baseline \
  > gpurun_out/r4_rehearsal_2rank.json 2> gpurun_out/r4_rehearsal_2rank.err; rc=$?
tail -3 gpurun_out/r4_rehearsal_2rank.err; cut -c1-700 gpurun_out/r4_rehearsal_2rank.json; exit $rc
