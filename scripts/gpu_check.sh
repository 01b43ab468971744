#!/bin/bash
# One GPU session: parity tests, smoke, short bench.  Stops at the first crash/timeout
# (exit codes other than 0/1 from pytest, any failure after that).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -q -rf --timeout=600 > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -30 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping: pytest crashed or timed out"; exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke failed"; tail -30 gpurun_out/smoke.log; exit 3; }
tail -3 gpurun_out/smoke.log
timeout -k 10 900 python bench.py --steps ${BENCH_STEPS:-5} --warmup 2 --cpu-seconds 10 > gpurun_out/bench.log 2>&1 || { echo "bench failed"; tail -30 gpurun_out/bench.log; exit 4; }
tail -1 gpurun_out/bench.log
