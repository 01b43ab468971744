#!/bin/bash
# PMC pass (separate from tracing, per MI355X_MICROARCH.md): FETCH_SIZE and WRITE_SIZE in
# their own passes, kernel-trace only beside them.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${PROF_TAG:-r1}
mkdir -p gpurun_out/pmc_$TAG
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 900 rocprofv3 --kernel-trace --pmc $C --output-format csv -d gpurun_out/pmc_$TAG/$C -o bench -- \
    python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/pmc_$TAG/$C.log 2>&1 \
    || { echo "pmc $C failed"; tail -20 gpurun_out/pmc_$TAG/$C.log; exit 6; }
done
find gpurun_out/pmc_$TAG -name "*.csv" | head
