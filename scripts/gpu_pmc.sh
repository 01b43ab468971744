#!/bin/bash
# PMC passes (separate from tracing, per MI355X_MICROARCH.md): every counter set in its own
# rocprofv3 run with --kernel-trace only beside it.  FETCH_SIZE and WRITE_SIZE never share a pass.
# Usage: PROF_TAG=r1e PMC_SETS="FETCH_SIZE;WRITE_SIZE;SQ_WAVES SQ_WAVE_CYCLES ..." [BENCH_ARGS="--dtype fp32h3 --no-overlap"] bash scripts/gpu_pmc.sh
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${PROF_TAG:-r1}
SETS=${PMC_SETS:-"FETCH_SIZE;WRITE_SIZE"}
mkdir -p gpurun_out/pmc_$TAG
i=0
IFS=';' read -ra ARR <<< "$SETS"
for C in "${ARR[@]}"; do
  i=$((i+1))
  timeout -k 10 600 rocprofv3 --kernel-trace --pmc $C --output-format csv -d gpurun_out/pmc_$TAG/set$i -o bench -- \
    python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-accuracy --no-parity --weights label-diverse ${BENCH_ARGS:-} > gpurun_out/pmc_$TAG/set$i.log 2>&1 \
    || { echo "pmc set $i ($C) failed"; tail -20 gpurun_out/pmc_$TAG/set$i.log; exit 6; }
  echo "$C" > gpurun_out/pmc_$TAG/set$i/counters.txt
  find gpurun_out/pmc_$TAG/set$i -name "*kernel_trace*" -delete
done
find gpurun_out/pmc_$TAG -name "*counter_collection*" | head
