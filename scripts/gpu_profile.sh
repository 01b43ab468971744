#!/bin/bash
# rocprofv3 kernel-trace + stats of a short bench run (no PMC counters in this pass).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${PROF_TAG:-r1}
mkdir -p gpurun_out/prof_$TAG
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o bench -- \
  python3 bench.py --steps ${BENCH_STEPS:-5} --warmup 2 --no-cpu-baseline --no-accuracy --no-parity --no-host-input ${BENCH_ARGS:-} > gpurun_out/prof_$TAG/bench_under_rocprof.log 2>&1 \
  || { echo "rocprof run failed"; tail -30 gpurun_out/prof_$TAG/bench_under_rocprof.log; exit 5; }
python3 scripts/kernel_stats_model.py gpurun_out/prof_$TAG --out gpurun_out/prof_$TAG/bench_kernel_stats_model.csv || exit 5
# keep the summaries only: the per-dispatch trace (weights fit included) would overflow the
# 64 MiB gpurun_out merge
find gpurun_out/prof_$TAG -name "*kernel_trace*" -delete
find gpurun_out/prof_$TAG -name "*stats*" | head
grep "^{\"metric\"" gpurun_out/prof_$TAG/bench_under_rocprof.log | cut -c1-400
