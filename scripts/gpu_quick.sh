#!/bin/bash
# Affected-tests + short bench lines for configs 2-5 (one GPU session, stops at the first failure).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
if [ -n "$TESTS" ]; then
  timeout -k 10 800 python -u -m pytest $TESTS -x -v --timeout 200 --timeout-method thread -m gpu > gpurun_out/q_tests.log 2>&1 \
    || { tail -30 gpurun_out/q_tests.log; exit 1; }
  tail -2 gpurun_out/q_tests.log
fi
for c in ${CONFIGS:-2 3}; do
  timeout -k 10 400 python bench.py --config $c --steps ${STEPS:-10} --warmup 2 --no-cpu-baseline $BENCH_ARGS > gpurun_out/q_bench_c$c.log 2>&1 \
    || { tail -20 gpurun_out/q_bench_c$c.log; exit 2; }
  tail -1 gpurun_out/q_bench_c$c.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print($c, round(d['value'],1), d['ms_per_step'], d['solver_status_counts'], d.get('keypoints_vs_gt_px'), d.get('accuracy_vs_fp32'))"
done
