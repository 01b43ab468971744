#!/bin/bash
# One profiling session for a profiles/<tag>_* snapshot: GPU suite, rocprofv3 kernel stats of
# the default bench, the bench line with per-launch table + CPU baseline, FETCH/WRITE PMC passes,
# and the BASELINE config 3-5 bench lines.  Stops at the first failure.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${PROF_TAG:-r1}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_pytest_gpu.log 2>&1 \
  || { tail -30 gpurun_out/${TAG}_pytest_gpu.log; exit 1; }
tail -1 gpurun_out/${TAG}_pytest_gpu.log
PROF_TAG=$TAG bash scripts/gpu_profile.sh || exit 2
timeout -k 10 600 python bench.py --steps 20 --warmup 3 --cpu-seconds 12 --launch-table gpurun_out/${TAG}_launch_table.json \
  > gpurun_out/${TAG}_bench.log 2>&1 || { tail -20 gpurun_out/${TAG}_bench.log; exit 3; }
tail -1 gpurun_out/${TAG}_bench.log | cut -c1-200
PROF_TAG=$TAG PMC_SETS="FETCH_SIZE;WRITE_SIZE" bash scripts/gpu_pmc.sh > /dev/null || exit 4
for c in 3 4 5; do
  timeout -k 10 600 python bench.py --config $c --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/${TAG}_bench_c$c.log 2>&1 \
    || { tail -20 gpurun_out/${TAG}_bench_c$c.log; exit 5; }
  tail -1 gpurun_out/${TAG}_bench_c$c.log | cut -c1-120
done
timeout -k 10 600 python bench.py --dtype fp32 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/${TAG}_bench_fp32.log 2>&1 \
  || { tail -20 gpurun_out/${TAG}_bench_fp32.log; exit 7; }
tail -1 gpurun_out/${TAG}_bench_fp32.log | cut -c1-160
timeout -k 10 600 python bench.py --dtype fp32x3 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/${TAG}_bench_fp32x3.log 2>&1 \
  || { tail -20 gpurun_out/${TAG}_bench_fp32x3.log; exit 8; }
tail -1 gpurun_out/${TAG}_bench_fp32x3.log | cut -c1-160
for mdl in rtdetr_r18 rtdetr_r50; do
  timeout -k 10 600 python bench.py --model $mdl --steps 20 --warmup 3 --cpu-seconds 12 > gpurun_out/${TAG}_bench_$mdl.log 2>&1 \
    || { tail -20 gpurun_out/${TAG}_bench_$mdl.log; exit 6; }
  tail -1 gpurun_out/${TAG}_bench_$mdl.log | cut -c1-120
done
KB="gemm --only 3x3" PROF_TAG=${TAG}_pconv bash scripts/gpu_pmc_sets.sh > gpurun_out/${TAG}_pmc_pconv.txt 2>&1 || { tail -20 gpurun_out/${TAG}_pmc_pconv.txt; exit 9; }
python3 scripts/pmc_summary.py gpurun_out/pmc_${TAG}_pconv --min-us 20 --json gpurun_out/${TAG}_counters_pconv.json > /dev/null
tail -6 gpurun_out/${TAG}_pmc_pconv.txt | cut -c1-200
