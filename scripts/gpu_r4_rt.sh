#!/bin/bash
# RT-DETR bench lines (pose-consistent weights) + their GPU tests
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
T="timeout -k 10"
for mdl in rtdetr_r50 rtdetr_r18; do
  $T 600 python -u bench.py --model $mdl --steps 20 --warmup 3 --cpu-seconds 12 > gpurun_out/rt_bench_$mdl.json 2> gpurun_out/rt_bench_$mdl.err \
    || { tail -20 gpurun_out/rt_bench_$mdl.err; exit 5; }
  python -c "
import json; d=json.loads(open('gpurun_out/rt_bench_$mdl.json').read().strip().splitlines()[-1])
print('$mdl', round(d['value']), d['ms_per_step'], d['solver_status_counts'], d.get('keypoints_vs_gt_px'), d.get('cpu_baseline',{}).get('value'))"
done
