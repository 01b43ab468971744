#!/bin/bash
# round-4 check: x6 tests (incl. the 128x64 DMA tile), x6 microbench, default bench, RT-DETR
# lines with the fitted last-layer point head.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
T="timeout -k 10"
bash scripts/gpu_r4_f.sh || exit $?
for mdl in rtdetr_r50 rtdetr_r18; do
  $T 600 python -u bench.py --model $mdl --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/g_bench_$mdl.json 2> gpurun_out/g_bench_$mdl.err \
    || { tail -20 gpurun_out/g_bench_$mdl.err; exit 5; }
  python -c "
import json; d=json.loads(open('gpurun_out/g_bench_$mdl.json').read().strip().splitlines()[-1])
print('$mdl', round(d['value']), d['ms_per_step'], d['solver_status_counts'], d.get('keypoints_vs_gt_px'))"
done
