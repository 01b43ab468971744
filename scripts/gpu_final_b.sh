#!/bin/bash
# round-end snapshot, part B: BASELINE configs 3-5, the fp32 / fp32x3 modes, the RT-DETR lines
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${PROF_TAG:-r4f}
mkdir -p gpurun_out
for c in 3 4 5; do
  timeout -k 10 600 python bench.py --config $c --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/${TAG}_bench_c$c.log 2>&1 \
    || { tail -20 gpurun_out/${TAG}_bench_c$c.log; exit 5; }
  tail -1 gpurun_out/${TAG}_bench_c$c.log | cut -c1-160
done
for dt in fp32 fp32x3 fp32x6; do
  timeout -k 10 600 python bench.py --dtype $dt --steps 10 --warmup 2 --no-cpu-baseline --no-parity > gpurun_out/${TAG}_bench_$dt.log 2>&1 \
    || { tail -20 gpurun_out/${TAG}_bench_$dt.log; exit 7; }
  tail -1 gpurun_out/${TAG}_bench_$dt.log | cut -c1-160
done
for mdl in rtdetr_r18 rtdetr_r50; do
  timeout -k 10 600 python bench.py --model $mdl --steps 20 --warmup 3 --cpu-seconds 12 > gpurun_out/${TAG}_bench_$mdl.log 2>&1 \
    || { tail -20 gpurun_out/${TAG}_bench_$mdl.log; exit 6; }
  tail -1 gpurun_out/${TAG}_bench_$mdl.log | cut -c1-160
done
