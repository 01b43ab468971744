#!/bin/bash
# Round-5 snapshot, part 2: BASELINE configs 3-5, the fp32 / fp32x3 / fp32x6 / fp32h3 lines, RT-DETR,
# per-class HBM bytes of a serialised bf16 step, the 2-rank shared-GPU rehearsal of the N > 1 line.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${PROF_TAG:-r5}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_parity.py \
  -k "h3 or forward_fp32" > gpurun_out/${TAG}_s2_tests.log 2>&1 || { grep -E "^E |FAILED" gpurun_out/${TAG}_s2_tests.log | head; exit 4; }
tail -1 gpurun_out/${TAG}_s2_tests.log
for c in 3 4 5; do
  # (config 3 = the north star's per-GPU shape at N = 8: 32 images, P3P-RANSAC + LM; its parity line is
  # the contract mode at that shape)
  np=--no-parity; [ $c = 3 ] && np=
  timeout -k 10 600 python bench.py --config $c --steps 10 --warmup 2 --no-cpu-baseline $np > gpurun_out/${TAG}_bench_c$c.log 2>&1 \
    || { tail -20 gpurun_out/${TAG}_bench_c$c.log; exit 5; }
  tail -1 gpurun_out/${TAG}_bench_c$c.log | cut -c1-120
done
for dt in fp32 fp32x3 fp32x6 fp32h3; do
  timeout -k 10 600 python bench.py --dtype $dt --steps 10 --warmup 2 --no-cpu-baseline --no-parity > gpurun_out/${TAG}_bench_$dt.log 2>&1 \
    || { tail -20 gpurun_out/${TAG}_bench_$dt.log; exit 7; }
  tail -1 gpurun_out/${TAG}_bench_$dt.log | cut -c1-160
done
for mdl in rtdetr_r18 rtdetr_r50; do
  timeout -k 10 600 python bench.py --model $mdl --steps 20 --warmup 3 --cpu-seconds 12 > gpurun_out/${TAG}_bench_$mdl.log 2>&1 \
    || { tail -20 gpurun_out/${TAG}_bench_$mdl.log; exit 6; }
  tail -1 gpurun_out/${TAG}_bench_$mdl.log | cut -c1-120
done
bash scripts/gpu_pmc_kinds.sh > gpurun_out/${TAG}_pmc_kinds.txt 2>&1 || { tail -20 gpurun_out/${TAG}_pmc_kinds.txt; exit 8; }
SPE_DIST_BACKEND=gloo SPE_BENCH_SHARE_GPU=1 timeout -k 10 600 python bench.py --gpus 2 --steps 5 --warmup 2 --no-parity \
  > gpurun_out/${TAG}_rehearsal2.json 2> gpurun_out/${TAG}_rehearsal2.err || { tail -20 gpurun_out/${TAG}_rehearsal2.err; exit 9; }
tail -1 gpurun_out/${TAG}_rehearsal2.json | cut -c1-200
echo s2 done
