#!/bin/bash
# Round 5, first GPU call: the touched GPU tests + the score-spread study (tests/test_gpu_precision.py),
# the bench line on the committed head fixture, the 2-rank shared-GPU rehearsal of the north-star
# shape, then a same-box A/B of the round-3 tree (ablate/r3, commit 84bc0b9, built in-tree) against
# this tree, alternating, two runs each.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
T="timeout -k 10"
$T 900 python -u -m pytest -x -v --timeout 900 --timeout-method thread tests/test_gpu_precision.py \
  > gpurun_out/a_precision.log 2>&1; rc=$?
tail -4 gpurun_out/a_precision.log; [ $rc = 0 ] || { grep -E "^E |FAILED|Error" gpurun_out/a_precision.log | head -20; }
$T 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_pipeline.py \
  tests/test_reference_front.py -k "cross_attention or decoder or pipeline or ceres or btail" > gpurun_out/a_tests.log 2>&1 \
  || { tail -30 gpurun_out/a_tests.log; exit 2; }
tail -2 gpurun_out/a_tests.log
$T 600 python bench.py > gpurun_out/a_bench.json 2> gpurun_out/a_bench.err || { tail -20 gpurun_out/a_bench.err; exit 3; }
SPE_DIST_BACKEND=gloo SPE_BENCH_SHARE_GPU=1 $T 600 python bench.py --gpus 2 --steps 5 --warmup 2 --no-parity \
  > gpurun_out/a_rehearsal2.json 2> gpurun_out/a_rehearsal2.err || { tail -20 gpurun_out/a_rehearsal2.err; exit 4; }
summ() {
  python -c "
import json,sys; d=json.loads(open('$1').read().strip().splitlines()[-1]); k=d['kernel_time_ms_per_step']
print('$2', round(d['value']), round(d['ms_per_step'],3), 'attn/launch', round(d['roofline']['avg_launch_ms'],4), {x: round(k[x],3) for x in ('attn.enc','ffn.enc','conv.1x1','conv.3x3','conv.neck','gemm.enc.qk','gemm.enc.o','attn.dec_cross') if x in k})"
}
for i in 1 2; do
  (cd ablate/r3 && $T 400 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-parity --no-accuracy) \
    > gpurun_out/a_ab_r3_$i.json 2> gpurun_out/a_ab_r3_$i.err || { tail -20 gpurun_out/a_ab_r3_$i.err; exit 5; }
  summ gpurun_out/a_ab_r3_$i.json r3
  $T 400 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-parity --no-accuracy \
    > gpurun_out/a_ab_head_$i.json 2> gpurun_out/a_ab_head_$i.err || { tail -20 gpurun_out/a_ab_head_$i.err; exit 6; }
  summ gpurun_out/a_ab_head_$i.json head
done
