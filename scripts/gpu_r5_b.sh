#!/bin/bash
# Round 5: same-box A/B of the round-3 tree (ablate/r3 = 84bc0b9, built in-tree) against this
# tree, alternating, two runs each, then the score-spread study again.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
T="timeout -k 10"
summ() {
  python -c "
import json,sys; d=json.loads(open('$1').read().strip().splitlines()[-1]); k=d['kernel_time_ms_per_step']
print('$2', round(d['value']), round(d['ms_per_step'],3), 'attn/launch', round(d['roofline']['avg_launch_ms'],4), {x: round(k[x],3) for x in ('attn.enc','ffn.enc','conv.1x1','conv.3x3','conv.neck','gemm.enc.qk','gemm.enc.o','attn.dec_cross') if x in k})"
}
for i in 1 2; do
  (cd ablate/r3 && $T 400 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-accuracy) \
    > gpurun_out/b_ab_r3_$i.json 2> gpurun_out/b_ab_r3_$i.err || { tail -20 gpurun_out/b_ab_r3_$i.err; exit 5; }
  summ gpurun_out/b_ab_r3_$i.json r3
  $T 400 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-parity --no-accuracy \
    > gpurun_out/b_ab_head_$i.json 2> gpurun_out/b_ab_head_$i.err || { tail -20 gpurun_out/b_ab_head_$i.err; exit 6; }
  summ gpurun_out/b_ab_head_$i.json head
done
$T 900 python -u -m pytest -x -v --timeout 900 --timeout-method thread tests/test_gpu_precision.py \
  > gpurun_out/b_precision.log 2>&1; rc=$?
tail -3 gpurun_out/b_precision.log
exit $rc
