#!/bin/bash
# Round 5: the fp32h3 kernel (scaled two-way fp16 split) -- kernel tests against fp64, the model
# against the reference goldens in every parity mode, the x6 kernels after the amax epilogue change,
# the bench's parity line in fp32h3; then the r3-vs-HEAD A/B.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
T="timeout -k 10"
$T 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "h3 or x6 or x3_close" \
  > gpurun_out/c_kernels.log 2>&1 || { grep -E "^E |FAILED|Error" gpurun_out/c_kernels.log | head -30; tail -5 gpurun_out/c_kernels.log; exit 2; }
tail -1 gpurun_out/c_kernels.log
$T 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "forward_fp32" \
  > gpurun_out/c_parity.log 2>&1 || { grep -E "^E |FAILED|Error" gpurun_out/c_parity.log | head -30; exit 3; }
tail -1 gpurun_out/c_parity.log
$T 600 python bench.py --parity-dtype fp32h3 --no-cpu-baseline > gpurun_out/c_bench_h3.json 2> gpurun_out/c_bench_h3.err \
  || { tail -20 gpurun_out/c_bench_h3.err; exit 4; }
python -c "
import json; d=json.loads(open('gpurun_out/c_bench_h3.json').read().strip().splitlines()[-1]); p=d['parity_mode']; a=p['accuracy_vs_fp32']
print('bf16', round(d['value']), 'h3', round(p['value']), round(p['ms_per_step'],2), 'kpt', a['kpt_norm_max'], 'score<=1e-4', a['frac_score_delta_le_1e-4'])
print({k: round(v,3) for k,v in p['kernel_time_ms_per_step'].items()})"
summ() {
  python -c "
import json,sys; d=json.loads(open('$1').read().strip().splitlines()[-1]); k=d['kernel_time_ms_per_step']
print('$2', round(d['value']), round(d['ms_per_step'],3), 'attn/launch', round(d['roofline']['avg_launch_ms'],4), {x: round(k[x],3) for x in ('attn.enc','ffn.enc','conv.1x1','conv.3x3','conv.neck','gemm.enc.qk','gemm.enc.o','attn.dec_cross') if x in k})"
}
for i in 1 2; do
  (cd ablate/r3 && $T 400 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-accuracy) \
    > gpurun_out/c_ab_r3_$i.json 2> gpurun_out/c_ab_r3_$i.err || { tail -20 gpurun_out/c_ab_r3_$i.err; exit 5; }
  summ gpurun_out/c_ab_r3_$i.json r3
  $T 400 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-parity --no-accuracy \
    > gpurun_out/c_ab_head_$i.json 2> gpurun_out/c_ab_head_$i.err || { tail -20 gpurun_out/c_ab_head_$i.err; exit 6; }
  summ gpurun_out/c_ab_head_$i.json head
done
