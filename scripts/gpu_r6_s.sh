#!/bin/bash
# Round 6: the fp32h3 fold on config 5 -- its spread study with fp32h3's per-image deltas, then the
# c4 / c5 lines with the fold and without it (SPE_XATTN_H3=0).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_precision.py -x -q -s --timeout 800 --timeout-method thread \
  -k "config and 5" > gpurun_out/r6s2_precision_c5.log 2>&1
grep -E "passed|failed" gpurun_out/r6s2_precision_c5.log | tail -2
cp gpurun_out/precision_score_c5.json gpurun_out/r6s2_precision_score_c5.json 2>/dev/null
for x in 1 0; do
for c in 4 5; do
  SPE_XATTN_H3=$x timeout -k 10 900 python bench.py --config $c --steps 10 --warmup 2 --no-cpu-baseline --no-host-input > gpurun_out/r6s2_bench_c${c}_x$x.log 2>&1 \
    || { tail -20 gpurun_out/r6s2_bench_c${c}_x$x.log; exit 5; }
  tail -1 gpurun_out/r6s2_bench_c${c}_x$x.log | python3 -c "
import json,sys; r=json.loads(sys.stdin.read()); p=r['parity_mode']; a=p['accuracy_vs_fp32']
print('xattn_h3=$x', $c, round(r['value'],1), round(r['ms_per_step'],2), round(p['value'],1), round(p['ms_per_step'],2), {k:a.get(k) for k in ('kpt_norm_max','frac_score_delta_le_1e-4','score_delta_max','score_delta_max_well_conditioned','meets_1e-4_kpt','score_within_fp32_spread','meets_1e-4_within_fp32_spread','reliable_agreement','reliable_within_fp32_spread')})"
done
done
