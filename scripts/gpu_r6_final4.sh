#!/bin/bash
# Round 6, the final tree (tag r6i): GPU suite + smoke, the default line, configs 3 and 4.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
T=${PROF_TAG:-r6i}
mkdir -p gpurun_out
PROF_TAG=$T bash scripts/gpu_r6_suite.sh || exit 1
timeout -k 10 900 python bench.py --steps 20 --warmup 3 --cpu-seconds 12 > gpurun_out/${T}_bench.log 2>&1 || { tail -20 gpurun_out/${T}_bench.log; exit 6; }
for c in 3 4; do
  timeout -k 10 600 python bench.py --config $c --steps 10 --warmup 2 --no-cpu-baseline --no-host-input > gpurun_out/${T}_bench_c$c.log 2>&1 || { tail -20 gpurun_out/${T}_bench_c$c.log; exit 7; }
done
for f in bench bench_c3 bench_c4; do
  tail -1 gpurun_out/${T}_$f.log | python3 -c "
import json,sys; r=json.loads(sys.stdin.read()); p=r['parity_mode']; a=p['accuracy_vs_fp32']
print('$f', round(r['value'],1), round(r['ms_per_step'],2), 'parity', round(p['value'],1), round(p['ms_per_step'],2), a['kpt_norm_max'], a['frac_score_delta_le_1e-4'], round(a['score_delta_max'],3), a['meets_1e-4_within_fp32_spread'])"
done
