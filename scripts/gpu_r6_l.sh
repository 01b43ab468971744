#!/bin/bash
# Round 6: c4 / c5 bench lines with their fp32h3 parity_mode held to the committed per-config spread.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${PROF_TAG:-r6l}
mkdir -p gpurun_out
for c in 4 5; do
  timeout -k 10 900 python bench.py --config $c --steps 10 --warmup 2 --no-cpu-baseline --no-host-input > gpurun_out/${TAG}_bench_c$c.log 2>&1 \
    || { tail -20 gpurun_out/${TAG}_bench_c$c.log; exit 5; }
  tail -1 gpurun_out/${TAG}_bench_c$c.log | python3 -c "
import json,sys; r=json.loads(sys.stdin.read()); p=r['parity_mode']; a=p['accuracy_vs_fp32']
print($c, r['value'], r['ms_per_step'], p['value'], p['ms_per_step'], {k:a.get(k) for k in ('kpt_norm_max','frac_score_delta_le_1e-4','score_delta_max','meets_1e-4_kpt','score_within_fp32_spread','meets_1e-4_within_fp32_spread','reliable_agreement','reliable_within_fp32_spread')})"
done
