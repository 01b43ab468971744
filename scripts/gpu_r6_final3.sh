#!/bin/bash
# Round 6, last tree (tag r6g): the whole GPU suite, smoke, and the default bench line.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
T=${PROF_TAG:-r6g}
mkdir -p gpurun_out
PROF_TAG=$T bash scripts/gpu_r6_suite.sh || exit 1
timeout -k 10 900 python bench.py --steps 20 --warmup 3 --cpu-seconds 12 --launch-table gpurun_out/${T}_launch_table.json \
  > gpurun_out/${T}_bench.log 2>&1 || { tail -20 gpurun_out/${T}_bench.log; exit 6; }
tail -1 gpurun_out/${T}_bench.log | python3 -c "
import json,sys; r=json.loads(sys.stdin.read()); p=r['parity_mode']; a=p['accuracy_vs_fp32']
print('bf16', round(r['value'],1), round(r['ms_per_step'],2), 'host', round(r['value_host_input'],1), 'parity', round(p['value'],1), round(p['ms_per_step'],2), a['kpt_norm_max'], a['meets_1e-4_within_fp32_spread'])"
