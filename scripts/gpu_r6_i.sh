#!/bin/bash
# Round 6: host-input A/B: the host_input object timed after and before the device-resident line.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${PROF_TAG:-r6i}
mkdir -p gpurun_out
for o in "" "--host-input-first"; do
  timeout -k 10 600 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-parity $o > gpurun_out/${TAG}_bench$o.log 2>&1 \
    || { tail -20 gpurun_out/${TAG}_bench$o.log; exit 2; }
  tail -1 gpurun_out/${TAG}_bench$o.log | python3 -c "
import json,sys; r=json.loads(sys.stdin.read()); h=r['host_input']
print(r['value'], r['ms_per_step'], h['value'], h['ms_per_step'], h['dominant_avg_launch_ms'], r['roofline']['avg_launch_ms'])
a=r['kernel_time_ms_per_step']; b=h['kernel_time_ms_per_step']
print({k:(round(a[k],3),round(b.get(k,0),3)) for k in a})"
done
