#!/bin/bash
# A/B one environment knob over the default bench: AB_VAR=name AB_VALUES="a b c" [BENCH_ARGS=...]
# prints img/s and the per-class kernel ms of each value (one bench process per value).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for v in $AB_VALUES; do
  env $AB_VAR=$v timeout -k 10 240 python bench.py --steps ${STEPS:-20} --warmup 3 --no-cpu-baseline $BENCH_ARGS > gpurun_out/ab_$v.log 2>&1 || { echo "bench $AB_VAR=$v failed"; tail -5 gpurun_out/ab_$v.log; exit 1; }
  tail -1 gpurun_out/ab_$v.log | python3 -c "
import json,sys
d=json.loads(sys.stdin.read())
k=d.get('kernel_time_ms_per_step',{})
print('$AB_VAR=$v', round(d['value'],1), 'img/s', round(d['ms_per_step'],3), 'ms/step |', ' '.join(f'{a}={b:.3f}' for a,b in sorted(k.items(), key=lambda x:-x[1])[:12]))"
done
