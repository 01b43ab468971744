#!/bin/bash
# Round 6 A/B: the four-stage one-work-group-per-CU h3p GEMM forms (SPE_H3P_S4=1) -- goldens, the serialized
# fp32h3 launch table per class, then the pipelined fp32h3 line, alternating.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
SPE_H3P_S4=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "fp32h3" --timeout 240 --timeout-method thread > gpurun_out/r6s4_parity.log 2>&1 \
  || { grep -E "^E |FAILED" gpurun_out/r6s4_parity.log | head; exit 1; }
tail -1 gpurun_out/r6s4_parity.log
for x in 0 1; do
  SPE_H3P_S4=$x timeout -k 10 400 python bench.py --dtype fp32h3 --no-parity --no-accuracy --no-cpu-baseline --no-host-input --no-overlap --steps 3 --warmup 2 \
    --launch-table gpurun_out/r6s4_lt_$x.json > gpurun_out/r6s4_lt_$x.log 2>&1 || { tail -5 gpurun_out/r6s4_lt_$x.log; exit 2; }
  python3 - gpurun_out/r6s4_lt_$x.json $x <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
t = {}
for r in d:
    t.setdefault(r["kind"], []).append(r["ms"])
print("X=" + sys.argv[2], round(sum(sum(v) for v in t.values()), 3), {k: round(sum(v), 3) for k, v in t.items() if sum(v) > 0.3})
PY
done
for x in 0 1 0 1; do
  SPE_H3P_S4=$x timeout -k 10 400 python bench.py --dtype fp32h3 --no-parity --no-accuracy --no-cpu-baseline --no-host-input --steps 10 --warmup 3 \
    > gpurun_out/r6s4_bench_$x.json 2> gpurun_out/r6s4_bench_$x.err || { tail -5 gpurun_out/r6s4_bench_$x.err; exit 3; }
  python3 -c "import json,sys; r=json.loads(open('gpurun_out/r6s4_bench_$x.json').read().strip().splitlines()[-1]); print('X=$x', round(r['value'],1), round(r['ms_per_step'],2))"
done
