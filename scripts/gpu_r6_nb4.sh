#!/bin/bash
# Round 6 A/B: four A register sets (three row tiles in flight per wave) for the q/k projection's
# residual streaming GEMM (SPE_SG_NB4=1) -- bf16 goldens, serialized launch tables, the default line.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
SPE_SG_NB4=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "bf16" --timeout 240 --timeout-method thread > gpurun_out/r6nb_parity.log 2>&1 \
  || { grep -E "^E |FAILED" gpurun_out/r6nb_parity.log | head; exit 1; }
tail -1 gpurun_out/r6nb_parity.log
for x in 0 1; do
  SPE_SG_NB4=$x timeout -k 10 400 python bench.py --no-parity --no-accuracy --no-cpu-baseline --no-host-input --no-overlap --steps 3 --warmup 2 \
    --launch-table gpurun_out/r6nb_lt_$x.json > gpurun_out/r6nb_lt_$x.log 2>&1 || { tail -5 gpurun_out/r6nb_lt_$x.log; exit 2; }
  python3 - gpurun_out/r6nb_lt_$x.json $x <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
t = {}
for r in d:
    t.setdefault(r["kind"], []).append(r["ms"])
print("NB4=" + sys.argv[2], {k: round(sum(v), 3) for k, v in t.items() if k.startswith("gemm.enc")})
PY
done
for x in 0 1 0 1; do
  SPE_SG_NB4=$x timeout -k 10 400 python bench.py --no-parity --no-accuracy --no-cpu-baseline --no-host-input --steps 20 --warmup 3 \
    > gpurun_out/r6nb_bench_$x.json 2> gpurun_out/r6nb_bench_$x.err || { tail -5 gpurun_out/r6nb_bench_$x.err; exit 3; }
  python3 -c "import json; r=json.loads(open('gpurun_out/r6nb_bench_$x.json').read().strip().splitlines()[-1]); print('NB4=$x', round(r['value'],1), round(r['ms_per_step'],3))"
done
