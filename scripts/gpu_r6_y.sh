#!/bin/bash
# Round 6: few-row fp32h3 GEMMs on 64-column three-stage tiles -- h3 GEMM kernel tests, fp32h3 goldens,
# the serialized fp32h3 launch table.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_parity.py -m gpu -x -q -k "h3" --timeout 300 --timeout-method thread > gpurun_out/r6y_tests.log 2>&1 \
  || { grep -E "^E |FAILED" gpurun_out/r6y_tests.log | head; exit 1; }
tail -1 gpurun_out/r6y_tests.log
timeout -k 10 400 python bench.py --dtype fp32h3 --no-parity --no-accuracy --no-cpu-baseline --no-host-input --no-overlap --steps 3 --warmup 2 \
  --launch-table gpurun_out/r6y_lt.json > gpurun_out/r6y_lt.log 2>&1 || { tail -5 gpurun_out/r6y_lt.log; exit 2; }
python3 - gpurun_out/r6y_lt.json <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
t = {}
for r in d:
    t.setdefault(r["kind"], []).append(r["ms"])
print({k: round(sum(v), 3) for k, v in t.items() if "dec" in k or "xsplit" in k})
print([round(r["ms"] * 1e3, 1) for r in d if r["kind"] == "gemm.dec"][:7])
PY
