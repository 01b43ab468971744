#!/bin/bash
# Round 6: fp32h3 fold kernel iteration -- goldens, then the serialized fp32h3 launch table.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
T=${TAG:-r6u}
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "fp32h3" --timeout 240 --timeout-method thread > gpurun_out/${T}_parity.log 2>&1 \
  || { grep -E "^E |FAILED" gpurun_out/${T}_parity.log | head; exit 1; }
tail -1 gpurun_out/${T}_parity.log
timeout -k 10 400 python bench.py --dtype fp32h3 --no-parity --no-accuracy --no-cpu-baseline --no-host-input --no-overlap --steps 3 --warmup 2 \
  --launch-table gpurun_out/${T}_lt_h3.json > gpurun_out/${T}_lt.log 2>&1 || { tail -5 gpurun_out/${T}_lt.log; exit 2; }
python3 - gpurun_out/${T}_lt_h3.json <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
tot = {}
for r in d:
    t = tot.setdefault(r["kind"], [0, 0]); t[0] += r["ms"]; t[1] += 1
print({k: round(v[0], 3) for k, v in tot.items() if "dec" in k or "xsplit" in k})
print([round(r["ms"] * 1e3, 1) for r in d if r["kind"] == "attn.dec_cross"])
PY
