#!/bin/bash
# Round 6: the fp32h3 decoder cross-attention against the memory (xattn_h3.hip) -- goldens, then
# the default line (bf16 value + fp32h3 parity_mode with accuracy_vs_fp32), then the same line with
# SPE_XATTN_H3=0 (the projected K / V^T path) for the A/B.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "fp32h3" --timeout 240 --timeout-method thread > gpurun_out/r6q_parity.log 2>&1 \
  || { grep -E "^E |FAILED|Error|assert" gpurun_out/r6q_parity.log | head -20; tail -5 gpurun_out/r6q_parity.log; exit 1; }
tail -1 gpurun_out/r6q_parity.log
timeout -k 10 400 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-host-input > gpurun_out/r6q_bench.json 2> gpurun_out/r6q_bench.err || { tail -5 gpurun_out/r6q_bench.err; exit 2; }
python3 - gpurun_out/r6q_bench.json <<'PY'
import json, sys
r = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
p = r.get("parity_mode", {})
print("bf16", round(r["value"], 1), round(r["ms_per_step"], 2))
print("fp32h3", {k: p.get(k) for k in ("value", "ms_per_step")}, json.dumps(p.get("accuracy_vs_fp32"))[:600])
PY
SPE_XATTN_H3=0 timeout -k 10 400 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-host-input > gpurun_out/r6q_bench_old.json 2> gpurun_out/r6q_bench_old.err || { tail -5 gpurun_out/r6q_bench_old.err; exit 3; }
python3 - gpurun_out/r6q_bench_old.json <<'PY'
import json, sys
r = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
p = r.get("parity_mode", {})
print("old fp32h3", {k: p.get(k) for k in ("value", "ms_per_step")}, json.dumps(p.get("accuracy_vs_fp32"))[:600])
PY
