#!/bin/bash
# Round 6: u8 crops / host-input tests and a default bench line with its host_input object.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${PROF_TAG:-r6h}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_pipeline.py -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/${TAG}_tests.log 2>&1 \
  || { grep -E "^E |FAILED|Error" gpurun_out/${TAG}_tests.log | head -20; tail -5 gpurun_out/${TAG}_tests.log; exit 1; }
tail -1 gpurun_out/${TAG}_tests.log
timeout -k 10 600 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-parity > gpurun_out/${TAG}_bench.log 2>&1 \
  || { tail -20 gpurun_out/${TAG}_bench.log; exit 2; }
tail -1 gpurun_out/${TAG}_bench.log | python3 -c "import json,sys; r=json.loads(sys.stdin.read()); print(r['value'], r['ms_per_step'], json.dumps(r.get('host_input')))"
