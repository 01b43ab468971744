#!/bin/bash
# Round 5, decoder cross-attention tail: the fused merge + value + out-projection + norm2 launch
# (decxproj) -- kernel tests, bf16 parity, one bench line with its launch table.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${PROF_TAG:-r5x}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_kernels.py \
  -k "cross_attention or decoder_out_projection or decoder_self or decoder_ffn or ffn or query_projection" > gpurun_out/${TAG}_tests.log 2>&1 \
  || { grep -E "^E |FAILED|Error" gpurun_out/${TAG}_tests.log | head -20; exit 4; }
tail -1 gpurun_out/${TAG}_tests.log
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py \
  -k "bf16" > gpurun_out/${TAG}_parity.log 2>&1 || { grep -E "^E |FAILED|Error" gpurun_out/${TAG}_parity.log | head -20; exit 5; }
tail -1 gpurun_out/${TAG}_parity.log
{ timeout -k 10 200 python scripts/kbench.py xattn --iters 50 && timeout -k 10 100 python scripts/kbench.py decsa --iters 50 && timeout -k 10 100 python scripts/kbench.py ffndec --iters 50; } > gpurun_out/${TAG}_kbench.log 2>&1 || { tail -20 gpurun_out/${TAG}_kbench.log; exit 7; }
cat gpurun_out/${TAG}_kbench.log
timeout -k 10 600 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-parity --launch-table gpurun_out/${TAG}_launch_table.json \
  > gpurun_out/${TAG}_bench.log 2>&1 || { tail -20 gpurun_out/${TAG}_bench.log; exit 6; }
tail -1 gpurun_out/${TAG}_bench.log | cut -c1-200
python3 scripts/launch_summary.py gpurun_out/${TAG}_launch_table.json --out gpurun_out/${TAG}_class_roofline.json | grep -E "dec|heads|total" || true
echo done
