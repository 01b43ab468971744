#!/bin/bash
# Round 5, decoder cross-attention tail: the fused merge + value + out-projection + norm2 launch
# (decxproj) -- kernel tests, bf16 parity, one bench line with its launch table.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${PROF_TAG:-r5x}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_kernels.py \
  -k "cross_attention or decoder" > gpurun_out/${TAG}_tests.log 2>&1 \
  || { grep -E "^E |FAILED|Error" gpurun_out/${TAG}_tests.log | head -20; exit 4; }
tail -1 gpurun_out/${TAG}_tests.log
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py \
  -k "bf16" > gpurun_out/${TAG}_parity.log 2>&1 || { grep -E "^E |FAILED|Error" gpurun_out/${TAG}_parity.log | head -20; exit 5; }
tail -1 gpurun_out/${TAG}_parity.log
{ timeout -k 10 200 python scripts/kbench.py xattn --iters 50; } > gpurun_out/${TAG}_kbench.log 2>&1 || { tail -20 gpurun_out/${TAG}_kbench.log; exit 7; }
cat gpurun_out/${TAG}_kbench.log
timeout -k 10 600 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-parity --launch-table gpurun_out/${TAG}_launch_table.json \
  > gpurun_out/${TAG}_bench.log 2>&1 || { tail -20 gpurun_out/${TAG}_bench.log; exit 6; }
tail -1 gpurun_out/${TAG}_bench.log | cut -c1-200
python3 scripts/launch_summary.py gpurun_out/${TAG}_launch_table.json --out gpurun_out/${TAG}_class_roofline.json | grep -E "dec|heads|total" || true

if [ -f ab_old/libspe.so ]; then
  for v in old main old main; do
    if [ "$v" = main ]; then unset SPE_LIB_PATH; else export SPE_LIB_PATH=ab_old/libspe.so; fi
    timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-accuracy --no-parity > gpurun_out/${TAG}_ab_$v.log 2>&1 \
      || { tail -20 gpurun_out/${TAG}_ab_$v.log; exit 8; }
    echo "$v $(tail -1 gpurun_out/${TAG}_ab_$v.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['kernel_time_ms_per_step']; print(round(d['value'],1), {x: round(k[x],3) for x in ('attn.dec_cross','dec.xproj','ffn.enc','conv.3x3') if x in k})")"
  done
fi
echo done
