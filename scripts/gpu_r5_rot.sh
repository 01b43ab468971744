#!/bin/bash
# Experiment: the encoder FFN's per-workgroup start-chunk rotation (SPE_FFN_ROT): tests, kbench, L2 misses.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc_rot
SPE_FFN_ROT=7 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_kernels.py -k "fused_ffn" \
  > gpurun_out/rot_t.log 2>&1 || { grep -E "^E |FAILED" gpurun_out/rot_t.log | head; exit 1; }
tail -1 gpurun_out/rot_t.log
for v in 0 7 0 7; do echo "== rot $v"; SPE_FFN_ROT=$v timeout -k 10 120 python scripts/kbench.py ffn --iters 30 || exit 2; done
SPE_FFN_ROT=7 timeout -s KILL 120 rocprofv3 --kernel-trace --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d gpurun_out/pmc_rot/hit -o k -- python3 scripts/kbench.py ffn --iters 3 > gpurun_out/pmc_rot/hit.log 2>&1 || exit 3
find gpurun_out/pmc_rot -name "*kernel_trace*" -delete
for v in 0 7 0 7; do
  SPE_FFN_ROT=$v timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-accuracy --no-parity > gpurun_out/rot_b_$v.log 2>&1 || exit 4
  echo "rot $v $(tail -1 gpurun_out/rot_b_$v.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['kernel_time_ms_per_step']; print(round(d['value'],1), {x: round(k[x],3) for x in ('ffn.enc','attn.enc') if x in k})")"
done
