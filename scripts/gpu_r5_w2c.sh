#!/bin/bash
# bf16 encoder FFN with W2 chunk-packed: kernel tests, bf16 parity, kbench both forms, PMC (FETCH, L2 hit)
# of both, and a same-box bench A/B against ab_old/libspe.so (row-major W2).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc_w2c
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_kernels.py -k "fused_ffn" \
  > gpurun_out/w2c_t.log 2>&1 || { grep -E "^E |FAILED" gpurun_out/w2c_t.log | head; exit 1; }
tail -1 gpurun_out/w2c_t.log
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k "bf16" \
  > gpurun_out/w2c_p.log 2>&1 || { grep -E "^E |FAILED" gpurun_out/w2c_p.log | head; exit 2; }
tail -1 gpurun_out/w2c_p.log
timeout -k 10 120 python scripts/kbench.py ffn --iters 30 || exit 3
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_w2c/fetch -o k -- python3 scripts/kbench.py ffn --iters 3 > gpurun_out/pmc_w2c/fetch.log 2>&1 || exit 4
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d gpurun_out/pmc_w2c/hit -o k -- python3 scripts/kbench.py ffn --iters 3 > gpurun_out/pmc_w2c/hit.log 2>&1 || exit 5
find gpurun_out/pmc_w2c -name "*kernel_trace*" -delete
for v in old main old main; do
  if [ "$v" = main ]; then unset SPE_LIB_PATH; else export SPE_LIB_PATH=ab_old/libspe.so; fi
  timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-accuracy --no-parity > gpurun_out/w2c_ab_$v.log 2>&1 \
    || { tail -20 gpurun_out/w2c_ab_$v.log; exit 6; }
  echo "$v $(tail -1 gpurun_out/w2c_ab_$v.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['kernel_time_ms_per_step']; print(round(d['value'],1), {x: round(k[x],3) for x in ('ffn.enc','attn.enc','conv.1x1') if x in k})")"
done
