#!/bin/bash
# Same-box A/B of the pconv tile choice at the north star's per-GPU batch (config 3, 32 images) and at
# config 2: ab_old/libspe.so (previous build) against the tree's, interleaved; conv kernel tests first.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -k "conv" \
  > gpurun_out/abp_t.log 2>&1 || { grep -E "^E |FAILED" gpurun_out/abp_t.log | head; exit 1; }
tail -1 gpurun_out/abp_t.log
for c in 3 2; do
  for v in old main old main; do
    if [ "$v" = main ]; then unset SPE_LIB_PATH; else export SPE_LIB_PATH=ab_old/libspe.so; fi
    timeout -k 10 300 python bench.py --config $c --steps 30 --warmup 5 --no-cpu-baseline --no-accuracy --no-parity \
      > gpurun_out/abp_c${c}_$v.log 2>&1 || { tail -20 gpurun_out/abp_c${c}_$v.log; exit 3; }
    echo "c$c $v $(tail -1 gpurun_out/abp_c${c}_$v.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['kernel_time_ms_per_step']; print(round(d['value'],1), {x: round(k[x],3) for x in ('conv.3x3','conv.1x1') if x in k})")"
  done
done
