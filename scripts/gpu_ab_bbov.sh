#!/bin/bash
# Backbone/encoder overlap A/B: pipeline tests, then the bench with and without --overlap-backbone
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_pipeline.py tests/test_capi.py -x -q --timeout 120 --timeout-method thread -m gpu > gpurun_out/bbov_t.log 2>&1 || { tail -30 gpurun_out/bbov_t.log; exit 1; }
tail -1 gpurun_out/bbov_t.log
for v in 0 1 0 1; do
  A=""; [ "$v" = 1 ] && A="--overlap-backbone"
  timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-accuracy $A > gpurun_out/bbov_b$v.log 2>&1 || { tail -20 gpurun_out/bbov_b$v.log; exit 3; }
  echo "ovb=$v $(tail -1 gpurun_out/bbov_b$v.log | grep -o '"value": [0-9.]*') $(tail -1 gpurun_out/bbov_b$v.log | grep -o '"ms_per_step": [0-9.]*')"
done
for c in 3 5; do
  for v in 0 1; do
    A=""; [ "$v" = 1 ] && A="--overlap-backbone"
    timeout -k 10 300 python bench.py --config $c --steps 10 --warmup 2 --no-cpu-baseline --no-accuracy $A > gpurun_out/bbov_c${c}_$v.log 2>&1 || { tail -20 gpurun_out/bbov_c${c}_$v.log; exit 4; }
    echo "c$c ovb=$v $(tail -1 gpurun_out/bbov_c${c}_$v.log | grep -o '"value": [0-9.]*')"
  done
done
