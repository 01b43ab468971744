# gemm2 pinned-schedule A/B: GEMM/conv parity tests, then bench + per-launch tables with SPE_GEMM2_PIN=0/1
cd "${GRAFT_REPO_ROOT:-/root/repo}"
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pin_t.log 2>&1 || { tail -30 gpurun_out/pin_t.log; exit 1; }
tail -1 gpurun_out/pin_t.log
for v in 0 1 0 1; do
  env "SPE_GEMM2_${KNOB:-PIN}=$v" timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --launch-table gpurun_out/lt_${KNOB:-PIN}$v.json > gpurun_out/ab_${KNOB:-PIN}$v.log 2>&1 || { tail -5 gpurun_out/ab_${KNOB:-PIN}$v.log; exit 3; }
  echo "${KNOB:-PIN}=$v $(tail -1 gpurun_out/ab_${KNOB:-PIN}$v.log | cut -c90-150)"
done
