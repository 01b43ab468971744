# FFN A/B: parity of the default variant, then kbench timings of "SCHED TAIL" pairs
# (SPE_FFN_SCHED / SPE_FFN_TAIL) given in VARIANTS as sched_tail words
cd "${GRAFT_REPO_ROOT:-/root/repo}"
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k "fused_ffn" -x -q --timeout 120 --timeout-method thread > gpurun_out/ffn_t.log 2>&1 || { tail -20 gpurun_out/ffn_t.log; exit 1; }
tail -1 gpurun_out/ffn_t.log
for v in ${VARIANTS:-0_0 6_0 6_1}; do
  echo "sched_tail=$v"; SPE_FFN_SCHED=${v%_*} SPE_FFN_TAIL=${v#*_} timeout -k 10 120 python scripts/kbench.py ffn --iters 50 || exit 2
done
