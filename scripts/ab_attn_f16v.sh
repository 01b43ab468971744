cd "${GRAFT_REPO_ROOT:-/root/repo}"
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k "attention" -x -q --timeout 120 --timeout-method thread > gpurun_out/attn_t.log 2>&1 || { tail -30 gpurun_out/attn_t.log; exit 1; }
tail -1 gpurun_out/attn_t.log
for d in 0 3 0 3; do echo "attn dtype $d"; timeout -k 10 120 python scripts/kbench.py attn --iters 30 --attn-dtype $d || exit 2; done
for v in 0 1 0 1; do SPE_ATTN_F16V=$v timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/ab_b$v.log 2>&1 || { tail -5 gpurun_out/ab_b$v.log; exit 3; }; echo "f16v=$v $(tail -1 gpurun_out/ab_b$v.log | cut -c1-150)"; done
