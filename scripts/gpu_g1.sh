cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/g1_pytest.log 2>&1 || { tail -30 gpurun_out/g1_pytest.log; exit 1; }
tail -2 gpurun_out/g1_pytest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/g1_smoke.log 2>&1 || { tail -20 gpurun_out/g1_smoke.log; exit 2; }
timeout -k 10 400 python bench.py --steps 20 --warmup 3 --cpu-seconds 10 --launch-table gpurun_out/g1_launch_table.json > gpurun_out/g1_bench.log 2>&1 || { tail -20 gpurun_out/g1_bench.log; exit 3; }
tail -1 gpurun_out/g1_bench.log | cut -c1-300
timeout -k 10 120 python scripts/kbench.py gemm --only 3x3 --iters 20 > gpurun_out/g1_kb.log 2>&1 || exit 4
cat gpurun_out/g1_kb.log
