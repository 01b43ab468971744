cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k "patch_conv3x3 or large_tile_conv or conv_nhwc" -x -q --timeout 120 --timeout-method thread -m gpu > gpurun_out/pc_tests.log 2>&1 || { tail -30 gpurun_out/pc_tests.log; exit 1; }
tail -3 gpurun_out/pc_tests.log
timeout -k 10 120 python scripts/kbench.py gemm --only 3x3 --iters 20 > gpurun_out/pc_kb1.log 2>&1 || { tail -20 gpurun_out/pc_kb1.log; exit 2; }
SPE_PCONV=0 timeout -k 10 120 python scripts/kbench.py gemm --only 3x3 --iters 20 > gpurun_out/pc_kb0.log 2>&1 || { tail -20 gpurun_out/pc_kb0.log; exit 3; }
echo new; cat gpurun_out/pc_kb1.log; echo old; cat gpurun_out/pc_kb0.log
