#!/bin/bash
# Round 6: the fp32h3 stem (7x7, 4 channels, per-lane tap decode) on three LDS stages instead of two
# (variant library ab_pl3/libspe.so) -- per-shape timing, h3 GEMM tests, bit-for-bit fp32h3 outputs.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${PROF_TAG:-r6pl}
mkdir -p gpurun_out
for v in main pl3 main pl3; do
  if [ "$v" = main ]; then unset SPE_LIB_PATH; else export SPE_LIB_PATH=ab_$v/libspe.so; fi
  echo "$v $(timeout -k 10 120 python scripts/x6_bench.py --only stem --dtypes fp32h3 --iters 20 | tr '\n' ' ')" || exit 1
done
unset SPE_LIB_PATH
timeout -k 10 600 python -u scripts/lab/bitwise_forward.py dump gpurun_out/${TAG}_main.npz > gpurun_out/${TAG}_dump_main.log 2>&1 || exit 2
export SPE_LIB_PATH=ab_pl3/libspe.so
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q -k "gemm_h3_close" --timeout 200 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 \
  || { grep -E "^E |FAILED" gpurun_out/${TAG}_tests.log | head; exit 3; }
timeout -k 10 600 python -u scripts/lab/bitwise_forward.py dump gpurun_out/${TAG}_pl3.npz > gpurun_out/${TAG}_dump_pl3.log 2>&1 || exit 4
echo "pl3 $(tail -1 gpurun_out/${TAG}_tests.log) $(python scripts/lab/bitwise_forward.py compare gpurun_out/${TAG}_main.npz gpurun_out/${TAG}_pl3.npz | tail -1)"
rm -f gpurun_out/${TAG}_*.npz
echo done
