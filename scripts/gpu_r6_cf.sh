#!/bin/bash
# Round 6: the under-filled long-K implicit-GEMM 3x3 (layer 4, 340 tiles of 128 x 128 on 512 slots) on
# persistent forms with smaller tiles / deeper pipelines (variant libraries ab_cf<v>/libspe.so) --
# per-shape timing, h3 GEMM tests and bit-for-bit fp32h3 outputs of each variant.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${PROF_TAG:-r6cf}
mkdir -p gpurun_out
for v in main cf1 cf2 cf3 main cf1 cf2 cf3; do
  if [ "$v" = main ]; then unset SPE_LIB_PATH; else export SPE_LIB_PATH=ab_$v/libspe.so; fi
  echo "$v $(timeout -k 10 120 python scripts/x6_bench.py --only l4 --dtypes fp32h3 --iters 20 | tr '\n' ' ')" || exit 1
done
timeout -k 10 600 python -u scripts/lab/bitwise_forward.py dump gpurun_out/${TAG}_main.npz > gpurun_out/${TAG}_dump_main.log 2>&1 || exit 2
for v in cf1 cf2 cf3; do
  export SPE_LIB_PATH=ab_$v/libspe.so
  timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q -k "gemm_h3_close" --timeout 200 --timeout-method thread > gpurun_out/${TAG}_${v}_tests.log 2>&1 \
    || { grep -E "^E |FAILED" gpurun_out/${TAG}_${v}_tests.log | head; exit 3; }
  timeout -k 10 600 python -u scripts/lab/bitwise_forward.py dump gpurun_out/${TAG}_$v.npz > gpurun_out/${TAG}_dump_$v.log 2>&1 || exit 4
  echo "$v $(tail -1 gpurun_out/${TAG}_${v}_tests.log) $(python scripts/lab/bitwise_forward.py compare gpurun_out/${TAG}_main.npz gpurun_out/${TAG}_$v.npz | tail -1)"
done
rm -f gpurun_out/${TAG}_*.npz
echo done
