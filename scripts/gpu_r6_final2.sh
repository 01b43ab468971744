#!/bin/bash
# Round 6 final snapshot, part 2 (tag r6z): the fp32h3 GEMM test as the first GPU call of a fresh
# process, the default bench line (host_input, parity_mode fp32h3 with accuracy and PMC traffic, CPU
# baseline, launch table), config 3 and the north-star line at N = 1.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
T=${PROF_TAG:-r6z}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  "tests/test_gpu_kernels.py::test_gemm_h3_close_to_fp64[linear-1.0]" > gpurun_out/${T}_h3_first_call.log 2>&1 \
  || { tail -20 gpurun_out/${T}_h3_first_call.log; exit 1; }
tail -1 gpurun_out/${T}_h3_first_call.log
timeout -k 10 900 python bench.py --steps 20 --warmup 3 --cpu-seconds 12 --launch-table gpurun_out/${T}_launch_table.json \
  > gpurun_out/${T}_bench.log 2>&1 || { tail -20 gpurun_out/${T}_bench.log; exit 6; }
tail -1 gpurun_out/${T}_bench.log | cut -c1-300
timeout -k 10 600 python bench.py --config 3 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/${T}_bench_c3.log 2>&1 \
  || { tail -20 gpurun_out/${T}_bench_c3.log; exit 7; }
tail -1 gpurun_out/${T}_bench_c3.log | cut -c1-200
timeout -k 10 800 python bench.py --north-star --no-cpu-baseline --no-host-input > gpurun_out/${T}_ns1.log 2>&1 \
  || { tail -20 gpurun_out/${T}_ns1.log; exit 8; }
tail -1 gpurun_out/${T}_ns1.log | cut -c1-200
echo final2 done
