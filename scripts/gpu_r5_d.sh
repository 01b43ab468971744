#!/bin/bash
# Round 5: fp32h3 after the amax-publish fix (read the slot before the atomic) -- kernel tests,
# goldens, the parity line in fp32h3 with its launch table, and fp32x6 on the same box.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
T="timeout -k 10"
$T 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "h3 or x6" \
  > gpurun_out/d_kernels.log 2>&1 || { grep -E "^E |FAILED|Error" gpurun_out/d_kernels.log | head -30; tail -5 gpurun_out/d_kernels.log; exit 2; }
tail -1 gpurun_out/d_kernels.log
$T 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "forward_fp32" \
  > gpurun_out/d_parity.log 2>&1 || { grep -E "^E |FAILED|Error" gpurun_out/d_parity.log | head -30; exit 3; }
tail -1 gpurun_out/d_parity.log
for dt in ${DTS:-fp32h3 fp32x6}; do
  $T 600 python bench.py --dtype $dt --no-parity --no-cpu-baseline --steps 10 --warmup 2 --launch-table gpurun_out/d_launch_$dt.json \
    > gpurun_out/d_bench_$dt.json 2> gpurun_out/d_bench_$dt.err || { tail -20 gpurun_out/d_bench_$dt.err; exit 4; }
  python -c "
import json; d=json.loads(open('gpurun_out/d_bench_$dt.json').read().strip().splitlines()[-1])
print('$dt', round(d['value']), round(d['ms_per_step'],2), {k: round(v,3) for k,v in d['kernel_time_ms_per_step'].items()})"
done
