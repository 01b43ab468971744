set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "periodic or stream or gemm_shapes" > gpurun_out/rm_t.log 2>&1; rc=$?; tail -1 gpurun_out/rm_t.log; [ $rc = 0 ] || { grep -E "^E |FAILED" gpurun_out/rm_t.log | head; exit 1; }
for v in 0 1 0 1; do
  SPE_SG_RMAP=$v timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-parity > gpurun_out/rm_b$v.json 2>gpurun_out/rm_b$v.err || { tail -5 gpurun_out/rm_b$v.err; exit 3; }
  python -c "
import json; d=json.loads(open('gpurun_out/rm_b$v.json').read().strip().splitlines()[-1]); k=d['kernel_time_ms_per_step']
print('rmap=$v', round(d['value']), round(d['ms_per_step'],3), {x: round(k[x],3) for x in ('gemm.enc.qk','attn.enc','conv.1x1')})"
done
