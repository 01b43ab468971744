#!/bin/bash
# A/B: the bf16 FFN with non-temporal x loads / y stores (spe/libspe_nt.so) against the tree's build
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for v in main nt main nt; do
  if [ $v = main ]; then unset SPE_LIB_PATH; else export SPE_LIB_PATH=satellite-pose-estimation_amd/spe/libspe_nt.so; fi
  timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-parity --no-accuracy > gpurun_out/nt_$v.json 2> gpurun_out/nt_$v.err \
    || { tail -5 gpurun_out/nt_$v.err; exit 2; }
  python -c "
import json; d=json.loads(open('gpurun_out/nt_$v.json').read().strip().splitlines()[-1]); k=d['kernel_time_ms_per_step']
print('$v', round(d['value']), round(d['ms_per_step'],3), {x: round(k[x],3) for x in ('ffn.enc','attn.enc','conv.1x1','gemm.enc.qk')})"
done
export SPE_LIB_PATH=satellite-pose-estimation_amd/spe/libspe_nt.so
bash scripts/gpu_pmc_kinds.sh > gpurun_out/nt_pmc.txt 2>&1 || { tail -5 gpurun_out/nt_pmc.txt; exit 3; }
python3 -c "
import json; d=json.load(open('gpurun_out/pmc_kinds/pmc_kinds.json'))['classes']
print({k: round(v['counter_over_algorithmic'],2) for k,v in d.items() if k in ('ffn.enc','conv.1x1','attn.enc')})"
