#!/bin/bash
# persistent fp32h3 GEMM alone: timing + PMC on linear1 / cross-K shapes
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python scripts/x6_bench.py --dtypes fp32h3 > gpurun_out/i_x6bench.log 2>&1 || { tail -20 gpurun_out/i_x6bench.log; exit 2; }
grep -v amdgpu.ids gpurun_out/i_x6bench.log
A="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"
B="SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_MFMA SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU"
W="TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum"
for sh in ffn1; do
  i=0; mkdir -p gpurun_out/pmc_i_$sh
  for S in "$A" "$B" "$W"; do
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $S --output-format csv -d gpurun_out/pmc_i_$sh/set$i -o kb -- \
      python3 scripts/x6_bench.py --only $sh --iters 3 --dtypes fp32h3 > gpurun_out/pmc_i_$sh/set$i.log 2>&1 \
      || { echo "pmc set $i failed"; tail -5 gpurun_out/pmc_i_$sh/set$i.log; exit 6; }
  done
  python3 scripts/pmc_summary.py gpurun_out/pmc_i_$sh --min-us 50
done
