#!/bin/bash
# PMC passes over the fp32x6 GEMM (scripts/x6_bench.py --only <shape>), one counter set per run
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${PROF_TAG:-x6}
ONLY=${ONLY:-ffn1}
A="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"
B="SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_MFMA SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU"
C="SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_VALU_MFMA_COEXEC_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MFMA SQ_INST_CYCLES_VMEM"
mkdir -p gpurun_out/pmc_$TAG
i=0
for S in "$A" "$B" "$C"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $S --output-format csv -d gpurun_out/pmc_$TAG/set$i -o kb -- \
    python3 scripts/x6_bench.py --only $ONLY --iters 3 > gpurun_out/pmc_$TAG/set$i.log 2>&1 \
    || { echo "pmc set $i failed"; tail -5 gpurun_out/pmc_$TAG/set$i.log; exit 6; }
done
python3 scripts/pmc_summary.py gpurun_out/pmc_$TAG --min-us 50
