#!/bin/bash
# Round 6: the fp32h3 encoder FFN (ffn_h3_kernel) alone -- timing and three SQ counter passes.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${PROF_TAG:-r6n}
timeout -k 10 120 python3 scripts/kbench.py ffnh3 --iters 10 2>&1 | grep ffn || exit 1
A="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"
B="SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_MFMA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_COEXEC_CYCLES"
C="SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_ACTIVE_INST_ANY SQ_INST_LEVEL_LDS SQ_LDS_DATA_FIFO_FULL SQ_LDS_ADDR_CONFLICT SQ_ACTIVE_INST_MFMA SQ_INST_CYCLES_VMEM"
KB="ffnh3" PROF_TAG=${TAG}_ffnh3 PMC_SETS="$A;$B;$C;FETCH_SIZE;WRITE_SIZE" bash scripts/gpu_pmc_kbench.sh > gpurun_out/${TAG}_pmc.log 2>&1 \
  || { tail -20 gpurun_out/${TAG}_pmc.log; exit 2; }
head -3 gpurun_out/${TAG}_pmc.log
