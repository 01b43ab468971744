#!/bin/bash
# Round 6: SQ counter passes over the split encoder attention (fp16 V planes) in kbench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${PROF_TAG:-r6c}
KBA="attn --attn-dtype 4 --presplit --split-dma --f16v"
A="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"
B="SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_MFMA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_COEXEC_CYCLES"
C="SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_ACTIVE_INST_ANY SQ_INST_LEVEL_LDS SQ_LDS_DATA_FIFO_FULL SQ_LDS_ADDR_CONFLICT SQ_ACTIVE_INST_MFMA SQ_INST_CYCLES_VMEM"
KB="$KBA" PROF_TAG=${TAG}_split PMC_SETS="$A;$B;$C" bash scripts/gpu_pmc_kbench.sh > gpurun_out/${TAG}_pmc_split.log 2>&1 \
  || { tail -20 gpurun_out/${TAG}_pmc_split.log; exit 2; }
head -3 gpurun_out/${TAG}_pmc_split.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread \
  -k "fp32_matches_reference" > gpurun_out/${TAG}_parity.log 2>&1 \
  || { grep -E "^E |FAILED|Error" gpurun_out/${TAG}_parity.log | head -20; tail -5 gpurun_out/${TAG}_parity.log; exit 3; }
tail -1 gpurun_out/${TAG}_parity.log
timeout -k 10 900 python -u -m pytest tests/test_gpu_precision.py -x -q -s --timeout 900 --timeout-method thread \
  > gpurun_out/${TAG}_precision.log 2>&1 \
  || { grep -E "^E |FAILED|Error" gpurun_out/${TAG}_precision.log | head -20; tail -5 gpurun_out/${TAG}_precision.log; exit 4; }
tail -1 gpurun_out/${TAG}_precision.log
timeout -k 10 600 python bench.py --dtype fp32h3 --steps 10 --warmup 2 --no-cpu-baseline --no-parity \
  > gpurun_out/${TAG}_bench_h3.log 2>&1 || { tail -20 gpurun_out/${TAG}_bench_h3.log; exit 5; }
tail -1 gpurun_out/${TAG}_bench_h3.log | cut -c1-300
