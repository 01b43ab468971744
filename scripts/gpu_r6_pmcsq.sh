#!/bin/bash
# Round 6: SQ counter passes (two sets, separate runs) over one serialised bench step in fp32h3 and
# in bf16 -- what binds the GEMM / conv / FFN kernels of each mode.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
A="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"
B="SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_MFMA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_COEXEC_CYCLES"
BENCH_ARGS="--dtype fp32h3 --no-overlap --no-host-input" PROF_TAG=r6sq_h3 PMC_SETS="$A;$B" bash scripts/gpu_pmc.sh > gpurun_out/r6sq_h3.log 2>&1 || { tail -20 gpurun_out/r6sq_h3.log; exit 1; }
python3 scripts/pmc_summary.py gpurun_out/pmc_r6sq_h3 --min-us 60 > gpurun_out/r6sq_h3_summary.txt 2>&1 || { tail -5 gpurun_out/r6sq_h3_summary.txt; exit 2; }
cat gpurun_out/r6sq_h3_summary.txt
BENCH_ARGS="--no-overlap --no-host-input" PROF_TAG=r6sq_bf16 PMC_SETS="$A;$B" bash scripts/gpu_pmc.sh > gpurun_out/r6sq_bf16.log 2>&1 || { tail -20 gpurun_out/r6sq_bf16.log; exit 3; }
python3 scripts/pmc_summary.py gpurun_out/pmc_r6sq_bf16 --min-us 40 > gpurun_out/r6sq_bf16_summary.txt 2>&1 || { tail -5 gpurun_out/r6sq_bf16_summary.txt; exit 4; }
cat gpurun_out/r6sq_bf16_summary.txt
