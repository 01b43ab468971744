#!/bin/bash
# Round 6, baseline of the accuracy-contract mode (fp32h3): the fp32x3 encoder attention alone
# (kbench, timing + two SQ counter passes), rocprofv3 kernel stats of the fp32h3 bench, and the
# per-class FETCH / WRITE passes of one serialised fp32h3 step.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${PROF_TAG:-r6a}
mkdir -p gpurun_out
KBA="attn --attn-dtype 4 --presplit"
timeout -k 10 120 python3 scripts/kbench.py $KBA --iters 20 > gpurun_out/${TAG}_kb_attn_x3.log 2>&1 \
  || { tail -20 gpurun_out/${TAG}_kb_attn_x3.log; exit 1; }
cat gpurun_out/${TAG}_kb_attn_x3.log
A="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"
B="SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_MFMA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_COEXEC_CYCLES"
KB="$KBA" PROF_TAG=${TAG}_x3 PMC_SETS="$A;$B" bash scripts/gpu_pmc_kbench.sh > gpurun_out/${TAG}_pmc_x3.log 2>&1 \
  || { tail -20 gpurun_out/${TAG}_pmc_x3.log; exit 2; }
tail -30 gpurun_out/${TAG}_pmc_x3.log
BENCH_ARGS="--dtype fp32h3" PROF_TAG=${TAG}_fp32h3 bash scripts/gpu_profile.sh || exit 3
BENCH_ARGS="--dtype fp32h3" PMC_SUFFIX=_${TAG}_h3 PMC_MODE=fp32h3 bash scripts/gpu_pmc_kinds.sh > gpurun_out/${TAG}_pmc_kinds_h3.log 2>&1 \
  || { tail -20 gpurun_out/${TAG}_pmc_kinds_h3.log; exit 4; }
echo a done
