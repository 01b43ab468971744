#!/bin/bash
# PMC passes over one kernel family of scripts/kbench.py (each counter set in its own run,
# --kernel-trace only beside it).  Usage: KB=ffn PROF_TAG=ffn1 PMC_SETS="A B;C D" bash scripts/gpu_pmc_kbench.sh
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${PROF_TAG:-kb}
KB=${KB:-ffn}
mkdir -p gpurun_out/pmc_$TAG
i=0
IFS=';' read -ra ARR <<< "$PMC_SETS"
for C in "${ARR[@]}"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $C --output-format csv -d gpurun_out/pmc_$TAG/set$i -o kb -- \
    python3 scripts/kbench.py $KB --iters 3 > gpurun_out/pmc_$TAG/set$i.log 2>&1 \
    || { echo "pmc set $i ($C) failed"; tail -20 gpurun_out/pmc_$TAG/set$i.log; exit 6; }
done
python3 scripts/pmc_summary.py gpurun_out/pmc_$TAG --min-us 50
