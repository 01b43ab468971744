#!/bin/bash
# PMC passes over the attention lab (each counter set in its own run).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc_lab
i=0
IFS=';' read -ra ARR <<< "$PMC_SETS"
for C in "${ARR[@]}"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $C --output-format csv -d gpurun_out/pmc_lab/set$i -o lab -- \
    scripts/lab/attn_lab ${ITERS:-3} > gpurun_out/pmc_lab/set$i.log 2>&1 || { echo "pmc set $i failed"; tail -5 gpurun_out/pmc_lab/set$i.log; exit 6; }
done
echo done
