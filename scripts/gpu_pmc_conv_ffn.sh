#!/bin/bash
# PMC sets over the 3x3 conv family (pconv) and the encoder FFN, summaries as JSON for profiles/.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
KB="gemm --only 3x3" PROF_TAG=pconv bash scripts/gpu_pmc_sets.sh > gpurun_out/pmc_pconv.txt 2>&1 || { tail -20 gpurun_out/pmc_pconv.txt; exit 1; }
cat gpurun_out/pmc_pconv.txt
python3 scripts/pmc_summary.py gpurun_out/pmc_pconv --min-us 20 --json gpurun_out/pmc_pconv.json > /dev/null
KB="ffn" PROF_TAG=ffn bash scripts/gpu_pmc_sets.sh > gpurun_out/pmc_ffn.txt 2>&1 || { tail -20 gpurun_out/pmc_ffn.txt; exit 2; }
cat gpurun_out/pmc_ffn.txt
python3 scripts/pmc_summary.py gpurun_out/pmc_ffn --min-us 20 --json gpurun_out/pmc_ffn.json > /dev/null
