#!/bin/bash
# pconv ablations (wrong results, timing only): 1 no barrier, 2 no weight DMA, 4 no fragment reads
cd "${GRAFT_REPO_ROOT:-/root/repo}"
for a in 0 1 2 4 3 7; do
  echo "abl=$a"; SPE_PCONV_ABL=$a timeout -k 10 120 python scripts/kbench.py gemm --only 3x3 --iters 20 2>&1 | grep 3x3 || exit 1
done
