#!/bin/bash
# Attention ablations (variants built by scripts/ab_build.sh) + per-kernel timings of the base build.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 180 python scripts/kbench.py all --iters 20 > gpurun_out/kbench_all.log 2>&1 || { cat gpurun_out/kbench_all.log; exit 1; }
cat gpurun_out/kbench_all.log
for v in ${VARIANTS:-base nomax noexp nols nostage noexpmax occ2 occ4}; do
  echo "== $v"; SPE_LIB_PATH=ablate/$v/libspe.so timeout -k 10 120 python scripts/kbench.py ${WHICH:-attn} --iters 20 || exit 2
done
