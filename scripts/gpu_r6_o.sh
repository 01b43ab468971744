#!/bin/bash
# Round 6 A/B: ffn_h3 with non-temporal activation accesses (kbench; variant library via SPE_LIB_PATH).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
for lib in libspe.so libspe_nt.so libspe.so libspe_nt.so; do
  echo -n "$lib "; SPE_LIB_PATH=satellite-pose-estimation_amd/spe/$lib timeout -k 10 120 python3 scripts/kbench.py ffnh3 --iters 20 2>&1 | grep ffn || exit 1
done
