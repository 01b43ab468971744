#!/bin/bash
# attention A/B: kernel tests on the tree's library, then the interleaved bench against ablate/old
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TESTK="attention" bash scripts/gpu_ab_lib.sh
