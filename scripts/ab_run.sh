cd "${GRAFT_REPO_ROOT:-/root/repo}"
timeout -k 10 120 python scripts/solver_bench.py --batch 32 || exit 1
timeout -k 10 120 python scripts/solver_bench.py --batch 256 || exit 1
for v in base nostage noexp nomax nols nostagebar occ2 occ4 noexpmax; do
  echo "== $v"; SPE_LIB_PATH=ablate/$v/libspe.so timeout -k 10 120 python scripts/kbench.py attn --iters 20 || exit 2
done
