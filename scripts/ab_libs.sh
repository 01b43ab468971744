# kbench A/B over libspe.so variants: LIBS="name ..." (ablate/<name>/libspe.so; "main" = the tree's own),
# KB="attn --attn-dtype 3" (kbench arguments).  Each variant runs twice, interleaved.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
for rep in 1 2; do
  for v in $LIBS; do
    if [ "$v" = main ]; then unset SPE_LIB_PATH; else export SPE_LIB_PATH=ablate/$v/libspe.so; fi
    echo "== $v"; timeout -k 10 120 python scripts/kbench.py $KB --iters 30 || exit 2
  done
done
