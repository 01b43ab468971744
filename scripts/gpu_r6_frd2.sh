#!/bin/bash
# Round 6: column width / depth of the few-row long-K h3 GEMM form (variant libraries ab_<v>/libspe.so):
# h3 GEMM tests, bit-for-bit fp32h3 outputs against ab_old, the serialized decoder launches.
# (ab_old/libspe.so: the previous commit built in a git worktree,
#  make -C <worktree>/satellite-pose-estimation_amd/csrc OBJDIR=/tmp/obj OUT=$PWD/ab_old/libspe.so)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${PROF_TAG:-r6frd2}
mkdir -p gpurun_out
SPE_LIB_PATH=ab_old/libspe.so timeout -k 10 600 python -u scripts/lab/bitwise_forward.py dump gpurun_out/${TAG}_old.npz > gpurun_out/${TAG}_dump_old.log 2>&1 \
  || { tail -5 gpurun_out/${TAG}_dump_old.log; exit 2; }
for v in ${VARIANTS:-fj1 fj1n7}; do
  if [ "$v" = main ]; then unset SPE_LIB_PATH; else export SPE_LIB_PATH=ab_$v/libspe.so; fi
  timeout -k 10 500 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_parity.py -m gpu -x -q -k "${TESTK:-gemm_h3_close}" --timeout 200 --timeout-method thread > gpurun_out/${TAG}_${v}_tests.log 2>&1 \
    || { grep -E "^E |FAILED" gpurun_out/${TAG}_${v}_tests.log | head; exit 1; }
  echo "$v $(tail -1 gpurun_out/${TAG}_${v}_tests.log)"
  timeout -k 10 600 python -u scripts/lab/bitwise_forward.py dump gpurun_out/${TAG}_$v.npz > gpurun_out/${TAG}_dump_$v.log 2>&1 \
    || { tail -5 gpurun_out/${TAG}_dump_$v.log; exit 3; }
  python scripts/lab/bitwise_forward.py compare gpurun_out/${TAG}_old.npz gpurun_out/${TAG}_$v.npz > gpurun_out/${TAG}_bitwise_$v.txt
  tail -1 gpurun_out/${TAG}_bitwise_$v.txt
  timeout -k 10 400 python bench.py --dtype fp32h3 --no-parity --no-accuracy --no-cpu-baseline --no-host-input --no-overlap --steps 3 --warmup 2 \
    --launch-table gpurun_out/${TAG}_lt_$v.json > gpurun_out/${TAG}_lt_$v.log 2>&1 || { tail -5 gpurun_out/${TAG}_lt_$v.log; exit 4; }
  python3 - gpurun_out/${TAG}_lt_$v.json <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
t = {}
for r in d:
    t.setdefault(r["kind"], []).append(r["ms"])
print({k: round(sum(v), 3) for k, v in t.items() if "dec" in k or "xsplit" in k})
print([round(r["ms"] * 1e3, 1) for r in d if r["kind"] == "gemm.dec"][:7])
PY
done
rm -f gpurun_out/${TAG}_*.npz
echo done
