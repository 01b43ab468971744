#!/bin/bash
# Round 6: the six-stage few-row h3 GEMM for the decoder's long-K linear2 -- h3 GEMM tests, fp32h3
# goldens, a bit-for-bit comparison of the fp32h3 model outputs (configs 2 / 4 / 5) against the
# previous tree's library (ab_old/libspe.so), the serialized launch table, and old / new bench lines.
# (ab_old/libspe.so: the previous commit built in a git worktree,
#  make -C <worktree>/satellite-pose-estimation_amd/csrc OBJDIR=/tmp/obj OUT=$PWD/ab_old/libspe.so)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${PROF_TAG:-r6frd}
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_parity.py -m gpu -x -q -k "h3" --timeout 300 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 \
  || { grep -E "^E |FAILED" gpurun_out/${TAG}_tests.log | head; exit 1; }
tail -1 gpurun_out/${TAG}_tests.log
SPE_LIB_PATH=ab_old/libspe.so timeout -k 10 600 python -u scripts/lab/bitwise_forward.py dump gpurun_out/${TAG}_old.npz > gpurun_out/${TAG}_dump_old.log 2>&1 \
  || { tail -5 gpurun_out/${TAG}_dump_old.log; exit 2; }
timeout -k 10 600 python -u scripts/lab/bitwise_forward.py dump gpurun_out/${TAG}_new.npz > gpurun_out/${TAG}_dump_new.log 2>&1 \
  || { tail -5 gpurun_out/${TAG}_dump_new.log; exit 3; }
python scripts/lab/bitwise_forward.py compare gpurun_out/${TAG}_old.npz gpurun_out/${TAG}_new.npz | tee gpurun_out/${TAG}_bitwise.txt
if [ -f ab_frdall/libspe.so ]; then
  SPE_LIB_PATH=ab_frdall/libspe.so timeout -k 10 600 python -u scripts/lab/bitwise_forward.py dump gpurun_out/${TAG}_all.npz > gpurun_out/${TAG}_dump_all.log 2>&1 \
    || { tail -5 gpurun_out/${TAG}_dump_all.log; exit 3; }
  python scripts/lab/bitwise_forward.py compare gpurun_out/${TAG}_old.npz gpurun_out/${TAG}_all.npz | tee gpurun_out/${TAG}_bitwise_all.txt
fi
rm -f gpurun_out/${TAG}_*.npz
timeout -k 10 400 python bench.py --dtype fp32h3 --no-parity --no-accuracy --no-cpu-baseline --no-host-input --no-overlap --steps 3 --warmup 2 \
  --launch-table gpurun_out/${TAG}_lt.json > gpurun_out/${TAG}_lt.log 2>&1 || { tail -5 gpurun_out/${TAG}_lt.log; exit 4; }
python3 - gpurun_out/${TAG}_lt.json <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
t = {}
for r in d:
    t.setdefault(r["kind"], []).append(r["ms"])
print({k: round(sum(v), 3) for k, v in t.items() if "dec" in k or "xsplit" in k})
print([round(r["ms"] * 1e3, 1) for r in d if r["kind"] == "gemm.dec"][:7])
PY
SPE_LIB_PATH=ab_frdall/libspe.so timeout -k 10 400 python bench.py --dtype fp32h3 --no-parity --no-accuracy --no-cpu-baseline --no-host-input --no-overlap --steps 3 --warmup 2 \
  --launch-table gpurun_out/${TAG}_lt_all.json > gpurun_out/${TAG}_lt_all.log 2>&1 || { tail -5 gpurun_out/${TAG}_lt_all.log; exit 4; }
python3 - gpurun_out/${TAG}_lt_all.json <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
t = {}
for r in d:
    t.setdefault(r["kind"], []).append(r["ms"])
print("all", {k: round(sum(v), 3) for k, v in t.items() if "dec" in k or "xsplit" in k})
print([round(r["ms"] * 1e3, 1) for r in d if r["kind"] == "gemm.dec"][:7])
PY
for v in old main all old main all; do
  case $v in main) unset SPE_LIB_PATH ;; old) export SPE_LIB_PATH=ab_old/libspe.so ;; all) export SPE_LIB_PATH=ab_frdall/libspe.so ;; esac
  timeout -k 10 300 python bench.py --dtype fp32h3 --steps 20 --warmup 3 --no-cpu-baseline --no-accuracy --no-parity > gpurun_out/${TAG}_ab_$v.log 2>&1 \
    || { tail -20 gpurun_out/${TAG}_ab_$v.log; exit 5; }
  echo "$v $(tail -1 gpurun_out/${TAG}_ab_$v.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['value'],1), round(d['ms_per_step'],2))")"
done
unset SPE_LIB_PATH
echo done
