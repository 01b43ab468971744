#!/bin/bash
# FETCH_SIZE and WRITE_SIZE of every launch class of one serialised bench step, each counter in
# its own rocprofv3 pass (--kernel-trace beside it only), then scripts/pmc_kinds.py.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
D=gpurun_out/pmc_kinds${PMC_SUFFIX:-}
mkdir -p $D
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 300 rocprofv3 --kernel-trace --pmc $C --kernel-exclude-regex "Cijk|at::|rocprim|hipcub|rocclr" \
    --output-format csv -d $D/$C -o run -- \
    python3 bench.py --steps 1 --warmup 1 --no-overlap --no-cpu-baseline --no-accuracy --no-parity --no-host-input ${BENCH_ARGS:-} \
    --launch-table $D/lt.json > $D/$C.log 2>&1 || { echo "pmc pass $C failed"; tail -5 $D/$C.log; exit 6; }
  find $D/$C -name "*kernel_trace*" -delete
done
python3 scripts/pmc_kinds.py $D --table $D/lt.json --out $D/pmc_kinds.json --mode ${PMC_MODE:-bf16}
