#!/bin/bash
# Same-box A/B of the decoder's 16-row kernels (decffn + decq, SPE_DECFFN) on the bench line.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${PROF_TAG:-r5ab}
mkdir -p gpurun_out
for i in 1 2; do
  for v in 0 1; do
    SPE_DECFFN=$v timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-parity --no-accuracy \
      > gpurun_out/${TAG}_decffn${v}_$i.json 2> gpurun_out/${TAG}_decffn${v}_$i.err || { tail -5 gpurun_out/${TAG}_decffn${v}_$i.err; exit 3; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], round(d['value'],1), round(d['ms_per_step'],3))" \
      gpurun_out/${TAG}_decffn${v}_$i.json "decffn=$v run $i"
  done
done
