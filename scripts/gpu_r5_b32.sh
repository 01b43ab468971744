#!/bin/bash
# Per-class time per image at the north star's per-GPU batch (32, config 3) against config 2's 64, same box.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${PROF_TAG:-r5y}
mkdir -p gpurun_out
for c in 2 3; do
  timeout -k 10 300 python bench.py --config $c --steps 20 --warmup 3 --no-cpu-baseline --no-parity --no-accuracy \
    --launch-table gpurun_out/${TAG}_c${c}_launch_table.json > gpurun_out/${TAG}_c$c.json 2> gpurun_out/${TAG}_c$c.err \
    || { tail -5 gpurun_out/${TAG}_c$c.err; exit 3; }
  python3 scripts/launch_summary.py gpurun_out/${TAG}_c${c}_launch_table.json --out gpurun_out/${TAG}_c${c}_class_roofline.json > /dev/null
  tail -1 gpurun_out/${TAG}_c$c.json | cut -c1-160
done
for c in 2 3; do
  timeout -k 10 300 python bench.py --config $c --dtype fp32h3 --steps 10 --warmup 2 --no-cpu-baseline --no-parity --no-accuracy \
    --launch-table gpurun_out/${TAG}_h3c${c}_launch_table.json > gpurun_out/${TAG}_h3c$c.json 2> gpurun_out/${TAG}_h3c$c.err \
    || { tail -5 gpurun_out/${TAG}_h3c$c.err; exit 4; }
  python3 scripts/launch_summary.py gpurun_out/${TAG}_h3c${c}_launch_table.json --out gpurun_out/${TAG}_h3c${c}_class_roofline.json > /dev/null
  tail -1 gpurun_out/${TAG}_h3c$c.json | cut -c1-160
done
