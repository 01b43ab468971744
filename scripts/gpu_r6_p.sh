#!/bin/bash
# Round 6 A/B: fp32h3 step with the default stream overlap vs without the backbone / encoder overlap.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
for o in "" "--no-overlap-backbone" "" "--no-overlap-backbone"; do
  echo -n "[$o] "; timeout -k 10 300 python bench.py --dtype fp32h3 --steps 20 --warmup 3 --no-cpu-baseline --no-parity --no-host-input $o 2>/dev/null \
    | tail -1 | python3 -c "import json,sys; r=json.loads(sys.stdin.read()); print(round(r['value'],1), round(r['ms_per_step'],2), round(r['roofline']['avg_launch_ms'],3))" || exit 1
done
