#!/bin/bash
# Kernel timeline of a short bench run (rocprofv3 --kernel-trace, CSV): per-dispatch start/end
# for the overlap analysis in scripts/timeline_summary.py.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/timeline
timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/timeline -o tl -- \
  python3 bench.py --steps 6 --warmup 2 --no-cpu-baseline --no-accuracy > gpurun_out/timeline/bench.log 2>&1 \
  || { tail -20 gpurun_out/timeline/bench.log; exit 1; }
f=$(find gpurun_out/timeline -name "*kernel_trace.csv" | head -1)
python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
keep = [r for r in rows if not r["Kernel_Name"].startswith(("void at::", "void rocprim", "__amd_rocclr", "Cijk_", "void (anonymous namespace)::indexing", "void (anonymous namespace)::elementwise_kernel_with_index"))]
# the last 4 bench steps: the final ~12*4 ms of our kernels
keep.sort(key=lambda r: int(r["Start_Timestamp"]))
out = open("gpurun_out/timeline/ours.csv", "w")
w = csv.writer(out)
w.writerow(["start", "end", "queue", "name"])
for r in keep[-2500:]:
    w.writerow([r["Start_Timestamp"], r["End_Timestamp"], r.get("Queue_Id", r.get("Stream_Id", "")), r["Kernel_Name"][:80]])
print(len(rows), len(keep))
PY
find gpurun_out/timeline -name "*kernel_trace.csv" -delete
