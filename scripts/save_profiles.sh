#!/bin/bash
# Copy one profiling session's summaries (scripts/gpu_round_profile.sh, PROF_TAG=<tag>) from the
# scratch gpurun_out/ into the tracked profiles/ directory.  Usage: bash scripts/save_profiles.sh <tag>
set -e
T=$1
cd "$(dirname "$0")/.."
cp gpurun_out/prof_$T/bench_kernel_stats.csv profiles/${T}_kernel_stats.csv
cp gpurun_out/prof_$T/bench_kernel_stats_model.csv profiles/${T}_kernel_stats_model.csv
grep '^{"metric"' gpurun_out/prof_$T/bench_under_rocprof.log > profiles/${T}_bench_under_rocprof.json
tail -1 gpurun_out/${T}_bench.log > profiles/${T}_bench.json
cp gpurun_out/${T}_launch_table.json profiles/
for c in 3 4 5; do tail -1 gpurun_out/${T}_bench_c$c.log > profiles/${T}_bench_c$c.json; done
tail -1 gpurun_out/${T}_bench_fp32.log > profiles/${T}_bench_fp32.json
tail -1 gpurun_out/${T}_bench_fp32x3.log > profiles/${T}_bench_fp32x3.json
for mdl in rtdetr_r18 rtdetr_r50; do tail -1 gpurun_out/${T}_bench_$mdl.log > profiles/${T}_bench_$mdl.json; done
tail -1 gpurun_out/${T}_pytest_gpu.log > profiles/${T}_pytest_gpu.log
python3 scripts/launch_summary.py gpurun_out/${T}_launch_table.json --out profiles/${T}_class_roofline.json
python3 scripts/pmc_traffic.py gpurun_out/pmc_$T --kernel "attn16_kernelILi0EDF16b" --kind attn.enc --grid 2883584 \
  --out profiles/pmc_attn.enc.json > /dev/null
cp gpurun_out/${T}_counters_pconv.json profiles/counters_pconv_${T}.json
