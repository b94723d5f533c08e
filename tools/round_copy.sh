#!/bin/bash
# Copy the judged artefacts of tools/gpu_round.sh from gpurun_out/round/ into profiles/ (round tag $1).
set -eu
R=${1:-r02}
cd "$(dirname "$0")/.."
IN=gpurun_out/round
for f in $IN/bench_*.log; do
  b=$(basename $f .log); tail -n 1 $f | python -m json.tool > profiles/${R}_$b.json
done
[ -f $IN/pytest_gpu.log ] && cp $IN/pytest_gpu.log profiles/${R}_pytest_gpu.log
[ -f $IN/smoke.log ] && cp $IN/smoke.log profiles/${R}_smoke.log
for d in $IN/kt_*; do
  c=${d##*/kt_}
  f=$(find $d -name '*kernel_stats.csv' | head -1); [ -n "$f" ] && cp "$f" profiles/${R}_kernel_stats_$c.csv
done
for f in $IN/pmc_summary_*.txt; do [ -f $f ] && cp $f profiles/${R}_$(basename $f); done
for f in $IN/pmc_blend_*.json; do [ -f $f ] && cp $f profiles/${R}_$(basename $f); done
ls -la profiles
