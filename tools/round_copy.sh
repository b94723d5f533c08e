#!/bin/bash
# Copy the judged artefacts of tools/gpu_round.sh from gpurun_out/round/ into profiles/ (round tag $1).
set -eu
R=${1:-r01}
cd "$(dirname "$0")/.."
IN=gpurun_out/round
for c in cfg2 cfg3 cfg5 cfg5_global; do tail -n 1 $IN/bench_$c.log | python -m json.tool > profiles/${R}_bench_$c.json; done
cp $IN/pytest_gpu.log profiles/${R}_pytest_gpu.log
cp "$(find $IN/kt -name '*kernel_stats.csv' | head -1)" profiles/${R}_kernel_stats_cfg2.csv
cp "$(find $IN/kt5 -name '*kernel_stats.csv' | head -1)" profiles/${R}_kernel_stats_cfg5_depthfirst.csv
cp $IN/pmc_summary.txt profiles/${R}_pmc_cfg2.txt
cp $IN/traffic.json profiles/traffic_${R}.json
ls -la profiles
