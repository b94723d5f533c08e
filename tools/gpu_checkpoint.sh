#!/bin/bash
# Round checkpoint: parity, smoke, bench (1080p + 4K), kernel-trace profile, PMC passes.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/gpu_check.sh || exit $?
timeout -k 10 600 python bench.py --config cfg3_5m_sh3_4k_f16 --steps 30 --warmup 3 --cpu-baseline 0 > gpurun_out/bench_4k.log 2>&1; rc=$?
echo "bench_4k rc=$rc"; tail -n 2 gpurun_out/bench_4k.log
[ $rc -eq 0 ] || exit $rc
bash tools/gpu_pmc.sh
