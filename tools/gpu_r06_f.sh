#!/bin/bash
# r06: GPU suite on the tree, kernel traces of configs 2 / 3 for HEAD against the tree, then the same-GPU
# N-rank rehearsals of bench.py's multi-GPU frame (tools/gpu_bench_same_gpu.sh).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc: $(tail -n 1 gpurun_out/pytest_gpu.log)"
[ $rc -eq 0 ] || { grep -E "^FAILED|Error|error" gpurun_out/pytest_gpu.log | head -20; grep -B5 -A60 "^_____" gpurun_out/pytest_gpu.log | head -150; exit $rc; }
VARIANTS="head cur" REPS=2 bash tools/gpu_ab_proj.sh || exit 1
bash tools/gpu_bench_same_gpu.sh || exit 1
echo "=== done"
