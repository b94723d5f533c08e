#!/bin/bash
# r06: the GPU suite, then the freed-uncached reuse child with its stderr (the mapping check's evidence).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc: $(tail -n 1 gpurun_out/pytest_gpu.log)"
[ $rc -eq 0 ] || { grep -E "^FAILED|Error|error" gpurun_out/pytest_gpu.log | head -20; grep -B5 -A60 "^_____" gpurun_out/pytest_gpu.log | head -150; exit $rc; }
timeout -k 10 240 python -u tests/mg_uc_reuse.py gpurun_out/uc_d.json > gpurun_out/uc_d.log 2>&1 || { echo "uc failed rc=$?"; tail -20 gpurun_out/uc_d.log; exit 1; }
grep -v amdgpu.ids gpurun_out/uc_d.log
echo "=== done"
