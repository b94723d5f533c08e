#!/bin/bash
# r06: the multi-GPU options / RCCL transport / mapping-check tests first, then the whole GPU suite and the
# extended VALU probe.  Each step under its own time limit; a failure ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_multigpu_rccl.py tests/test_multigpu_ipc.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_mg.log 2>&1
rc=$?; echo "pytest mg rc=$rc: $(tail -n 1 gpurun_out/pytest_mg.log)"
[ $rc -eq 0 ] || { grep -E "PASS|FAIL|ERROR" gpurun_out/pytest_mg.log | tail -30; tail -n 60 gpurun_out/pytest_mg.log; exit $rc; }
if [ "${FULL:-1}" = 1 ]; then
  timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
  rc=$?; echo "pytest rc=$rc: $(tail -n 1 gpurun_out/pytest_gpu.log)"
  [ $rc -eq 0 ] || { tail -n 40 gpurun_out/pytest_gpu.log; exit $rc; }
fi
if [ "${PEAK:-1}" = 1 ]; then
  timeout -k 10 300 tools/exp/valu_peak > gpurun_out/valu_peak_r06.txt 2>&1 || { echo "valu_peak failed"; tail -5 gpurun_out/valu_peak_r06.txt; exit 1; }
  grep -E "waves/SIMD=(4|8)" gpurun_out/valu_peak_r06.txt | tail -12
fi
echo "=== done"
