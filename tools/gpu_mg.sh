#!/bin/bash
# Multi-GPU frame checks on a one-GPU box: the product path with processes sharing the GPU, the
# virtual-rank tests, and the bench's N=2 rehearsal.  Every GPU step has its own time limit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "--- $name rc=$rc"; tail -n 30 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "ABORT after $name (rc=$rc)"; exit $rc; fi
  return $rc
}
step mg_tests 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread ${MG_TESTS:-tests/test_multigpu_ipc.py tests/test_multigpu_rccl.py}
if [ "${MG_BENCH:-1}" = "1" ]; then
  BENCH_SAME_GPU=1 step bench_w2 600 python bench.py --gpus 2 --steps 20 --warmup 3 --multi-extra-config none
fi
echo "=== done"
