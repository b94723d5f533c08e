#!/bin/bash
# One GPU session: parity tests, smoke, benchmark, kernel-trace profile.
# Every GPU step has its own time limit; a crash/timeout (rc other than 0/1) ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "--- $name rc=$rc"; tail -n 25 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "ABORT after $name (rc=$rc)"; exit $rc; fi
  return $rc
}
step pytest_gpu 1100 python -m pytest tests -m gpu -q -rf ${PYTEST_ARGS:-}
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench 600 python bench.py --steps ${BENCH_STEPS:-50} --warmup 5
if [ "${PROFILE:-1}" = "1" ]; then
  step rocprof 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- \
       python bench.py --steps 20 --warmup 3 --cpu-baseline 0 --parity 0 --orbit-steps 0 --inflight-steps 0 --virtual-ranks 0
  find gpurun_out/prof -name "*kernel_stats.csv" -exec cp {} gpurun_out/kernel_stats.csv \; 2>/dev/null
  head -n 30 gpurun_out/kernel_stats.csv 2>/dev/null
fi
echo "=== done"
