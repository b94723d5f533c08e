#!/bin/bash
# Round-2 GPU session helper: parity tests, then kernel traces of configs 2 and 3.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r02
mkdir -p $OUT
export TMPDIR=/tmp
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "--- $name rc=$rc"; tail -n 4 "$OUT/$name.log"
  if [ $rc -ne 0 ]; then echo "ABORT after $name (rc=$rc)"; exit $rc; fi
}
if [ "${TESTS:-1}" = 1 ]; then
  step pytest_gpu 700 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread
fi
for cfg in ${CFGS:-cfg2_1m_sh3_1080p_f16 cfg3_5m_sh3_4k_f16}; do
  step kt_$cfg 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt_$cfg -o run -- \
       python bench.py --config $cfg --steps 20 --warmup 3 --cpu-baseline 0 --parity 0
  find $OUT/kt_$cfg -name "*kernel_stats.csv" -exec cp {} $OUT/stats_$cfg.csv \;
  tail -n 1 $OUT/kt_$cfg.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['value'],1), {k: round(v*1e3,1) for k,v in d['stages_ms'].items()})"
done
echo "=== done"
