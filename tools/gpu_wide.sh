#!/bin/bash
# Wide radix digits A/B (GSM_SORT_WIDE=0|1): GPU tests, DepthFirst (config 5) and config-2 kernel
# traces, virtual-rank multi-GPU frame at config 4.  Each GPU step has its own time limit; a crash
# or timeout (rc other than 0/1) ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/wide
export TMPDIR=/tmp
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$to" "$@" > "gpurun_out/wide/$name.log" 2>&1
  local rc=$?
  echo "--- $name rc=$rc"; tail -n 6 "gpurun_out/wide/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "ABORT after $name (rc=$rc)"; exit $rc; fi
  return $rc
}
step pytest_gpu 600 python -u -m pytest tests -m gpu -x -q -rf --timeout 120 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"}
for w in ${WIDE_AB:-1 0}; do
  export GSM_SORT_WIDE=$w
  step kt_cfg5_w$w 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/wide/kt5_w$w -o run -- \
       python bench.py --config cfg5_1m_sh2_stereo_2x1440x1600_f16 --steps 20 --warmup 3 --cpu-baseline 0 --parity 0 --orbit-steps 0 --inflight-steps 0 --virtual-ranks 0
  step vr_cfg3_w$w 300 python tools/exp_virtual_ranks.py --config cfg3_5m_sh3_4k_f16 --world 8 --frames 5
  step vr_cfg2_w$w 300 python tools/exp_virtual_ranks.py --config cfg2_1m_sh3_1080p_f16 --world 8 --frames 5
  step vr2_cfg2_w$w 300 python tools/exp_virtual_ranks.py --config cfg2_1m_sh3_1080p_f16 --world 2 --frames 5
done
unset GSM_SORT_WIDE
step vr_trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/wide/vr_prof -o run -- \
     python tools/exp_virtual_ranks.py --config cfg3_5m_sh3_4k_f16 --world 8 --frames 3 --stages 0
for d in gpurun_out/wide/kt5_w1 gpurun_out/wide/kt5_w0 gpurun_out/wide/vr_prof; do
  f=$(find $d -name '*kernel_stats.csv' | head -1)
  [ -n "$f" ] && cp "$f" $d.csv && python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
print(sys.argv[1])
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:16]:
    print(f"  {r['Name'].split('(')[0][:58]:58s} calls={int(r['Calls']):5d} avg_us={float(r['AverageNs'])/1e3:8.1f}")
PY
done
echo "=== done"
