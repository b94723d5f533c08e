#!/bin/bash
# Kernel-trace summary (rocprofv3 --kernel-trace --stats) of bench.py for each config in $CFGS:
# per-kernel average microseconds, into gpurun_out/kt/<cfg>.txt.  Usage on the box: bash tools/kt.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/kt
for cfg in ${CFGS:-cfg2_1m_sh3_1080p_f16 cfg3_5m_sh3_4k_f16}; do
  rm -rf gpurun_out/kt/$cfg
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kt/$cfg -o run -- \
    python bench.py --config $cfg --steps 20 --warmup 3 --cpu-baseline 0 --parity 0 --orbit-steps 0 --inflight-steps 0 --virtual-ranks 0 \
    > gpurun_out/kt/$cfg.log 2>&1 || { echo "rocprof failed for $cfg"; tail -5 gpurun_out/kt/$cfg.log; exit 1; }
  f=$(find gpurun_out/kt/$cfg -name '*kernel_stats.csv' | head -1)
  python3 - "$f" "$cfg" <<'PY' | tee gpurun_out/kt/$cfg.txt
import csv, sys, json
rows = list(csv.DictReader(open(sys.argv[1])))
print(sys.argv[2])
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"])):
    print(f"  {r['Name'].split('(')[0][:58]:58s} calls={int(r['Calls']):5d} avg_us={float(r['AverageNs'])/1e3:8.1f}")
PY
  grep '"metric"' gpurun_out/kt/$cfg.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('  fps', round(d['value'],1), {k: round(v*1e3,1) for k,v in d['stages_ms'].items()})"
done
