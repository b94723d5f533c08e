#!/bin/bash
# A/B of the first tile pass width (GSM_SORT_LOBITS) on configs 2 and 3: kernel-trace stats + bench line.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/lobits; mkdir -p $OUT; export TMPDIR=/tmp
for cfg in cfg2_1m_sh3_1080p_f16 cfg3_5m_sh3_4k_f16; do
  for lb in 0 ${LBS:-5 6 7 8}; do
    GSM_SORT_LOBITS=$lb timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt_${lb}_$cfg -o run -- \
      python bench.py --config $cfg --steps 30 --warmup 3 --cpu-baseline 0 --parity 0 --orbit-steps 0 --inflight-steps 0 \
      > $OUT/kt_${lb}_$cfg.log 2>&1 || { echo "rocprof failed $lb $cfg"; tail -n 5 $OUT/kt_${lb}_$cfg.log; exit 1; }
    f=$(find $OUT/kt_${lb}_$cfg -name '*kernel_stats.csv' | head -n 1)
    python3 - "$f" "lobits=$lb $cfg" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
print(sys.argv[2])
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:10]:
    if 'radix' in r['Name'] or 'tile' in r['Name']:
        print(f"  {r['Name'].split('(')[0][:60]:60s} calls={int(r['Calls']):5d} avg_us={float(r['AverageNs'])/1e3:8.1f}")
PY
    GSM_SORT_LOBITS=$lb timeout -k 10 300 python bench.py --config $cfg --steps 50 --warmup 5 --cpu-baseline 0 --orbit-steps 0 \
      --inflight-steps 0 --traffic-json /dev/null > $OUT/bench_${lb}_$cfg.log 2>&1 || { echo "bench failed $lb $cfg"; tail -n 5 $OUT/bench_${lb}_$cfg.log; exit 1; }
    grep '"metric"' $OUT/bench_${lb}_$cfg.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('  bench', round(d['value'],1), 'parity', d.get('parity_vs_oracle'), {k: round(x*1e3,1) for k,x in d['stages_ms'].items()})"
  done
done
echo "=== done"
