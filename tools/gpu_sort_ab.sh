#!/bin/bash
# r05: scanless narrow radix passes (default) against the k_radix_scan passes (GSM_SORT_SCAN=kernel):
# GPU parity tests, bench lines of configs 2 and 3 both ways (twice, interleaved), and a kernel trace of
# config 2 with the default.  Extra variants: VARIANTS="label:ENV=a,ENV=b ..." (config 2).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/sort; mkdir -p $O; export TMPDIR=/tmp
if [ "${TESTS:-1}" = 1 ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
  rc=$?; echo "pytest rc=$rc: $(tail -n 1 $O/pytest.log)"
  [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/pytest.log | head -20; exit $rc; }
fi
b() {  # label cfg env...
  local label=$1 cfg=$2; shift 2
  env "$@" timeout -k 10 300 python bench.py --config $cfg --steps ${STEPS:-100} --warmup 5 --cpu-baseline 0 \
    --orbit-steps ${ORBIT:-50} --inflight-steps 0 --virtual-ranks 0 --traffic-json /dev/null > $O/bench_$label.log 2>&1
  local rc=$?
  [ $rc -eq 0 ] || { echo "bench $label rc=$rc"; tail -n 5 $O/bench_$label.log; exit $rc; }
  grep '"metric"' $O/bench_$label.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); o=d.get('orbit') or {}; print('$label', round(d['value'],1), 'ms', round(d['ms_per_step'],4), 'parity', d.get('parity_vs_oracle'), {k: round(x*1e3,1) for k, x in d['stages_ms'].items()}, 'orbit', round(o.get('value',0),1), o.get('parity_last_frame'))"
}
for r in 1 2; do
  b scanless_cfg2_$r cfg2_1m_sh3_1080p_f16 GSM_SORT_SCAN=none
  b kernel_cfg2_$r cfg2_1m_sh3_1080p_f16 GSM_SORT_SCAN=kernel
done
for v in ${VARIANTS:-}; do
  b ${v%%:*}_cfg2 cfg2_1m_sh3_1080p_f16 $(echo ${v#*:} | tr ',' ' ')
done
b scanless_cfg3 cfg3_5m_sh3_4k_f16 GSM_SORT_SCAN=none
b kernel_cfg3 cfg3_5m_sh3_4k_f16 GSM_SORT_SCAN=kernel
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 bench.py \
  --config cfg2_1m_sh3_1080p_f16 --steps 30 --warmup 3 --cpu-baseline 0 --parity 0 --orbit-steps 0 --inflight-steps 0 \
  --virtual-ranks 0 > $O/kt.log 2>&1 || { echo "kt rc=$?"; exit 1; }
python3 - <<'EOF'
import csv, glob
f = glob.glob("gpurun_out/sort/kt/**/*kernel_stats.csv", recursive=True)
for r in list(csv.DictReader(open(f[0])))[:12]:
    print(f'{r["Name"][:60]:60s} {r["Calls"]:>6} {float(r["AverageNs"])/1e3:8.2f}')
EOF
echo done
