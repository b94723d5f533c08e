#!/bin/bash
# r05: the pair-walk blend (k_blend_pw, GSM_BLEND_PAIRS=1 default) against one unit per wave
# (GSM_BLEND_PAIRS=0): GPU parity tests, then bench lines (static + orbit) of configs 2 and 3.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/pw; mkdir -p $O; export TMPDIR=/tmp
if [ "${TESTS:-1}" = 1 ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
  rc=$?; echo "pytest rc=$rc: $(tail -n 1 $O/pytest.log)"
  [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/pytest.log | head -20; exit $rc; }
fi
b() {  # label cfg env...
  local label=$1 cfg=$2; shift 2
  env "$@" timeout -k 10 300 python bench.py --config $cfg --steps ${STEPS:-50} --warmup 5 --cpu-baseline 0 --cpu-threads 16 \
    --orbit-steps ${ORBIT:-50} --inflight-steps 0 --virtual-ranks 0 --traffic-json /dev/null > $O/bench_$label.log 2>&1
  local rc=$?
  [ $rc -eq 0 ] || { echo "bench $label rc=$rc"; tail -n 5 $O/bench_$label.log; exit $rc; }
  grep '"metric"' $O/bench_$label.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); o=d.get('orbit') or {}; print('$label', round(d['value'],1), 'parity', d.get('parity_vs_oracle'), 'blend_us', round(d['stages_ms']['blend_timed_region']*1e3,1), 'orbit', round(o.get('value',0),1), round((o.get('blend_ms') or 0)*1e3,1), o.get('parity_last_frame'))"
}
for v in ${CFG2_VARIANTS:-}; do  # label:ENV=a,ENV=b
  b ${v%%:*}_cfg2 cfg2_1m_sh3_1080p_f16 $(echo ${v#*:} | tr ',' ' ')
done
b px_cfg2 cfg2_1m_sh3_1080p_f16 GSM_BLEND_PAIRS=0
for v in ${CFG3_VARIANTS:-}; do
  b ${v%%:*}_cfg3 cfg3_5m_sh3_4k_f16 $(echo ${v#*:} | tr ',' ' ')
done
echo done
