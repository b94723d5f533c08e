#!/bin/bash
# A/B of blend waves per workgroup (GSM_BLEND_WAVES=8|12|16; 0 = by frame size) on the bench lines.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/waves; mkdir -p $OUT; export TMPDIR=/tmp
for cfg in ${CFGS:-cfg2_1m_sh3_1080p_f16 cfg3_5m_sh3_4k_f16}; do
  for w in ${WAVES:-0 8 12 16}; do
    extra=""; [ "${cfg%%_*}" = cfg5 ] && extra="--stereo-path global"
    GSM_BLEND_WAVES=$w timeout -k 10 300 python bench.py --config $cfg $extra --steps 50 --warmup 5 --cpu-baseline 0 \
      --orbit-steps ${ORBIT:-50} --inflight-steps 0 --traffic-json /dev/null > $OUT/bench_${w}_$cfg.log 2>&1 || { echo "bench failed $w $cfg"; tail -n 5 $OUT/bench_${w}_$cfg.log; exit 1; }
    grep '"metric"' $OUT/bench_${w}_$cfg.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); o=d.get('orbit') or {}; print('waves=$w $cfg', round(d['value'],1), 'orbit', round(o.get('value',0),1), 'parity', d.get('parity_vs_oracle'), o.get('parity_last_frame'), 'blend', round(d['stages_ms']['blend']*1e3,1))"
  done
done
echo "=== done"
