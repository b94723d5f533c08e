#!/bin/bash
# A/B of the blend queue claim point (GSM_BLEND_CLAIM=early|late|auto): bench lines (parity, orbit)
# of configs 2 and 3, and the 4K slab blend of 8 virtual ranks.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/claim; mkdir -p $OUT; export TMPDIR=/tmp
for m in early late auto; do
  for cfg in ${CFGS:-cfg2_1m_sh3_1080p_f16 cfg3_5m_sh3_4k_f16}; do
    GSM_BLEND_CLAIM=$m timeout -k 10 300 python bench.py --config $cfg --steps 50 --warmup 5 --cpu-baseline 0 \
      --orbit-steps 50 --inflight-steps 0 --traffic-json /dev/null > $OUT/bench_${m}_$cfg.log 2>&1 || { echo "bench failed $m $cfg"; tail -n 5 $OUT/bench_${m}_$cfg.log; exit 1; }
    grep '"metric"' $OUT/bench_${m}_$cfg.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$m $cfg', round(d['value'],1), 'orbit', round(d['orbit']['value'],1), 'parity', d.get('parity_vs_oracle'), d['orbit'].get('parity_last_frame'), 'blend', round(d['stages_ms']['blend']*1e3,1))"
  done
  if [ "${VR:-1}" = 1 ]; then
    GSM_BLEND_CLAIM=$m timeout -k 10 300 python tools/exp_virtual_ranks.py --config cfg3_5m_sh3_4k_f16 --world 8 --frames 5 --trace-rank 7 \
      > $OUT/vr_$m.log 2>&1 || { echo "vr failed $m"; tail -n 5 $OUT/vr_$m.log; exit 1; }
    python3 -c "
import json; d=json.loads(open('$OUT/vr_$m.log').read().strip().splitlines()[-1])
print('$m vr device', d['device_frame_ms'], 'phases', d['max_phase_ms'], 'blend', [s['blend'] for s in d['slab_stages_ms']], 'trace', {k: d['blend_trace'][k] for k in ['span_us','max_unit_us','sum_unit_us']})"
  fi
done
echo "=== done"
