#!/bin/bash
# r06: the blend's claim point (GSM_BLEND_CLAIM late = default, auto = one batch before last frame's walk
# ends) after the latency pass -- kernel traces of configs 2 / 3 and the virtual-rank config-4 frame, two
# alternating rounds.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/claim
rm -rf $OUT && mkdir -p $OUT
for rep in 1 2; do
  for cl in late auto; do
    for cfg in cfg2_1m_sh3_1080p_f16 cfg3_5m_sh3_4k_f16; do
      label=${cl}_${cfg%%_*}_r$rep
      GSM_BLEND_CLAIM=$cl timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$label -o run -- \
        python bench.py --config $cfg --steps 20 --warmup 3 --cpu-baseline 0 --parity 1 --orbit-steps 20 --inflight-steps 0 \
        --virtual-ranks 0 > $OUT/$label.log 2>&1 || { echo "run $label failed"; tail -5 $OUT/$label.log; exit 1; }
      f=$(find $OUT/$label -name '*kernel_stats.csv' | head -1)
      python3 - "$f" "$label" "$OUT/$label.log" <<'PY' | tee -a $OUT/summary.txt
import csv, sys, json
rows = {r["Name"].split("(")[0]: float(r["AverageNs"]) / 1e3 for r in csv.DictReader(open(sys.argv[1]))}
b = next((v for k, v in rows.items() if "k_blend" in k), float("nan"))
d = next(json.loads(l) for l in open(sys.argv[3]) if l.startswith("{") and '"metric"' in l)
print(f"{sys.argv[2]:18s} blend {b:6.1f}  fps {d['value']:7.1f}  orbit {d['orbit']['value']:7.1f}  parity {d.get('parity_vs_oracle')} {d['orbit'].get('parity_last_frame')}")
PY
    done
    GSM_BLEND_CLAIM=$cl timeout -k 10 300 python tools/exp_virtual_ranks.py --config cfg3_5m_sh3_4k_f16 --world 8 --frames 5 \
      > $OUT/vr_${cl}_$rep.log 2>&1 || { echo "vr failed: $cl"; tail -n 5 $OUT/vr_${cl}_$rep.log; exit 1; }
    grep '^{' $OUT/vr_${cl}_$rep.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('vr $cl', d['device_frame_ms'], d['max_phase_ms'], {k: round(max(s[k] for s in d['slab_stages_ms'])*1e3,1) for k in d['slab_stages_ms'][0]})" | tee -a $OUT/summary.txt
  done
done
echo "=== done"
