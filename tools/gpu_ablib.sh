#!/bin/bash
# A/B of compile-time library variants on one MI355X.  Variant A is gsm-renderer_amd/lib (the
# default build); variant X is gsm-renderer_amd/lib_X (make BUILD=build_X LIB=lib_X EXTRA=...).
# Env: TESTS=1 runs the GPU tests on A first (and on every variant with TESTS=all); VARIANTS="b c";
# CFGS.  Per variant and config: a rocprofv3 kernel-trace summary and the bench line (parity on),
# into gpurun_out/ab/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/ab
mkdir -p $OUT
export TMPDIR=/tmp
LIBDIR=gsm-renderer_amd/lib
cp $LIBDIR/libgsm_amd.so /tmp/libgsm_amd_A.so
use() { if [ "$1" = A ]; then cp /tmp/libgsm_amd_A.so $LIBDIR/libgsm_amd.so; else cp gsm-renderer_amd/lib_$1/libgsm_amd.so $LIBDIR/libgsm_amd.so; fi; }
for v in A ${VARIANTS:-}; do
  use $v
  if [ "${TESTS:-1}" = all ] || { [ "${TESTS:-1}" = 1 ] && [ $v = A ]; }; then
    timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest_$v.log 2>&1
    rc=$?; echo "pytest $v rc=$rc: $(tail -n 1 $OUT/pytest_$v.log)"
    [ $rc -eq 0 ] || { tail -n 30 $OUT/pytest_$v.log; use A; exit $rc; }
  fi
  for cfg in ${CFGS:-cfg2_1m_sh3_1080p_f16 cfg3_5m_sh3_4k_f16}; do
    rm -rf $OUT/kt_${v}_$cfg
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt_${v}_$cfg -o run -- \
      python bench.py --config $cfg --steps 20 --warmup 3 --cpu-baseline 0 --parity 0 --orbit-steps 0 --inflight-steps 0 --virtual-ranks 0 \
      > $OUT/kt_${v}_$cfg.log 2>&1 || { echo "rocprof failed: $v $cfg"; tail -n 5 $OUT/kt_${v}_$cfg.log; use A; exit 1; }
    f=$(find $OUT/kt_${v}_$cfg -name '*kernel_stats.csv' | head -n 1)
    python3 - "$f" "$v $cfg" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
print(sys.argv[2])
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:12]:
    print(f"  {r['Name'].split('(')[0][:52]:52s} calls={int(r['Calls']):5d} avg_us={float(r['AverageNs'])/1e3:8.1f}")
PY
    timeout -k 10 300 python bench.py --config $cfg --steps 50 --warmup 5 --cpu-baseline 0 --orbit-steps ${ORBIT:-0} --virtual-ranks 0 \
      --traffic-json /dev/null > $OUT/bench_${v}_$cfg.log 2>&1 || { echo "bench failed: $v $cfg"; tail -n 5 $OUT/bench_${v}_$cfg.log; use A; exit 1; }
    grep '"metric"' $OUT/bench_${v}_$cfg.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('  bench', '$v', round(d['value'],1), 'parity', d.get('parity_vs_oracle'), 'inflight2', (d.get('inflight2') or {}).get('value'), (d.get('inflight2') or {}).get('parity_both_targets'), {k: round(x*1e3,1) for k,x in d['stages_ms'].items()})"
  done
  if [ "${VR:-0}" = 1 ]; then  # virtual-rank multi-GPU frame (config 4: 5M / 4K / 8 ranks)
    timeout -k 10 300 python tools/exp_virtual_ranks.py --config cfg3_5m_sh3_4k_f16 --world 8 --frames 5 \
      > $OUT/vr_$v.log 2>&1 || { echo "vr failed: $v"; tail -n 5 $OUT/vr_$v.log; use A; exit 1; }
    grep '^{' $OUT/vr_$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('  vr', '$v', d['device_frame_ms'], d['max_phase_ms'], {k: round(max(s[k] for s in d['slab_stages_ms'])*1e3,1) for k in d['slab_stages_ms'][0]})"
  fi
done
use A
echo "=== done"
