#!/bin/bash
# Blend LDS attribution / A/B of compile-time blend variants (lib_X built with make BUILD=build_X
# LIB=lib_X EXTRA=-D...): per variant and config one PMC pass of the LDS counters on the blend and a
# bench line (static + orbit, parity on), into gpurun_out/lds/.  VARIANTS="b c", CFGS, TESTS=X runs the
# GPU suite on variant X at the end.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/lds
mkdir -p $OUT
export TMPDIR=/tmp
LIBDIR=gsm-renderer_amd/lib
cp $LIBDIR/libgsm_amd.so /tmp/libgsm_amd_A.so
use() { if [ "$1" = A ]; then cp /tmp/libgsm_amd_A.so $LIBDIR/libgsm_amd.so; else cp gsm-renderer_amd/lib_$1/libgsm_amd.so $LIBDIR/libgsm_amd.so; fi; }
CTR="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VALU SQ_WAVES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
for v in ${VARIANTS:-A}; do
  use $v
  for cfg in ${CFGS:-cfg2_1m_sh3_1080p_f16}; do
    CMD="python bench.py --config $cfg --steps 5 --warmup 2 --cpu-baseline 0 --parity 0 --orbit-steps ${PMC_ORBIT:-0} --inflight-steps 0 --virtual-ranks 0"
    rm -rf $OUT/pmc_${v}_$cfg
    timeout -s KILL 120 rocprofv3 --pmc $CTR --output-format csv -d $OUT/pmc_${v}_$cfg -o p -- $CMD > $OUT/pmc_${v}_$cfg.log 2>&1 \
      || { echo "pmc failed: $v $cfg"; tail -n 5 $OUT/pmc_${v}_$cfg.log; use A; exit 1; }
    python3 - $OUT/pmc_${v}_$cfg "$v $cfg" <<'PY'
import csv, glob, os, sys
from collections import defaultdict
acc = defaultdict(lambda: defaultdict(list))
for p in glob.glob(os.path.join(sys.argv[1], "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(p)):
        acc[r["Kernel_Name"].split("(")[0]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, cs in acc.items():
    if "blend" not in k:
        continue
    m = {c: sum(v) / len(v) for c, v in cs.items()}
    bc, act = m.get("SQ_LDS_BANK_CONFLICT", 0), m.get("SQ_LDS_IDX_ACTIVE", 1)
    print(f"  {sys.argv[2]} {k[:40]}: conflict {bc/1e6:.2f}M / active {act/1e6:.2f}M = {bc/act:.3f}; "
          f"LDS insts {m.get('SQ_INSTS_LDS',0)/1e6:.2f}M VALU {m.get('SQ_INSTS_VALU',0)/1e6:.2f}M waves {m.get('SQ_WAVES',0):.0f}")
PY
    timeout -k 10 300 python bench.py --config $cfg --steps 50 --warmup 5 --cpu-baseline 0 --cpu-threads 16 --orbit-steps ${ORBIT:-50} \
      --inflight-steps 0 --virtual-ranks 0 --traffic-json /dev/null > $OUT/bench_${v}_$cfg.log 2>&1 \
      || { echo "bench failed: $v $cfg"; tail -n 5 $OUT/bench_${v}_$cfg.log; use A; exit 1; }
    grep '"metric"' $OUT/bench_${v}_$cfg.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); o=d.get('orbit') or {}; print('  bench', '$v', '$cfg', round(d['value'],1), 'parity', d.get('parity_vs_oracle'), 'blend_us', round(d['stages_ms']['blend_timed_region']*1e3,1), 'orbit', round(o.get('value',0),1), o.get('blend_ms'), o.get('parity_last_frame'))"
  done
done
if [ -n "${TESTS:-}" ]; then
  use $TESTS
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest_$TESTS.log 2>&1
  rc=$?; echo "pytest $TESTS rc=$rc: $(tail -n 1 $OUT/pytest_$TESTS.log)"
  use A
  [ $rc -eq 0 ] || { tail -n 30 $OUT/pytest_$TESTS.log; exit $rc; }
fi
use A
echo "=== done"
