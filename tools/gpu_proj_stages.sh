#!/bin/bash
# Stage attribution of k_project: kernel traces of the GSM_PROJ_STOP builds
# (gsm-renderer_amd/lib_ps<k>, tools/build_proj_stages.sh) at configs 2 and 3, one PMC pass per build at
# config 2, and the VALU issue probe (tools/exp/valu_peak).  Output: gpurun_out/ps/.  SCHED=0 runs every
# build with GSM_BLEND_SCHED=0: no blend-schedule workgroup in the projection launch (block 0, which
# otherwise sets a floor under the truncated builds' duration).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
[ "${SCHED:-1}" = 0 ] && export GSM_BLEND_SCHED=0
OUT=gpurun_out/${OUTDIR:-ps}
mkdir -p $OUT
LIBDIR=gsm-renderer_amd/lib
cp $LIBDIR/libgsm_amd.so /tmp/libgsm_amd_A.so
use() { if [ "$1" = A ]; then cp /tmp/libgsm_amd_A.so $LIBDIR/libgsm_amd.so; else cp gsm-renderer_amd/lib_$1/libgsm_amd.so $LIBDIR/libgsm_amd.so; fi; }
if [ "${PEAK:-1}" = 1 ]; then
  timeout -k 10 240 tools/exp/valu_peak > $OUT/valu_peak.txt 2>&1 || { echo "valu_peak failed"; tail -5 $OUT/valu_peak.txt; exit 1; }
  echo "valu_peak done"
fi
BENCH="bench.py --steps 20 --warmup 3 --cpu-baseline 0 --parity 0 --orbit-steps 0 --inflight-steps 0 --virtual-ranks 0"
for v in A ${VARIANTS:-ps1 ps2 ps3 ps4 ps5 ps6 ps7 ps8}; do
  use $v
  for cfg in ${CFGS:-cfg2_1m_sh3_1080p_f16 cfg3_5m_sh3_4k_f16}; do
    c=${cfg%%_*}
    rm -rf $OUT/kt_${v}_$c
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt_${v}_$c -o run -- \
      python $BENCH --config $cfg > $OUT/kt_${v}_$c.log 2>&1 || { echo "kt failed $v $c"; tail -5 $OUT/kt_${v}_$c.log; use A; exit 1; }
    f=$(find $OUT/kt_${v}_$c -name '*kernel_stats.csv' | head -n 1)
    python3 - "$f" "$v $c" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows:
    if r['Name'].startswith('void gsm::k_project<'):
        print(f"{sys.argv[2]:12s} {r['Name'].split('(')[0]:34s} calls={int(r['Calls']):4d} avg_us={float(r['AverageNs'])/1e3:7.2f} min_us={float(r['MinNs'])/1e3:7.2f}")
PY
  done
  if [ "${PMC:-1}" = 1 ]; then
    timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE \
      --output-format csv -d $OUT/pmc_$v -o p -- python bench.py --steps 5 --warmup 2 --cpu-baseline 0 --parity 0 --orbit-steps 0 --inflight-steps 0 --virtual-ranks 0 \
      > $OUT/pmc_$v.log 2>&1 || { echo "pmc failed $v"; tail -5 $OUT/pmc_$v.log; use A; exit 1; }
    python3 tools/pmc_summary.py $OUT/pmc_$v | grep -A9 "k_project<true, 3>" > $OUT/pmc_$v.txt
    echo "pmc $v: $(tr -s ' ' < $OUT/pmc_$v.txt | grep -E 'INSTS_VALU|WAIT_INST|WAVE_CYCLES' | cut -c1-60 | tr '\n' ';')"
  fi
done
use A
echo "=== done"
