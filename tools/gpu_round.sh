#!/bin/bash
# Round artefacts on one MI355X: GPU parity tests, smoke, PMC passes (blend traffic, VALU count and mix)
# of configs 2, 3 and 5, the bench lines of every single-GPU config, and rocprofv3 kernel-trace
# summaries.  Everything lands in gpurun_out/round/; tools/round_copy.sh TAG copies what is judged
# into profiles/.  Env: TESTS=0 skips the tests, PMC=0 the counter passes, CFGS limits the configs.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/round
mkdir -p $OUT
export TMPDIR=/tmp
step() {  # name timeout cmd...   (stdout+stderr -> $OUT/name.log; crash/timeout ends the script)
  local name=$1 to=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "--- $name rc=$rc"; tail -n 2 "$OUT/$name.log" | cut -c1-400
  if [ $rc -ne 0 ]; then echo "ABORT after $name (rc=$rc)"; exit $rc; fi
}
if [ "${TESTS:-1}" = 1 ]; then
  step pytest_gpu 700 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread
  step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
fi
CFGS=${CFGS:-cfg2_1m_sh3_1080p_f16 cfg3_5m_sh3_4k_f16 cfg5_1m_sh2_stereo_2x1440x1600_f16}
if [ "${PMC:-1}" = 1 ]; then
  for cfg in $CFGS; do
    c=${cfg%%_*}
    kern=k_blend_px; [ $c = cfg5 ] && kern=k_df_blend_eye; [ $c = cfg3 ] && kern=k_blend_pw
    CMD="python bench.py --config $cfg --steps 5 --warmup 2 --cpu-baseline 0 --parity 0 --orbit-steps 0 --inflight-steps 0 --virtual-ranks 0"
    i=0
    for set in "FETCH_SIZE" "WRITE_SIZE" \
               "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE" \
               "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM" \
               "SQ_INSTS_VALU_ADD_F16 SQ_INSTS_VALU_MUL_F16 SQ_INSTS_VALU_FMA_F16 SQ_INSTS_VALU_TRANS_F16 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_CVT SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32" \
               "SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_INT64 SQ_THREAD_CYCLES_VALU"; do
      i=$((i+1))
      step pmc_${c}_$i 180 rocprofv3 --pmc $set --output-format csv -d $OUT/pmc_$c/p$i -o p$i -- $CMD
    done
    python tools/pmc_summary.py $OUT/pmc_$c > $OUT/pmc_summary_$c.txt
    python tools/traffic.py $OUT/pmc_$c $kern $cfg > $OUT/pmc_blend_$c.json
    cat $OUT/pmc_blend_$c.json
  done
fi
for cfg in $CFGS; do
  c=${cfg%%_*}
  step bench_$c 600 python bench.py --config $cfg --traffic-json $OUT/pmc_blend_$c.json
  [ $c = cfg5 ] && step bench_${c}_global 600 python bench.py --config $cfg --stereo-path global --cpu-baseline 0 \
       --traffic-json /dev/null
  step kt_$c 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt_$c -o run -- \
       python bench.py --config $cfg --steps 50 --warmup 5 --cpu-baseline 0 --parity 0 --orbit-steps 0 --inflight-steps 0 --virtual-ranks 0
done
echo "=== done"
