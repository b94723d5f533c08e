#!/bin/bash
# PMC passes over the DepthFirst stereo bench (config 5): VALU/LDS instruction counts and LDS
# conflicts of k_df_blend_eye.  Counters only with --kernel-trace/--stats-free runs.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/dfpmc
mkdir -p $OUT
export TMPDIR=/tmp
CMD="python bench.py --config cfg5_1m_sh2_stereo_2x1440x1600_f16 --steps 5 --warmup 2 --cpu-baseline 0 --parity 0"
i=0
for set in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM SQ_WAIT_INST_LDS"; do
  i=$((i+1))
  echo "=== pmc pass $i"
  timeout -k 10 -s KILL 120 rocprofv3 --pmc $set --output-format csv -d $OUT/p$i -o p$i -- $CMD > $OUT/p$i.log 2>&1
  rc=$?
  echo "rc=$rc"
  if [ $rc -ne 0 ]; then tail -20 $OUT/p$i.log; exit $rc; fi
done
python tools/pmc_summary.py $OUT > $OUT/pmc_summary.txt
grep -A18 "k_df_blend" $OUT/pmc_summary.txt
python tools/traffic.py $OUT k_df_blend_eye cfg5_1m_sh2_stereo_2x1440x1600_f16 > $OUT/traffic_cfg5.json
cat $OUT/traffic_cfg5.json
