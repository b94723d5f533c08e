#!/bin/bash
# PMC passes (counters only with --kernel-trace/--stats; never with sys/runtime traces).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
# CFG=<bench config> (default config 2), OUT=<dir under gpurun_out> (default pmc), PMC_CMD=<another
# program, e.g. tools/exp_virtual_ranks.py> instead of the bench line
OUT=gpurun_out/${OUT:-pmc}
mkdir -p $OUT
export TMPDIR=/tmp
CMD=${PMC_CMD:-"python bench.py --config ${CFG:-cfg2_1m_sh3_1080p_f16} --steps 5 --warmup 2 --cpu-baseline 0 --parity 0 --orbit-steps 0 --inflight-steps 0 --virtual-ranks 0"}
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM" \
           "FETCH_SIZE" "WRITE_SIZE" "SQ_INSTS_BRANCH SQ_IFETCH SQ_INSTS_SMEM SQ_WAIT_INST_LDS"; do
  i=$((i+1))
  echo "=== pmc pass $i: $set"
  timeout -k 10 300 rocprofv3 --pmc $set --output-format csv -d $OUT/p$i -o p$i -- $CMD > $OUT/p$i.log 2>&1
  rc=$?
  echo "rc=$rc"
  if [ $rc -ne 0 ]; then tail -20 $OUT/p$i.log; [ $i -ge 5 ] && continue; exit $rc; fi
done
python3 tools/pmc_summary.py $OUT > $OUT/summary.txt 2>&1
echo "=== done"
