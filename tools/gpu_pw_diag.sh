#!/bin/bash
# r05: pair-walk diagnosis -- per-unit traces of config 2 with and without pairs, and one PMC pass each
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/pwd; mkdir -p $O; export TMPDIR=/tmp
for v in 1 0; do
  GSM_BLEND_PAIRS=$v timeout -k 10 120 python tools/blend_trace.py > $O/trace_cfg2_p$v.txt 2>&1 || { echo "trace $v failed"; tail -3 $O/trace_cfg2_p$v.txt; exit 1; }
  mv gpurun_out/blend_trace_cfg2_1m_sh3_1080p_f16_0.npz $O/trace_cfg2_p$v.npz
  tail -n 1 $O/trace_cfg2_p$v.txt
  CMD="python bench.py --config cfg2_1m_sh3_1080p_f16 --steps 5 --warmup 2 --cpu-baseline 0 --parity 0 --orbit-steps 0 --inflight-steps 0 --virtual-ranks 0"
  GSM_BLEND_PAIRS=$v timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE --output-format csv -d $O/pmc_p$v -o p -- $CMD > $O/pmc_p$v.log 2>&1 || { echo "pmc $v failed"; tail -3 $O/pmc_p$v.log; exit 1; }
  python tools/pmc_summary.py $O/pmc_p$v | grep -A9 "blend" 
done
echo done
