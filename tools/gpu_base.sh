#!/bin/bash
# Single-GPU baseline of a round: kernel traces of configs 2 and 3 (timelines), then blend PMC passes
# (instruction mix by class, LDS) at config 2.  Each GPU step has its own time limit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T=${TAG:-base}
mkdir -p gpurun_out/$T
for cfg in ${CFGS:-cfg2_1m_sh3_1080p_f16 cfg3_5m_sh3_4k_f16}; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$T/kt_$cfg -o run -- \
    python bench.py --config $cfg --steps 20 --warmup 3 --cpu-baseline 0 --parity 0 --orbit-steps 0 --inflight-steps 0 --virtual-ranks 0 \
    > gpurun_out/$T/kt_$cfg.log 2>&1 || { echo "trace failed $cfg"; tail -5 gpurun_out/$T/kt_$cfg.log; exit 1; }
  echo "== $cfg"; tail -1 gpurun_out/$T/kt_$cfg.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('fps', round(d['value'],1), {k: round(v*1e3,1) for k,v in d['stages_ms'].items()})"
  python3 tools/timeline.py $(find gpurun_out/$T/kt_$cfg -name '*kernel_trace.csv' | head -1) | tee gpurun_out/$T/timeline_$cfg.txt
done
if [ "${PMC:-1}" = "1" ]; then
  i=0
  for set in "SQ_INSTS_VALU_ADD_F16 SQ_INSTS_VALU_MUL_F16 SQ_INSTS_VALU_FMA_F16 SQ_INSTS_VALU_TRANS_F16 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_CVT SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32" \
             "SQ_INSTS_VALU SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_INT64 SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_WAVE_CYCLES GRBM_GUI_ACTIVE" \
             "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_ADDR_CONFLICT SQ_INSTS_SALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_BUSY_CYCLES"; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --pmc $set --output-format csv -d gpurun_out/$T/pmc$i -o p -- \
      python bench.py --steps 5 --warmup 2 --cpu-baseline 0 --parity 0 --orbit-steps 0 --inflight-steps 0 --virtual-ranks 0 > gpurun_out/$T/pmc$i.log 2>&1 || { echo "pmc $i failed"; tail -5 gpurun_out/$T/pmc$i.log; exit 1; }
  done
  python3 tools/pmc_summary.py gpurun_out/$T > gpurun_out/$T/pmc_summary.txt 2>&1; grep -A26 "k_blend" gpurun_out/$T/pmc_summary.txt | head -30
fi
echo "=== done"
