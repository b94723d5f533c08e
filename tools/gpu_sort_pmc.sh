#!/bin/bash
# r06: memory-side counters of the two 4K tile passes (k_radix_upsweep<7> /
# k_radix_downsweep<7, *, false|true>) at config 3, one rocprofv3 --pmc pass per counter group (the
# hardware's per-block limits), summarised per kernel into gpurun_out/sort_pmc/summary.txt.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
CFG=${CFG:-cfg3_5m_sh3_4k_f16}
OUT=gpurun_out/sort_pmc
rm -rf $OUT && mkdir -p $OUT
i=0
while read -r counters; do
  [ -z "$counters" ] && continue
  i=$((i + 1))
  timeout -s KILL 120 rocprofv3 --pmc $counters --output-format csv -d $OUT/p$i -o p -- \
    python bench.py --config $CFG --steps 5 --warmup 2 --cpu-baseline 0 --parity 0 --orbit-steps 0 --inflight-steps 0 \
    --virtual-ranks 0 > $OUT/p$i.log 2>&1 || { echo "pmc pass $i failed ($counters)"; tail -5 $OUT/p$i.log; exit 1; }
  echo "pass $i ok: $counters"
done <<'EOF'
FETCH_SIZE TCC_EA0_RDREQ_DRAM_sum
WRITE_SIZE TCC_EA0_WRREQ_DRAM_sum TCC_EA0_WRREQ_STALL_sum
TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_STALL_MULTI_MISS_sum TCP_PENDING_STALL_CYCLES_sum
TCC_HIT_sum TCC_MISS_sum TCC_TAG_STALL_sum TCC_EA0_RDREQ_sum
TCP_TCC_WRITE_REQ_LATENCY_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_WRITE_REQ_sum TCP_TCC_READ_REQ_sum
SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE
EOF
python3 tools/pmc_summary.py $OUT > $OUT/summary.txt
grep -A40 -E "^void gsm::k_radix|^gsm::k_scatter" $OUT/summary.txt | head -150
echo "=== done"
