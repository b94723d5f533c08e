#!/bin/bash
# FETCH_SIZE / WRITE_SIZE / SQ_INSTS_VALU of the blend for one config (default config 2), one pass each.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
cfg=${CFG:-cfg2_1m_sh3_1080p_f16}
kern=${KERN:-k_blend_px}
OUT=gpurun_out/pmcq
rm -rf $OUT; mkdir -p $OUT
CMD="python bench.py --config $cfg --steps 5 --warmup 2 --cpu-baseline 0 --parity 0 --orbit-steps 0 --inflight-steps 0 --virtual-ranks 0"
i=0
for set in FETCH_SIZE WRITE_SIZE "SQ_INSTS_VALU SQ_WAVES GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set --output-format csv -d $OUT/p$i -o p$i -- $CMD > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $OUT/p$i.log; exit 1; }
done
python tools/traffic.py $OUT $kern $cfg
