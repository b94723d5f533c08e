#!/bin/bash
# r05: PMC of the blend under environment variants (VARIANTS="label:ENV=.. label2:ENV=..", CFG)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/pwp; mkdir -p $O; export TMPDIR=/tmp
cfg=${CFG:-cfg2_1m_sh3_1080p_f16}
for v in ${VARIANTS}; do
  label=${v%%:*}; envs=${v#*:}; envs=${envs//,/ }
  CMD="python bench.py --config $cfg --steps 5 --warmup 2 --cpu-baseline 0 --parity 0 --orbit-steps 0 --inflight-steps 0 --virtual-ranks 0"
  env $envs timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE --output-format csv -d $O/pmc_$label -o p -- $CMD > $O/pmc_$label.log 2>&1 || { echo "pmc $label failed"; tail -3 $O/pmc_$label.log; exit 1; }
  echo "== $label ($envs)"; python tools/pmc_summary.py $O/pmc_$label | grep -A8 "k_blend"
done
