#!/bin/bash
# (the duo walk is not in the product: apply tools/exp/duo_walk.patch to gsm_blend.hip to rebuild it)
# per-unit blend traces of rank 3's slab (config 2, W = 8) with and without duo walks
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/duot; mkdir -p $O gpurun_out; export TMPDIR=/tmp
for e in 0 1; do
  for cfg in ${CFGS:-cfg2_1m_sh3_1080p_f16}; do
    GSM_BLEND_DUO=$e timeout -k 10 300 python tools/exp_virtual_ranks.py --config $cfg --world 8 --frames 3 --trace-rank 3 > $O/vr_${cfg%%_*}_$e.log 2>&1 || { echo "rc=$?"; tail -5 $O/vr_${cfg%%_*}_$e.log; exit 1; }
    mv gpurun_out/vr_trace_${cfg}_w8_r3.npz $O/trace_${cfg%%_*}_$e.npz
    python tools/unit_rates.py $O/trace_${cfg%%_*}_$e.npz
  done
done
