#!/bin/bash
# Virtual-rank multi-GPU frame (tools/exp_virtual_ranks.py) under create-time env variants.
# Env: VR_ENVS="default GSM_BLEND_WAVES=16 ..." (each a space-free NAME=VALUE or "default"),
# VR_CFGS, VR_WORLD.  Output: gpurun_out/vrenv/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/vrenv
mkdir -p $OUT
export TMPDIR=/tmp
for e in ${VR_ENVS:-default}; do
  for cfg in ${VR_CFGS:-cfg3_5m_sh3_4k_f16 cfg2_1m_sh3_1080p_f16}; do
    log=$OUT/${cfg%%_*}_${e//=/-}.log
    if [ "$e" = default ]; then
      timeout -k 10 300 python tools/exp_virtual_ranks.py --config $cfg --world ${VR_WORLD:-8} --frames 5 > $log 2>&1
    else
      timeout -k 10 300 env $e python tools/exp_virtual_ranks.py --config $cfg --world ${VR_WORLD:-8} --frames 5 > $log 2>&1
    fi
    rc=$?; [ $rc -eq 0 ] || { echo "vr failed ($e $cfg) rc=$rc"; tail -n 5 $log; exit $rc; }
    grep '^{' $log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$e', '${cfg%%_*}', d['device_frame_ms'], d['max_phase_ms'], {k: round(max(s[k] for s in d['slab_stages_ms'])*1e3,1) for k in d['slab_stages_ms'][0]})"
  done
done
