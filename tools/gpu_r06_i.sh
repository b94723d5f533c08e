#!/bin/bash
# r06: the config-4 slab blend (2025 tiles: quadrant units, P = 1) against half tiles (P = 2) -- virtual-rank frames,
# three alternating rounds (GSM_AB_P1TILES: tiles per CU up to which the blend takes quadrant units).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/vri
export TMPDIR=/tmp
for rep in 1 2 3; do
  for p1 in 8 4; do
    GSM_AB_P1TILES=$p1 timeout -k 10 300 python tools/exp_virtual_ranks.py --config cfg3_5m_sh3_4k_f16 --world 8 --frames 5 \
      > gpurun_out/vri/p${p1}_$rep.log 2>&1 || { echo "vr failed: $p1"; tail -n 5 gpurun_out/vri/p${p1}_$rep.log; exit 1; }
    grep '^{' gpurun_out/vri/p${p1}_$rep.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('vr p1tiles=$p1', d['device_frame_ms'], d['max_phase_ms'], {k: round(max(s[k] for s in d['slab_stages_ms'])*1e3,1) for k in d['slab_stages_ms'][0]})" | tee -a gpurun_out/vri/summary.txt
  done
done
echo "=== done"
