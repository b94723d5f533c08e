#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/vrw; export TMPDIR=/tmp
for w in 0 8 16; do
  GSM_BLEND_WAVES=$w timeout -k 10 300 python tools/exp_virtual_ranks.py --config cfg3_5m_sh3_4k_f16 --world 8 --frames 5 > gpurun_out/vrw/w$w.log 2>&1 || { echo fail; tail -5 gpurun_out/vrw/w$w.log; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/vrw/w$w.log').read().strip().splitlines()[-1])
print('waves=$w device', d['device_frame_ms'], 'max phases', d['max_phase_ms'], 'blend', [s['blend'] for s in d['slab_stages_ms']], 'sort', [s['sort'] for s in d['slab_stages_ms']])"
done
