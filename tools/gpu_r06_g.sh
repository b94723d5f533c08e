#!/bin/bash
# r06: unpredicated loads (Tail4) -- GPU suite on the tree, kernel traces of configs 2 / 3 / 5 for HEAD
# against the tree (two alternating rounds), then the virtual-rank config-4 frame for both libraries.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc: $(tail -n 1 gpurun_out/pytest_gpu.log)"
[ $rc -eq 0 ] || { grep -E "^FAILED|Error|error" gpurun_out/pytest_gpu.log | head -20; grep -B5 -A60 "^_____" gpurun_out/pytest_gpu.log | head -150; exit $rc; }
VARIANTS="${VARIANTS:-head cur}" REPS=2 CFGS="cfg2_1m_sh3_1080p_f16 cfg3_5m_sh3_4k_f16 cfg5_1m_sh2_stereo_2x1440x1600_f16" bash tools/gpu_ab_proj.sh || exit 1
for rep in 1 2; do
  for v in ${VARIANTS:-head cur}; do
    if [ $v = cur ]; then lib=$PWD/gsm-renderer_amd/lib/libgsm_amd.so; else lib=$PWD/gsm-renderer_amd/lib_ab_$v/libgsm_amd.so; fi
    GSM_AMD_LIB=$lib timeout -k 10 300 python tools/exp_virtual_ranks.py --config cfg3_5m_sh3_4k_f16 --world 8 --frames 5 \
      > gpurun_out/vr_${v}_$rep.log 2>&1 || { echo "vr failed: $v"; tail -n 5 gpurun_out/vr_${v}_$rep.log; exit 1; }
    grep '^{' gpurun_out/vr_${v}_$rep.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('  vr', '$v', d['device_frame_ms'], d.get('device_speedup'), d['max_phase_ms'], {k: round(max(s[k] for s in d['slab_stages_ms'])*1e3,1) for k in d['slab_stages_ms'][0]})" | tee -a gpurun_out/abp/summary.txt
  done
done
echo "=== done"
