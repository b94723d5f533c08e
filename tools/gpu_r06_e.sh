#!/bin/bash
# r06: GPU suite on the working tree, then kernel traces of configs 2 / 3 for HEAD against the tree
# (tools/build_ab.sh head), then the config-4 virtual-rank frame for both (one run each, alternating twice).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc: $(tail -n 1 gpurun_out/pytest_gpu.log)"
[ $rc -eq 0 ] || { grep -E "^FAILED|Error|error" gpurun_out/pytest_gpu.log | head -20; grep -B5 -A60 "^_____" gpurun_out/pytest_gpu.log | head -150; exit $rc; }
VARIANTS="${VARIANTS:-head cur}" REPS=2 bash tools/gpu_ab_proj.sh || exit 1
for rep in 1 2; do
  for v in ${VARIANTS:-head cur}; do
    if [ $v = cur ]; then lib=$PWD/gsm-renderer_amd/lib/libgsm_amd.so; else lib=$PWD/gsm-renderer_amd/lib_ab_$v/libgsm_amd.so; fi
    GSM_AMD_LIB=$lib timeout -k 10 300 python tools/exp_virtual_ranks.py --frames 5 --stages 0 --single 0 > gpurun_out/vr_${v}_$rep.log 2>&1 || { echo "vr $v failed"; tail -5 gpurun_out/vr_${v}_$rep.log; exit 1; }
    python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(sys.argv[2], d['device_frame_ms'], d['max_phase_ms'], d['timeouts'])" gpurun_out/vr_${v}_$rep.log ${v}_$rep
  done
done
# the slab blend's waves per CU (GSM_BLEND_WAVES, create-time) on the virtual-rank frame
for wv in 16 8; do
  GSM_BLEND_WAVES=$wv timeout -k 10 300 python tools/exp_virtual_ranks.py --frames 5 --stages 1 --single 0 > gpurun_out/vr_w$wv.log 2>&1 || { echo "vr w$wv failed"; tail -5 gpurun_out/vr_w$wv.log; exit 1; }
  python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(sys.argv[2], d['device_frame_ms'], d['max_phase_ms'], [s['blend'] for s in d['slab_stages_ms'] if s])" gpurun_out/vr_w$wv.log waves$wv
done
echo "=== done"
