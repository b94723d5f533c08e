#!/bin/bash
# r06: the multi-GPU push (k_part_copy) and its neighbours -- GPU suite on the tree, the virtual-rank
# config-4 frame for HEAD and the tree (three alternating rounds, per-phase and slab-stage times), then
# the same-GPU N-rank rehearsal of bench.py's multi-GPU frame on the tree.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/vrh
export TMPDIR=/tmp
timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc: $(tail -n 1 gpurun_out/pytest_gpu.log)"
[ $rc -eq 0 ] || { grep -E "^FAILED|Error|error" gpurun_out/pytest_gpu.log | head -20; grep -B5 -A60 "^_____" gpurun_out/pytest_gpu.log | head -150; exit $rc; }
for rep in 1 2 3; do
  for v in ${VARIANTS:-head cur}; do
    if [ $v = cur ]; then lib=$PWD/gsm-renderer_amd/lib/libgsm_amd.so; else lib=$PWD/gsm-renderer_amd/lib_ab_$v/libgsm_amd.so; fi
    for cfg in cfg3_5m_sh3_4k_f16 cfg2_1m_sh3_1080p_f16; do
      GSM_AMD_LIB=$lib timeout -k 10 300 python tools/exp_virtual_ranks.py --config $cfg --world 8 --frames 5 \
        > gpurun_out/vrh/${v}_${cfg%%_*}_$rep.log 2>&1 || { echo "vr failed: $v $cfg"; tail -n 5 gpurun_out/vrh/${v}_${cfg%%_*}_$rep.log; exit 1; }
      grep '^{' gpurun_out/vrh/${v}_${cfg%%_*}_$rep.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('vr', '$v', '${cfg%%_*}', d['device_frame_ms'], d['max_phase_ms'], {k: round(max(s[k] for s in d['slab_stages_ms'])*1e3,1) for k in d['slab_stages_ms'][0]})" | tee -a gpurun_out/vrh/summary.txt
    done
  done
done
bash tools/gpu_bench_same_gpu.sh || exit 1
echo "=== done"
