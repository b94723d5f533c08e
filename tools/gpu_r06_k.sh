#!/bin/bash
# r06: the records path's fused scan (multi-GPU slabs) -- the multi-GPU GPU tests on the tree, then the
# virtual-rank frames of configs 4 and 2 for HEAD and the tree, three alternating rounds.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
rm -rf gpurun_out/vrk && mkdir -p gpurun_out/vrk
export TMPDIR=/tmp
if [ "${TESTS:-1}" = 1 ]; then
  timeout -k 10 700 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_multigpu_ipc.py tests/test_multigpu_rccl.py tests/test_gpu_parity.py -k "multigpu or virtual or processes or config4 or partition or rccl or records or fused or scan" > gpurun_out/vrk/pytest.log 2>&1
  rc=$?; echo "pytest rc=$rc: $(tail -n 1 gpurun_out/vrk/pytest.log)"; [ $rc -eq 0 ] || { tail -30 gpurun_out/vrk/pytest.log; exit $rc; }
fi
for rep in 1 2 3; do
  for v in head cur; do
    if [ $v = cur ]; then lib=$PWD/gsm-renderer_amd/lib/libgsm_amd.so; else lib=$PWD/gsm-renderer_amd/lib_ab_$v/libgsm_amd.so; fi
    for cfg in cfg3_5m_sh3_4k_f16 cfg2_1m_sh3_1080p_f16; do
      GSM_AMD_LIB=$lib timeout -k 10 300 python tools/exp_virtual_ranks.py --config $cfg --world 8 --frames 5 \
        > gpurun_out/vrk/${v}_${cfg%%_*}_$rep.log 2>&1 || { echo "vr failed: $v $cfg"; tail -n 5 gpurun_out/vrk/${v}_${cfg%%_*}_$rep.log; exit 1; }
      grep '^{' gpurun_out/vrk/${v}_${cfg%%_*}_$rep.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('vr', '$v', '${cfg%%_*}', d['device_frame_ms'], d['max_phase_ms'], {k: round(max(s[k] for s in d['slab_stages_ms'])*1e3,1) for k in d['slab_stages_ms'][0]})" | tee -a gpurun_out/vrk/summary.txt
    done
  done
done
echo "=== done"
