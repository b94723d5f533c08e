#!/bin/bash
# (the duo walk is not in the product: apply tools/exp/duo_walk.patch to gsm_blend.hip to rebuild it)
# r05: duo walks (producer/consumer wave pairs for the quadrant kernel's longest units, GSM_BLEND_DUO)
# -- GPU parity tests, then the virtual-rank frame (config 4 and config 2 at W = 8) with and without,
# twice interleaved, and the single-GPU bench line of config 2 (not a quadrant frame: unchanged).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/duo; mkdir -p $O; export TMPDIR=/tmp
if [ "${TESTS:-1}" = 1 ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
  rc=$?; echo "pytest rc=$rc: $(tail -n 1 $O/pytest.log)"
  [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/pytest.log | head -20; exit $rc; }
fi
for r in 1 2; do
  for e in GSM_BLEND_DUO=0 GSM_BLEND_DUO=1; do
    for cfg in cfg3_5m_sh3_4k_f16 cfg2_1m_sh3_1080p_f16; do
      log=$O/vr_${cfg%%_*}_${e#*=}_$r.log
      timeout -k 10 300 env $e python tools/exp_virtual_ranks.py --config $cfg --world 8 --frames 5 > $log 2>&1
      rc=$?; [ $rc -eq 0 ] || { echo "vr failed ($e $cfg) rc=$rc"; tail -n 5 $log; exit $rc; }
      grep '^{' $log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$e', '${cfg%%_*}', d['device_frame_ms'], d['max_phase_ms'], {k: round(max(s[k] for s in d['slab_stages_ms'])*1e3,1) for k in d['slab_stages_ms'][0]})"
    done
  done
done
echo done
