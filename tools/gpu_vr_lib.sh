#!/bin/bash
# Virtual-rank multi-GPU frames (tools/exp_virtual_ranks.py) for library variants: A = gsm-renderer_amd/lib,
# X = gsm-renderer_amd/lib_X (make BUILD=build_X LIB=lib_X EXTRA=...).  Env: VARIANTS, VR_CASES
# ("cfg:world ...").  Output: gpurun_out/vrlib/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/vrlib
mkdir -p $OUT
export TMPDIR=/tmp
LIBDIR=gsm-renderer_amd/lib
cp $LIBDIR/libgsm_amd.so /tmp/libgsm_amd_A.so
use() { if [ "$1" = A ]; then cp /tmp/libgsm_amd_A.so $LIBDIR/libgsm_amd.so; else cp gsm-renderer_amd/lib_$1/libgsm_amd.so $LIBDIR/libgsm_amd.so; fi; }
for v in A ${VARIANTS:-}; do
  use $v
  for cw in ${VR_CASES:-cfg3_5m_sh3_4k_f16:8 cfg2_1m_sh3_1080p_f16:2 cfg2_1m_sh3_1080p_f16:4 cfg2_1m_sh3_1080p_f16:8}; do
    cfg=${cw%%:*}; w=${cw##*:}
    log=$OUT/${v}_${cfg%%_*}_w$w.log
    timeout -k 10 300 python tools/exp_virtual_ranks.py --config $cfg --world $w --frames 5 > $log 2>&1
    rc=$?; [ $rc -eq 0 ] || { echo "vr failed ($v $cfg $w) rc=$rc"; tail -n 5 $log; use A; exit $rc; }
    grep '^{' $log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', '${cfg%%_*}', 'W=$w', d['device_frame_ms'], d['max_phase_ms'], {k: round(max(s[k] for s in d['slab_stages_ms'])*1e3,1) for k in d['slab_stages_ms'][0]})"
  done
done
use A
