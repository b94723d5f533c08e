#!/bin/bash
# r05 session A: new multi-GPU tests, per-unit blend traces (configs 2 / 3, static and orbit), the
# alive-curve statistics build (lib_z2), the uncached-memory diagnosis.  Every GPU step time-limited.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05; mkdir -p $O; export TMPDIR=/tmp
st() { local n=$1 t=$2; shift 2; timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?; echo "$n rc=$rc: $(tail -n 1 $O/$n.log)"; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi; }
st trace_cfg2_0 120 python tools/blend_trace.py
st trace_cfg2_13 120 python tools/blend_trace.py --angle 13.75
st trace_cfg3_0 200 python tools/blend_trace.py --config cfg3_5m_sh3_4k_f16
st mg_uncached_diag 300 python -u tools/exp/mg_uncached_diag.py 2
echo done
