set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python tools/blend_trace.py > gpurun_out/trace.log 2>&1; rc=$?; tail -3 gpurun_out/trace.log; echo rc=$rc
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/blend_trace.py --config cfg3_5m_sh3_4k_f16 > gpurun_out/trace4k.log 2>&1; rc=$?; tail -3 gpurun_out/trace4k.log; echo rc=$rc
