set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python tools/exp_graph.py > gpurun_out/exp_graph.log 2>&1; rc=$?; tail -3 gpurun_out/exp_graph.log; echo rc=$rc
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/exp_graph.py --config cfg3_5m_sh3_4k_f16 --frames 20 > gpurun_out/exp_graph4k.log 2>&1; rc=$?; tail -1 gpurun_out/exp_graph4k.log; echo rc=$rc
