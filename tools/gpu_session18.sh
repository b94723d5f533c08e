set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -q -x -k "golden or full_size or partition" > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_gpu.log; echo pytest rc=$rc
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python tools/exp_frame.py --var GSM_BLEND_PRIO=1,0 > gpurun_out/exp18.log 2>&1; rc=$?; grep variant gpurun_out/exp18.log; echo exp rc=$rc
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/exp_frame.py --config cfg3_5m_sh3_4k_f16 --rounds 2 --frames 10 --var GSM_BLEND_PRIO=1,0 > gpurun_out/exp18_4k.log 2>&1; rc=$?; grep variant gpurun_out/exp18_4k.log; echo exp4k rc=$rc
