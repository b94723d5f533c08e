set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python tools/exp_frame.py --var GSM_BLEND_SKIP_DYN=0 --var GSM_BLEND_EXITG_DYN=4 --var GSM_BLEND_WG_WAVES_DYN=8,16 --var GSM_BLEND_SCHED_DYN=0,1 > gpurun_out/exp_sens.log 2>&1; rc=$?; grep variant gpurun_out/exp_sens.log; echo exp rc=$rc
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/exp_frame.py --config cfg3_5m_sh3_4k_f16 --rounds 2 --frames 10 --var GSM_BLEND_SKIP_DYN=0 --var GSM_BLEND_EXITG_DYN=4 --var GSM_BLEND_WG_WAVES_DYN=8,16 --var GSM_BLEND_SCHED_DYN=0,1 > gpurun_out/exp_sens4k.log 2>&1; rc=$?; grep variant gpurun_out/exp_sens4k.log; echo exp4k rc=$rc
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -m pytest tests -m gpu -q -x > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_gpu.log; echo pytest rc=$rc
