set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -q -x > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_gpu.log; echo pytest rc=$rc
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python tools/exp_frame.py --var GSM_BLEND_SKIP_DYN=1,0 --var GSM_BLEND_EXITG_DYN=1,2,4 --var GSM_BLEND_WG_WAVES_DYN=16,8 > gpurun_out/exp.log 2>&1; rc=$?; grep variant gpurun_out/exp.log; echo exp rc=$rc
[ $rc -eq 0 ] || exit $rc
bash tools/gpu_trace.sh
timeout -k 10 300 python tools/exp_frame.py --config cfg3_5m_sh3_4k_f16 --var GSM_BLEND_SKIP_DYN=1,0 --var GSM_BLEND_EXITG_DYN=1,4 --var GSM_BLEND_WG_WAVES_DYN=16,8 --rounds 2 --frames 10 > gpurun_out/exp4k.log 2>&1; rc=$?; grep variant gpurun_out/exp4k.log; echo exp4k rc=$rc
