set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python tools/exp_frame.py --var GSM_BLEND_WG_WAVES_DYN=16,12,8,4 > gpurun_out/exp_waves.log 2>&1; rc=$?; cat gpurun_out/exp_waves.log | grep variant; echo rc=$rc
[ $rc -eq 0 ] || exit $rc
bash tools/gpu_pmc.sh
