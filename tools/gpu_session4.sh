set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python tools/exp_frame.py --var GSM_BLEND_DIAG_DYN=0,1 > gpurun_out/exp_diag.log 2>&1; rc=$?; grep variant gpurun_out/exp_diag.log; echo rc=$rc
[ $rc -eq 0 ] || exit $rc
bash tools/gpu_pmc.sh
