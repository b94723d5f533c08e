set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python tools/exp_frame.py --var GSM_BLEND_PRIO=1,0 --var GSM_BLEND_WAVES=8,16 > gpurun_out/exp17.log 2>&1; rc=$?; grep variant gpurun_out/exp17.log; echo exp rc=$rc
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/exp_frame.py --config cfg3_5m_sh3_4k_f16 --rounds 2 --frames 10 --var GSM_BLEND_PRIO=1,0 --var GSM_BLEND_WAVES=8,16 --var GSM_BLEND_SCHED=0,1 > gpurun_out/exp17_4k.log 2>&1; rc=$?; grep variant gpurun_out/exp17_4k.log; echo exp4k rc=$rc
