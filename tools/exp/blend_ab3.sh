set -u
cd $GRAFT_REPO_ROOT; source tools/exp/ab_lib.sh
run split X=1 || exit 1
run nosplit GSM_BLEND_SPLIT=0 || exit 1
timeout -k 10 200 python tools/blend_trace.py
