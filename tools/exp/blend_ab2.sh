set -u
cd $GRAFT_REPO_ROOT; source tools/exp/ab_lib.sh
run base X=1 || exit 1
run notable GSM_BLEND_EXPT=1 || exit 1
run nobreak GSM_BLEND_EXPT=2 || exit 1
