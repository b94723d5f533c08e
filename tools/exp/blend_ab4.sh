set -u
cd $GRAFT_REPO_ROOT; source tools/exp/ab_lib.sh
run w8 X=1 || exit 1
run w12 GSM_BLEND_WAVES=12 || exit 1
run w16 GSM_BLEND_WAVES=16 || exit 1
run w8nc GSM_BLEND_COMPACT=0 || exit 1
BENCH_ARGS="--config cfg3_5m_sh3_4k_f16" run 4k_w16 X=1 || exit 1
BENCH_ARGS="--config cfg3_5m_sh3_4k_f16" run 4k_w12 GSM_BLEND_WAVES=12 || exit 1
BENCH_ARGS="--config cfg3_5m_sh3_4k_f16" run 4k_w8 GSM_BLEND_WAVES=8 || exit 1
BENCH_ARGS="--config cfg3_5m_sh3_4k_f16" run 4k_w16nc GSM_BLEND_COMPACT=0 || exit 1
