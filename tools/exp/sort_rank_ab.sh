source tools/exp/ab_lib.sh
for c in cfg3_5m_sh3_4k_f16 cfg2_1m_sh3_1080p_f16; do
  export BENCH_ARGS="--config $c --orbit-steps 0 --inflight-steps 0 --virtual-ranks 0"
  run ${c}_atomic X=1 || exit 1
  run ${c}_ballot GSM_SORT_RANK=ballot || exit 1
  run ${c}_atomic2 X=1 || exit 1
  run ${c}_ballot2 GSM_SORT_RANK=ballot || exit 1
done
