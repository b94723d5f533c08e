#!/bin/bash
# r06 A/B on one box: kernel traces of configs 2 and 3 for the library variants of tools/build_ab.sh
# (VARIANTS, "cur" = gsm-renderer_amd/lib), REPS rounds alternating the variants; per run the k_project,
# tile-pass and frame averages into gpurun_out/abp/summary.txt.  Then (SORT=1) the sort's LDS counters at
# config 3 and the tile passes with ballot ranks; (UC=1) the freed-uncached reuse child once.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/abp
rm -rf $OUT && mkdir -p $OUT
summ() {  # dir label
  f=$(find $1 -name '*kernel_stats.csv' | head -1)
  python3 - "$f" "$2" "$1.log" <<'PY' | tee -a $OUT/summary.txt
import csv, sys, json
rows = {r["Name"].split("(")[0]: float(r["AverageNs"]) / 1e3 for r in csv.DictReader(open(sys.argv[1]))}
pick = lambda p: next((v for k, v in rows.items() if k.startswith(p)), float("nan"))
fps = float("nan")
for l in open(sys.argv[3]):
    if l.startswith("{") and '"metric"' in l: fps = json.loads(l)["value"]
print(f"{sys.argv[2]:28s} k_project {pick('void gsm::k_project<'):7.1f}  down1 {pick('void gsm::k_radix_downsweep<7, false, false>') if 'cfg3' in sys.argv[2] else pick('void gsm::k_radix_downsweep<6, false, false>'):6.1f}"
      f"  down2 {pick('void gsm::k_radix_downsweep<7, false, true>') if 'cfg3' in sys.argv[2] else pick('void gsm::k_radix_downsweep<6, false, true>'):6.1f}  tile_sort {pick('void gsm::k_tile_sort<'):6.1f}"
      f"  scatter {pick('gsm::k_scatter'):6.1f}  blend {pick('void gsm::k_blend'):6.1f}  wide_down {pick('void gsm::k_wide_downsweep'):6.1f}"
      f"  up {pick('void gsm::k_radix_upsweep'):5.1f}  scan {pick('gsm::k_scan_blocks'):5.1f}  fps {fps:7.1f}")
PY
}
run() {  # label lib cfg [env...]
  local label=$1 lib=$2 cfg=$3; shift 3
  env "$@" GSM_AMD_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$label -o run -- \
    python bench.py --config $cfg --steps 20 --warmup 3 --cpu-baseline 0 --parity 0 --orbit-steps 0 --inflight-steps 0 \
    --virtual-ranks 0 > $OUT/$label.log 2>&1 || { echo "run $label failed"; tail -5 $OUT/$label.log; return 1; }
  summ $OUT/$label $label
}
for rep in $(seq 1 ${REPS:-2}); do
  for v in ${VARIANTS:-cur}; do
    if [ $v = cur ]; then lib=$PWD/gsm-renderer_amd/lib/libgsm_amd.so; else lib=$PWD/gsm-renderer_amd/lib_ab_$v/libgsm_amd.so; fi
    for cfg in ${CFGS:-cfg2_1m_sh3_1080p_f16 cfg3_5m_sh3_4k_f16}; do
      run ${v}_${cfg%%_*}_r$rep $lib $cfg || exit 1
    done
  done
done
if [ "${SORT:-0}" = 1 ]; then
  run ballot_cfg3 $PWD/gsm-renderer_amd/lib/libgsm_amd.so cfg3_5m_sh3_4k_f16 GSM_SORT_RANK=ballot || exit 1
  timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_ADDR_CONFLICT SQ_ACTIVE_INST_LDS SQ_LDS_UNALIGNED_STALL SQ_INSTS_LDS_ATOMIC \
    --output-format csv -d $OUT/pmc_lds -o p -- python bench.py --config cfg3_5m_sh3_4k_f16 --steps 5 --warmup 2 --cpu-baseline 0 \
    --parity 0 --orbit-steps 0 --inflight-steps 0 --virtual-ranks 0 > $OUT/pmc_lds.log 2>&1 || { echo "pmc lds failed"; tail -5 $OUT/pmc_lds.log; exit 1; }
  python3 tools/pmc_summary.py $OUT/pmc_lds > $OUT/pmc_lds.txt
  grep -A9 -E "k_radix_downsweep<7|k_tile_sort|k_radix_upsweep<7" $OUT/pmc_lds.txt
fi
if [ "${UC:-0}" = 1 ]; then
  timeout -k 10 240 python -u tests/mg_uc_reuse.py $OUT/uc.json > $OUT/uc.log 2>&1 || { echo "uc failed rc=$?"; tail -20 $OUT/uc.log; exit 1; }
  grep -E '^\{|refuses|check failed' $OUT/uc.log
fi
echo "=== done"
