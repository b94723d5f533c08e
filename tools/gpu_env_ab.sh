#!/bin/bash
# r06 A/B of environment switches on one box: kernel traces of $CFG (default config 3) for each entry of
# $CASES ("label:VAR=VALUE,VAR=VALUE" or "label:" for the defaults), $REPS rounds alternating; per run the
# sort, scatter and projection kernel averages into gpurun_out/envab/summary.txt.  Then $UC_RUNS runs of the
# freed-uncached reuse child (its stderr: the mapping check's evidence).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/envab
rm -rf $OUT && mkdir -p $OUT
CFG=${CFG:-cfg3_5m_sh3_4k_f16}
for rep in $(seq 1 ${REPS:-2}); do
  for c in $CASES; do
    label=${c%%:*}_r$rep; envs=${c#*:}
    env $(echo "$envs" | tr ',' ' ') timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$label -o run -- \
      python bench.py --config $CFG --steps 20 --warmup 3 --cpu-baseline 0 --parity 0 --orbit-steps 0 --inflight-steps 0 \
      --virtual-ranks 0 > $OUT/$label.log 2>&1 || { echo "run $label failed"; tail -5 $OUT/$label.log; exit 1; }
    f=$(find $OUT/$label -name '*kernel_stats.csv' | head -1)
    python3 - "$f" "$label" <<'PY' | tee -a $OUT/summary.txt
import csv, sys
rows = [(r["Name"].split("(")[0], float(r["AverageNs"]) / 1e3) for r in csv.DictReader(open(sys.argv[1]))]
keep = [f"{n.replace('void gsm::', '').replace('gsm::', '')} {v:.1f}" for n, v in rows
        if any(k in n for k in ("radix", "tile_sort", "scatter", "k_project<", "wide"))]
print(f"{sys.argv[2]:22s} " + " | ".join(sorted(keep)))
PY
  done
done
for i in $(seq 1 ${UC_RUNS:-0}); do
  timeout -k 10 240 python -u tests/mg_uc_reuse.py $OUT/uc_$i.json > $OUT/uc_$i.log 2>&1 || { echo "uc $i failed rc=$?"; tail -20 $OUT/uc_$i.log; exit 1; }
  echo "uc run $i"; grep -v amdgpu.ids $OUT/uc_$i.log
done
echo "=== done"
