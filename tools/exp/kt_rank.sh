set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/ktr
export TMPDIR=/tmp
for v in atomic ballot; do
  GSM_SORT_RANK=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ktr/$v -o run -- python3 bench.py --config cfg3_5m_sh3_4k_f16 --steps 20 --warmup 3 --cpu-baseline 0 --parity 0 --orbit-steps 0 --inflight-steps 0 --virtual-ranks 0 > gpurun_out/ktr/$v.log 2>&1 || exit 1
  python3 - "$v" <<'PY'
import csv, glob, sys
f = glob.glob(f"gpurun_out/ktr/{sys.argv[1]}/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    if "radix" in r["Name"] or "tile_sort" in r["Name"]:
        print(sys.argv[1], r["Name"].split("(")[0], r["Calls"], round(float(r["AverageNs"])/1e3,1))
PY
done
