#!/bin/bash
# r05 experiment (not kept: the grouped-scan patch is not in the tree): GSM_SCAN=grouped against fused / kernel: bench lines
# (twice, interleaved) and kernel traces of configs 2 and 3.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/scanab; mkdir -p $O; export TMPDIR=/tmp
b() {  # label cfg mode
  GSM_SCAN=$3 timeout -k 10 300 python bench.py --config $2 --steps 100 --warmup 5 --cpu-baseline 0 --orbit-steps 0 \
    --inflight-steps 0 --virtual-ranks 0 --traffic-json /dev/null > $O/bench_$1.log 2>&1 || { echo "bench $1 failed"; tail -5 $O/bench_$1.log; exit 1; }
  grep '"metric"' $O/bench_$1.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$1', round(d['value'],1), 'parity', d.get('parity_vs_oracle'), {k: round(x*1e3,1) for k, x in d['stages_ms'].items()})"
}
kt() {  # label cfg mode
  GSM_SCAN=$3 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_$1 -o run -- python3 bench.py \
    --config $2 --steps 30 --warmup 3 --cpu-baseline 0 --parity 0 --orbit-steps 0 --inflight-steps 0 --virtual-ranks 0 \
    > $O/kt_$1.log 2>&1 || { echo "kt $1 failed"; exit 1; }
  python3 - "$O/kt_$1" "$1" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
rows = {r["Name"].split("(")[0].replace("void ", ""): float(r["AverageNs"]) / 1e3 for r in csv.DictReader(open(f))}
print(sys.argv[2], {k: round(v, 1) for k, v in rows.items() if "scatter" in k or "scan" in k or "project" in k})
PY
}
for r in 1 2; do
  b g2_$r cfg2_1m_sh3_1080p_f16 grouped
  b f2_$r cfg2_1m_sh3_1080p_f16 fused
  b g3_$r cfg3_5m_sh3_4k_f16 grouped
  b k3_$r cfg3_5m_sh3_4k_f16 kernel
done
kt g2 cfg2_1m_sh3_1080p_f16 grouped
kt f2 cfg2_1m_sh3_1080p_f16 fused
kt g3 cfg3_5m_sh3_4k_f16 grouped
kt k3 cfg3_5m_sh3_4k_f16 kernel
echo done
