# kernel traces of configs 2 / 3 (timelines) and PMC passes at config 3 (projection, radix
# downsweeps, tile sort: which roof binds)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/${OUT:-prof}
for cfg in cfg2_1m_sh3_1080p_f16 cfg3_5m_sh3_4k_f16; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${OUT:-prof}/kt_$cfg -o run -- \
    python bench.py --config $cfg --steps 20 --warmup 3 --cpu-baseline 0 --parity 0 --orbit-steps 0 --inflight-steps 0 --virtual-ranks 0 \
    > gpurun_out/${OUT:-prof}/kt_$cfg.log 2>&1 || { echo "trace failed $cfg"; tail -5 gpurun_out/${OUT:-prof}/kt_$cfg.log; exit 1; }
  echo "== $cfg"; tail -1 gpurun_out/${OUT:-prof}/kt_$cfg.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('fps', round(d['value'],1), {k: round(v*1e3,1) for k,v in d['stages_ms'].items()})"
  python3 tools/timeline.py $(find gpurun_out/${OUT:-prof}/kt_$cfg -name '*kernel_trace.csv' | head -1) > gpurun_out/${OUT:-prof}/timeline_$cfg.txt 2>&1
  cp $(find gpurun_out/${OUT:-prof}/kt_$cfg -name '*kernel_stats.csv' | head -1) gpurun_out/${OUT:-prof}/kernel_stats_$cfg.csv
done
CFG=cfg3_5m_sh3_4k_f16 OUT=${OUT:-prof}/pmc3 bash tools/gpu_pmc.sh > gpurun_out/${OUT:-prof}/pmc3.log 2>&1 || { tail -20 gpurun_out/${OUT:-prof}/pmc3.log; exit 1; }
grep -A14 "k_project<\|k_radix_downsweep\|k_tile_sort" gpurun_out/${OUT:-prof}/pmc3/summary.txt | head -80
