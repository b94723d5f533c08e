# Blend change check: the GPU parity tests, then bench lines of configs 2 and 3 (static + orbit blend).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${OUT:-blend}
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log | cut -c1-300; exit 1; }
tail -1 $O/pytest.log
for cfg in cfg2_1m_sh3_1080p_f16 cfg3_5m_sh3_4k_f16; do
  timeout -k 10 300 python -u bench.py --config $cfg --steps 50 --warmup 5 --cpu-baseline 0 --virtual-ranks 0 --inflight-steps 0 > $O/bench_$cfg.log 2>&1 || { tail -20 $O/bench_$cfg.log; exit 1; }
  tail -1 $O/bench_$cfg.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); o=d.get('orbit') or {}; print('$cfg fps', round(d['value'],1), 'parity', d['parity_vs_oracle'], 'orbit', round(o.get('value',0),1), 'orbit blend', round(o.get('blend_ms',0)*1e3,1), {k: round(v*1e3,1) for k,v in d['stages_ms'].items()})"
done
