#!/bin/bash
# Global path A/B: GPU parity tests, then bench lines (config in G_CONFIG, default config 2) for the
# variants in G_VARIANTS (each "NAME:ENV=VAL,ENV=VAL").
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_g.log 2>&1 || { tail -30 gpurun_out/pytest_g.log; exit 1; }
tail -1 gpurun_out/pytest_g.log
for cfg in ${G_CONFIG:-cfg2_1m_sh3_1080p_f16}; do
for v in ${G_VARIANTS:-default:}; do
  name=${v%%:*}; envs=${v#*:}
  env ${envs//,/ } timeout -k 10 240 python bench.py --config $cfg --steps 50 --warmup 5 --cpu-baseline 0 > gpurun_out/g_bench_$name.log 2>&1 || exit 1
  python3 -c "import json;d=json.loads(open('gpurun_out/g_bench_$name.log').read().strip().splitlines()[-1]);print('$cfg $name',round(d['value'],1),{k:round(x,4) for k,x in d['stages_ms'].items()},d['parity_vs_oracle'])"
done
done
