#!/bin/bash
# DepthFirst stereo (config 5): GPU tests, then bench lines for the variants in DF_VARIANTS
# (each "NAME:ENV=VAL,ENV=VAL"; default: the shipped path).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
timeout -k 10 300 python -u -m pytest tests/test_depthfirst.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_df.log 2>&1 || { tail -30 gpurun_out/pytest_df.log; exit 1; }
tail -1 gpurun_out/pytest_df.log
for v in ${DF_VARIANTS:-default:}; do
  name=${v%%:*}; envs=${v#*:}
  env ${envs//,/ } timeout -k 10 240 python bench.py --config cfg5_1m_sh2_stereo_2x1440x1600_f16 --steps 30 --warmup 5 --cpu-baseline 0 > gpurun_out/df_bench_$name.log 2>&1 || exit 1
  python3 -c "import json;d=json.loads(open('gpurun_out/df_bench_$name.log').read().strip().splitlines()[-1]);print('$name',round(d['value'],1),{k:round(x,4) for k,x in d['stages_ms'].items()},d['parity_vs_oracle'],d.get('blend_walk'))"
done
