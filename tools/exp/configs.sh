set -u
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
for c in cfg3_5m_sh3_4k_f16 cfg5_1m_sh2_stereo_2x1440x1600_f16; do
  timeout -k 10 300 python bench.py --config $c --steps 20 --warmup 3 --cpu-baseline 0 ${EXTRA:-} > gpurun_out/bench_$c.log 2>&1 || exit $?
  python -c "import json;d=json.loads(open('gpurun_out/bench_$c.log').read().strip().splitlines()[-1]);print('$c',round(d['value'],1),d['parity_vs_oracle'],{k:round(v*1000,1) for k,v in d['stages_ms'].items()})"
done
