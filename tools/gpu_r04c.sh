set -o pipefail
mkdir -p gpurun_out/r04c
timeout -k 10 120 ./tools/exp/uc_write_probe > gpurun_out/r04c/uc_write_probe.log 2>&1 || { cat gpurun_out/r04c/uc_write_probe.log; exit 1; }
cat gpurun_out/r04c/uc_write_probe.log
timeout -k 10 600 python -u bench.py > gpurun_out/r04c/bench.log 2>&1 || { tail -20 gpurun_out/r04c/bench.log; exit 1; }
tail -1 gpurun_out/r04c/bench.log > gpurun_out/r04c/bench_cfg2.json
python3 -c "
import json; d=json.load(open('gpurun_out/r04c/bench_cfg2.json'))
print('fps', round(d['value'],1), 'parity', d['parity_vs_oracle'], 'blend', d['stages_ms']['blend'], 'orbit', d['orbit']['value'] if d['orbit'] else None)
print('cpu', json.dumps(d['cpu_baseline'])[:600])
print('vr', json.dumps(d.get('virtual_ranks_config4'))[:1500])
"
