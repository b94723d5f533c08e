set -o pipefail
mkdir -p gpurun_out/r04d
timeout -k 10 120 ./tools/exp/uc_alloc_probe > gpurun_out/r04d/uc_alloc_probe.log 2>&1 || exit 1; cat gpurun_out/r04d/uc_alloc_probe.log
timeout -k 10 700 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_multigpu_ipc.py tests/test_gpu_parity.py -k "multigpu or virtual or processes or config4 or 2_32 or 12bit or partition" > gpurun_out/r04d/pytest_mg.log 2>&1 || { tail -30 gpurun_out/r04d/pytest_mg.log; exit 1; }
tail -2 gpurun_out/r04d/pytest_mg.log
timeout -k 10 300 python -u tools/exp_virtual_ranks.py --config cfg3_5m_sh3_4k_f16 --world 8 --frames 5 --stages 1 --single 1 > gpurun_out/r04d/vr_cfg3_w8.json 2>gpurun_out/r04d/vr.err || { tail -20 gpurun_out/r04d/vr.err; exit 1; }
python3 -c "
import json; d=json.loads([l for l in open('gpurun_out/r04d/vr_cfg3_w8.json') if l.startswith('{')][-1])
print('vr', d['device_frame_ms'], d['max_phase_ms'], d['device_speedup'], d['xgmi_model']['modelled_frame_ms'])
print('stages', d['slab_stages_ms'][:3])
"
for m in uncached-ab fine; do GSM_MG_MEM=$m timeout -k 10 300 python -u tools/exp/mg_memkind_ab.py 3 > gpurun_out/r04d/memkind_$m.log 2>&1 || exit 1; tail -1 gpurun_out/r04d/memkind_$m.log; done
for w in 0 1; do
GSM_SORT_WIDE12=$w timeout -k 10 300 python -u bench.py --cpu-baseline 0 --virtual-ranks 0 --orbit-steps 0 --inflight-steps 0 > gpurun_out/r04d/bench_w12_$w.log 2>&1 || { tail -20 gpurun_out/r04d/bench_w12_$w.log; exit 1; }
tail -1 gpurun_out/r04d/bench_w12_$w.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('wide12=$w fps', round(d['value'],1), d['parity_vs_oracle'], {k: round(v*1e3,1) for k,v in d['stages_ms'].items()})"
done
