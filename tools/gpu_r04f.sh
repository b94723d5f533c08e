set -o pipefail
mkdir -p gpurun_out/r04f
timeout -k 10 700 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_multigpu_ipc.py tests/test_gpu_parity.py -k "multigpu or virtual or processes or config4 or 2_32 or 12bit or partition" > gpurun_out/r04f/pytest_mg.log 2>&1 || { tail -30 gpurun_out/r04f/pytest_mg.log; exit 1; }
tail -2 gpurun_out/r04f/pytest_mg.log
timeout -k 10 300 python -u tools/exp_virtual_ranks.py --config cfg3_5m_sh3_4k_f16 --world 8 --frames 5 --stages 1 --single 1 > gpurun_out/r04f/vr_cfg3_w8.json 2>gpurun_out/r04f/vr.err || { tail -20 gpurun_out/r04f/vr.err; exit 1; }
python3 -c "
import json; d=json.loads([l for l in open('gpurun_out/r04f/vr_cfg3_w8.json') if l.startswith('{')][-1])
print('vr', d['device_frame_ms'], d['max_phase_ms'], d['device_speedup'], d['xgmi_model']['modelled_frame_ms'])
print('stages', d['slab_stages_ms'][:3])
"
for m in uncached-ab fine; do GSM_MG_MEM=$m timeout -k 10 300 python -u tools/exp/mg_memkind_ab.py 3 > gpurun_out/r04f/memkind_$m.log 2>&1 || exit 1; tail -1 gpurun_out/r04f/memkind_$m.log; done
