set -o pipefail
O=gpurun_out/r04r
mkdir -p $O
timeout -k 10 700 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_multigpu_ipc.py tests/test_multigpu_rccl.py > $O/pytest_mg.log 2>&1 || { tail -40 $O/pytest_mg.log | cut -c1-300; exit 1; }
tail -1 $O/pytest_mg.log
for c in cfg3_5m_sh3_4k_f16 cfg2_1m_sh3_1080p_f16; do
  timeout -k 10 300 python -u tools/exp_virtual_ranks.py --config $c --world 8 --frames 7 --stages 1 --single 1 --interval 20 > $O/vr_$c.json 2>$O/vr.err || { tail -20 $O/vr.err; exit 1; }
  GSM_MG_PIPELINE=1 timeout -k 10 300 python -u tools/exp_virtual_ranks.py --config $c --world 8 --interval 20 > $O/vr_pipe_$c.json 2>$O/vr.err || { tail -20 $O/vr.err; exit 1; }
  python3 -c "
import json
d=json.loads([l for l in open('$O/vr_$c.json') if l.startswith('{')][-1])
e=json.loads([l for l in open('$O/vr_pipe_$c.json') if l.startswith('{')][-1])
print('$c one-frame', d['device_frame_ms'], d['max_phase_ms'], 'speedup', d['device_speedup'], '1gpu', d['one_gpu_frame_ms'])
print('   interval serial', d['interval'], )
print('   interval pipelined', e['interval'])
"
done
