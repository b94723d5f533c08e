set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/fs
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/fs/pytest.log 2>&1 || { tail -30 gpurun_out/fs/pytest.log; exit 1; }
tail -1 gpurun_out/fs/pytest.log
for r in 1 2; do for v in 1 0; do
  GSM_SCAN_FUSED=$v timeout -k 10 240 python bench.py --config cfg2_1m_sh3_1080p_f16 --steps 100 --warmup 5 --cpu-baseline 0 --orbit-steps 0 --virtual-ranks 0 --inflight-steps 0 > gpurun_out/fs/b_${v}_${r}.log 2>&1 || exit 1
  python3 -c "import json;d=json.loads(open('gpurun_out/fs/b_${v}_${r}.log').read().strip().splitlines()[-1]);print('fused=$v',round(d['value'],1),{k:round(x*1e3,1) for k,x in d['stages_ms'].items()},d['parity_vs_oracle'])"
done; done
for v in 1 0; do
  GSM_SCAN_FUSED=$v timeout -k 10 300 python tools/exp_virtual_ranks.py --config cfg2_1m_sh3_1080p_f16 --world 8 --frames 5 > gpurun_out/fs/vr_$v.log 2>&1 || exit 1
  grep '^{' gpurun_out/fs/vr_$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('vr cfg2 w8 fused=$v', d['device_frame_ms'], d['max_phase_ms'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/fs/kt -o run -- python3 bench.py --config cfg2_1m_sh3_1080p_f16 --steps 20 --warmup 3 --cpu-baseline 0 --parity 0 --orbit-steps 0 --inflight-steps 0 --virtual-ranks 0 > gpurun_out/fs/kt.log 2>&1 || exit 1
