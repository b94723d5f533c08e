# N-rank rehearsals of bench.py's multi-GPU frame with the processes sharing one GPU (BENCH_SAME_GPU=1):
# N = 2 and 4, serial and pipelined (--mg-pipeline 1).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${OUT:-samegpu}
mkdir -p $O
for n in 2 4; do
  for p in 0 1; do
    BENCH_SAME_GPU=1 timeout -k 10 600 python -u bench.py --gpus $n --steps 30 --warmup 5 --mg-pipeline $p > $O/bench_w${n}_p$p.log 2>&1 || { tail -30 $O/bench_w${n}_p$p.log; exit 1; }
    tail -1 $O/bench_w${n}_p$p.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); c=d.get('config4') or {}; print('N=$n pipe=$p fps', round(d['value'],1), 'parity', d['parity_vs_oracle'], 'transport', d.get('multi_transport'), 'timeouts', d.get('barrier_timeouts'), d.get('failed_peer_arrivals'), 'cfg4', round(c.get('value',0),1), c.get('barrier_timeouts'))"
  done
done
