set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --cpu-baseline 0 > gpurun_out/bench_n1.log 2>&1; rc=$?; tail -1 gpurun_out/bench_n1.log | cut -c1-300; echo bench1 rc=$rc
[ $rc -eq 0 ] || exit $rc
BENCH_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 5 --warmup 2 > gpurun_out/bench_n2_gloo.log 2>&1; rc=$?; tail -3 gpurun_out/bench_n2_gloo.log | cut -c1-400; echo bench2 rc=$rc
[ $rc -eq 0 ] || exit $rc
BENCH_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 2 --steps 5 --warmup 2 --multi replicas > gpurun_out/bench_n2r_gloo.log 2>&1; rc=$?; tail -1 gpurun_out/bench_n2r_gloo.log | cut -c1-300; echo bench2r rc=$rc
