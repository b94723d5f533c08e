set -o pipefail
mkdir -p gpurun_out/r04u
BENCH_SAME_GPU=1 timeout -k 10 600 python -u bench.py --gpus 2 --steps 30 --warmup 5 > gpurun_out/r04u/bench_w2.log 2>&1 || { tail -30 gpurun_out/r04u/bench_w2.log; exit 1; }
tail -1 gpurun_out/r04u/bench_w2.log | cut -c1-1500
