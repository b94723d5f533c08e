set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --cpu-baseline 0 > gpurun_out/bench.log 2>&1; rc=$?; tail -1 gpurun_out/bench.log | cut -c1-250; echo bench rc=$rc
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --config cfg3_5m_sh3_4k_f16 --steps 30 --warmup 3 --cpu-baseline 0 > gpurun_out/bench_4k.log 2>&1; rc=$?; tail -1 gpurun_out/bench_4k.log | cut -c1-250; echo bench4k rc=$rc
