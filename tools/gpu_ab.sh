set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -5 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
for mode in default radix4; do
  if [ $mode = radix4 ]; then export GSM_SORT=radix4; else unset GSM_SORT; fi
  timeout -k 10 300 python bench.py --steps 50 --warmup 5 --cpu-baseline 0 > gpurun_out/bench_$mode.log 2>&1 || exit $?
  python -c "import json;d=json.loads(open('gpurun_out/bench_$mode.log').read().strip().splitlines()[-1]);print('$mode',round(d['value'],1),d['parity_vs_oracle'],{k:round(v*1000,1) for k,v in d['stages_ms'].items()})"
done
unset GSM_SORT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python bench.py --steps 20 --warmup 3 --cpu-baseline 0 --parity 0 > gpurun_out/rocprof.log 2>&1 || exit $?
find gpurun_out/prof -name "*kernel_stats.csv" -exec cp {} gpurun_out/kernel_stats.csv \;
cut -c1-60,200-260 gpurun_out/kernel_stats.csv | head -20
