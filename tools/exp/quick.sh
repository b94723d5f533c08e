# quick check: parity tests (optional), one bench line, kernel averages from rocprofv3
set -u
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
if [ "${TESTS:-1}" = 1 ]; then
  timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 300 python bench.py --steps 50 --warmup 5 --cpu-baseline 0 ${BENCH_ARGS:-} > gpurun_out/bench.log 2>&1 || exit $?
python -c "import json;d=json.loads(open('gpurun_out/bench.log').read().strip().splitlines()[-1]);print(round(d['value'],1),d['parity_vs_oracle'],{k:round(v*1000,1) for k,v in d['stages_ms'].items()})"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python bench.py --steps 20 --warmup 3 --cpu-baseline 0 --parity 0 ${BENCH_ARGS:-} > gpurun_out/rocprof.log 2>&1 || exit $?
python - <<'PY'
import csv, glob
f = glob.glob('gpurun_out/prof/**/*kernel_stats.csv', recursive=True)[0]
tot = 0
for r in csv.DictReader(open(f)):
    print(r['Name'][:60].ljust(60), r['Calls'].rjust(4), round(float(r['AverageNs'])/1000, 1))
PY
