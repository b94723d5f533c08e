mkdir -p gpurun_out; export TMPDIR=/tmp
run() {  # label env...
  local label=$1; shift
  env "$@" timeout -k 10 120 python bench.py --steps 30 --warmup 5 --cpu-baseline 0 --parity 0 ${BENCH_ARGS:-} > gpurun_out/ab_$label.log 2>&1 || { echo "$label failed"; tail -3 gpurun_out/ab_$label.log; return 1; }
  python -c "import json;d=json.loads(open('gpurun_out/ab_$label.log').read().strip().splitlines()[-1]);print('$label',round(d['value'],1),'blend',round(d['stages_ms']['blend_timed_region']*1000,1), {k:round(v*1000,1) for k,v in d['stages_ms'].items()})"
}
