set -u
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
for b in 12 14 28; do timeout -k 5 60 ./tools/exp/rocprim_sort_probe 2632483 $b || exit $?; done
timeout -k 5 60 ./tools/exp/rocprim_sort_probe 13000000 14 || exit $?
timeout -k 10 300 python bench.py --steps 50 --warmup 5 --cpu-baseline 0 > gpurun_out/bench.log 2>&1 || exit $?
python -c "import json;d=json.loads(open('gpurun_out/bench.log').read().strip().splitlines()[-1]);print(round(d['value'],1),d['parity_vs_oracle'],{k:round(v*1000,1) for k,v in d['stages_ms'].items()})"
