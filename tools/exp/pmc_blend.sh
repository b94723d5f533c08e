set -u
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
for v in 1 0; do
  GSM_BLEND_COMPACT=$v timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY --output-format csv -d gpurun_out/pmc_c$v -o run -- python bench.py --steps 10 --warmup 3 --cpu-baseline 0 --parity 0 > gpurun_out/pmc_c$v.log 2>&1 || exit $?
  python - "$v" <<'PY'
import csv, glob, sys, collections
v = sys.argv[1]
f = glob.glob(f'gpurun_out/pmc_c{v}/**/*counter_collection.csv', recursive=True)[0]
acc = collections.defaultdict(list)
for r in csv.DictReader(open(f)):
    if 'blend_px' in r['Kernel_Name']:
        acc[r['Counter_Name']].append(float(r['Counter_Value']))
print('compact', v, {k: round(sum(x)/len(x)/1e6, 2) for k, x in sorted(acc.items())}, 'n', len(next(iter(acc.values()))))
PY
done
