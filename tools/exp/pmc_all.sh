set -u
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM SQ_WAIT_ANY --output-format csv -d gpurun_out/pmc_all -o run -- python bench.py --steps 10 --warmup 3 --cpu-baseline 0 --parity 0 ${BENCH_ARGS:-} > gpurun_out/pmc_all.log 2>&1 || exit $?
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_INSTS_SMEM --output-format csv -d gpurun_out/pmc_all2 -o run -- python bench.py --steps 10 --warmup 3 --cpu-baseline 0 --parity 0 ${BENCH_ARGS:-} > gpurun_out/pmc_all2.log 2>&1 || exit $?
python - <<'PY'
import csv, glob, collections
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for d in ('pmc_all', 'pmc_all2'):
    f = glob.glob(f'gpurun_out/{d}/**/*counter_collection.csv', recursive=True)[0]
    for r in csv.DictReader(open(f)):
        k = r['Kernel_Name'].split('(')[0][-40:]
        acc[k][r['Counter_Name']].append(float(r['Counter_Value']))
for k, c in acc.items():
    print(k.ljust(40), {n: round(sum(x)/len(x)/1e6, 3) for n, x in sorted(c.items())})
PY
