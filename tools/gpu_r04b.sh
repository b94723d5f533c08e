set -o pipefail
mkdir -p gpurun_out/r04b
python3 -c "import os; print('affinity', len(os.sched_getaffinity(0)), 'cpus', os.cpu_count())" > gpurun_out/r04b/cpus.log; cat /sys/fs/cgroup/cpu.max >> gpurun_out/r04b/cpus.log 2>&1
true
echo probe-done
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_multigpu_ipc.py tests/test_gpu_parity.py -k "multigpu or virtual or processes or config4 or 2_32 or partition" > gpurun_out/r04b/pytest_mg.log 2>&1 || { tail -30 gpurun_out/r04b/pytest_mg.log; exit 1; }
tail -3 gpurun_out/r04b/pytest_mg.log
for m in uncached fine cached; do GSM_MG_MEM=$m timeout -k 10 300 python -u tools/exp/mg_memkind_ab.py 3 > gpurun_out/r04b/memkind_$m.log 2>&1 || exit 1; tail -1 gpurun_out/r04b/memkind_$m.log; done
cat gpurun_out/r04b/l2_alias_probe.log gpurun_out/r04b/cpus.log
