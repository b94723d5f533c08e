# Multi-GPU frame check on one GPU: the multi-GPU tests, the per-rank device frame of
# 8 virtual ranks at configs 3 / 2 (tools/exp_virtual_ranks.py), and a kernel trace of config 4.
# OUT=<dir under gpurun_out> (default mg); extra environment (GSM_MG_*) passes through for A/B runs.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${OUT:-mg}
mkdir -p $O
timeout -k 10 700 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_multigpu_ipc.py tests/test_multigpu_rccl.py tests/test_gpu_parity.py -k "multigpu or virtual or processes or config4 or partition or rccl or records" > $O/pytest_mg.log 2>&1 || { tail -40 $O/pytest_mg.log | cut -c1-300; exit 1; }
tail -1 $O/pytest_mg.log
for c in cfg3_5m_sh3_4k_f16 cfg2_1m_sh3_1080p_f16; do
  timeout -k 10 300 python -u tools/exp_virtual_ranks.py --config $c --world 8 --frames 7 --stages 1 --single 1 > $O/vr_$c.json 2>$O/vr.err || { tail -20 $O/vr.err; exit 1; }
  python3 -c "
import json; d=json.loads([l for l in open('$O/vr_$c.json') if l.startswith('{')][-1])
print('$c', d['device_frame_ms'], d['max_phase_ms'], d['device_speedup'], d['one_gpu_frame_ms'], d['xgmi_model']['modelled_frame_ms'])
print(d['slab_stages_ms'][:2])
"
done
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o vr -- python3 tools/exp_virtual_ranks.py --config cfg3_5m_sh3_4k_f16 --world 8 --frames 5 --stages 0 > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
python3 - <<PY
import csv
rows=list(csv.DictReader(open('$O/prof/vr_kernel_stats.csv')))
for r in sorted(rows, key=lambda r: -float(r['TotalDurationNs']))[:14]:
    print(r['Name'][:70], r['Calls'], round(float(r['AverageNs'])/1e3,1))
PY
