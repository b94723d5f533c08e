set -o pipefail
mkdir -p gpurun_out/r04g
for d in 1 0; do
timeout -k 10 300 python -u tools/exp_virtual_ranks.py --config cfg3_5m_sh3_4k_f16 --world 8 --frames 5 --stages 1 --depth $d > gpurun_out/r04g/vr_d$d.json 2>gpurun_out/r04g/vr.err || { tail -20 gpurun_out/r04g/vr.err; exit 1; }
python3 -c "
import json; d=json.loads([l for l in open('gpurun_out/r04g/vr_d$d.json') if l.startswith('{')][-1])
print('depth $d vr', d['device_frame_ms'], d['max_phase_ms'])
print('stages', d['slab_stages_ms'][:2])
"
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r04g/prof -o vr -- python3 tools/exp_virtual_ranks.py --config cfg3_5m_sh3_4k_f16 --world 8 --frames 5 --stages 0 > gpurun_out/r04g/prof.log 2>&1 || { tail -20 gpurun_out/r04g/prof.log; exit 1; }
find gpurun_out/r04g/prof -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} gpurun_out/r04g/kernel_stats.csv
python3 - <<'PY'
import csv
rows=list(csv.DictReader(open('gpurun_out/r04g/kernel_stats.csv')))
for r in sorted(rows, key=lambda r: -float(r['TotalDurationNs']))[:22]:
    print(r['Name'][:90], r['Calls'], round(float(r['AverageNs'])/1e3,1))
PY
