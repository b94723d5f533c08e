#!/bin/bash
# summary of tools/gpu_wide.sh output (gpurun_out/wide)
cd "$(dirname "$0")/.."
for f in gpurun_out/wide/vr*_w*.log; do python3 - "$f" <<'PY'
import json,sys
for line in open(sys.argv[1]):
    if line.startswith('{'):
        d=json.loads(line)
        st=d['slab_stages_ms']
        print(sys.argv[1].split('/')[-1], d['device_frame_ms'], d['max_phase_ms'], 'sort', max(s['sort'] for s in st), 'blend', max(s['blend'] for s in st))
PY
done
for f in gpurun_out/wide/kt_cfg5_w*.log; do echo -n "$f "; grep -h '"metric"' $f | python3 -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l); print(round(d['value'],1), {k: round(v*1e3,1) for k,v in d['stages_ms'].items()})"; done
for d in gpurun_out/wide/kt5_w1 gpurun_out/wide/kt5_w0 gpurun_out/wide/vr_prof; do
python3 - $d.csv <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
print(sys.argv[1])
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:14]:
    print(f"  {r['Name'].split('(')[0][:58]:58s} calls={int(r['Calls']):5d} avg_us={float(r['AverageNs'])/1e3:8.1f}")
PY
done
