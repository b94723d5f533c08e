#!/bin/bash
# per-rank kernel times of the 8-rank frame (virtual ranks) with and without the blend schedule block
mkdir -p gpurun_out; export TMPDIR=/tmp
for s in 1 0; do
  GSM_BLEND_SCHED=$s timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/vrs$s -o run -- \
     python tools/exp_virtual_ranks.py --config ${CFG:-cfg3_5m_sh3_4k_f16} --world 8 --frames 3 --stages 0 > gpurun_out/vrs$s.log 2>&1 || exit 1
  echo "== GSM_BLEND_SCHED=$s"
  tail -1 gpurun_out/vrs$s.log | python -c "import json,sys;d=json.loads(sys.stdin.read());print(d['max_phase_ms'],d['device_frame_ms'])"
  find gpurun_out/vrs$s -name "*kernel_stats.csv" -exec python -c "
import csv,sys
for r in csv.DictReader(open(sys.argv[1])):
    print('  %-28s %6d calls %8.1f us' % (r['Name'].split('(')[0].replace('void gsm::','').replace('gsm::','')[:28], int(r['Calls']), float(r['AverageNs'])/1e3))
" {} \;
done
