#!/bin/bash
# r06: the wide downsweep's first-chunk preload -- config 5 kernel traces (DepthFirst depth sort: 3 wide
# passes) and config-4 virtual-rank kernel traces (the slab's wide tile pass), HEAD against the tree.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
CFGS="cfg5_1m_sh2_stereo_2x1440x1600_f16" VARIANTS="head cur" REPS=2 bash tools/gpu_ab_proj.sh || exit 1
for rep in 1 2; do
  for v in head cur; do
    if [ $v = cur ]; then lib=$PWD/gsm-renderer_amd/lib/libgsm_amd.so; else lib=$PWD/gsm-renderer_amd/lib_ab_$v/libgsm_amd.so; fi
    rm -rf gpurun_out/vrw_${v}_$rep
    GSM_AMD_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/vrw_${v}_$rep -o run -- \
      python tools/exp_virtual_ranks.py --frames 5 --stages 0 --single 0 > gpurun_out/vrw_${v}_$rep.log 2>&1 || { echo "vr $v failed"; exit 1; }
    f=$(find gpurun_out/vrw_${v}_$rep -name '*kernel_stats.csv' | head -1)
    python3 - "$f" ${v}_$rep <<'PY'
import csv, sys
r = {x["Name"].split("(")[0]: float(x["AverageNs"]) / 1e3 for x in csv.DictReader(open(sys.argv[1]))}
print(sys.argv[2], {k.replace("void gsm::", ""): round(v, 1) for k, v in r.items() if "wide" in k or "tile_sort" in k})
PY
  done
done
echo "=== done"
