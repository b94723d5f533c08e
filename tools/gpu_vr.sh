#!/bin/bash
# Virtual-rank timing of the multi-GPU frame (tools/exp_virtual_ranks.py) + its kernel trace.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-vr}
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "--- $name rc=$rc"; tail -n 5 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "ABORT after $name (rc=$rc)"; exit $rc; fi
  return $rc
}
for cfg in ${VR_CONFIGS:-cfg3_5m_sh3_4k_f16 cfg2_1m_sh3_1080p_f16}; do
  step ${TAG}_${cfg}_w${VR_WORLD:-8} 300 python tools/exp_virtual_ranks.py --config $cfg --world ${VR_WORLD:-8} --frames 5
done
if [ "${VR_TRACE:-1}" = "1" ]; then
  step ${TAG}_trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o run -- \
     python tools/exp_virtual_ranks.py --config cfg3_5m_sh3_4k_f16 --world 8 --frames 3 --stages 0
  find gpurun_out/${TAG}_prof -name "*kernel_stats.csv" -exec cp {} gpurun_out/${TAG}_kernel_stats.csv \; 2>/dev/null
  head -n 30 gpurun_out/${TAG}_kernel_stats.csv
fi
echo "=== done"
