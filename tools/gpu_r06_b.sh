#!/bin/bash
# r06: the freed-uncached reuse child twice (mapping check), the correctly rounded sqrt / reciprocal check over
# every 32-bit input, and the extended VALU issue probe.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 120 tools/exp/crmath_check > gpurun_out/crmath_check.txt 2>&1 || { echo "crmath failed"; tail gpurun_out/crmath_check.txt; exit 1; }
cat gpurun_out/crmath_check.txt
for i in 1 2; do
  timeout -k 10 240 python -u tests/mg_uc_reuse.py gpurun_out/uc_$i.json > gpurun_out/uc_$i.log 2>&1 || { echo "uc run $i failed rc=$?"; tail -20 gpurun_out/uc_$i.log; exit 1; }
  echo "uc run $i"; grep '^{' gpurun_out/uc_$i.log | cut -c1-300
done
timeout -k 10 300 tools/exp/valu_peak > gpurun_out/valu_peak_r06.txt 2>&1 || { echo "valu_peak failed"; exit 1; }
grep -E "waves/SIMD=(4|8)" gpurun_out/valu_peak_r06.txt | tail -12
