#!/bin/bash
# r06: the whole GPU suite, then kernel traces of configs 2 and 3 (k_project and the frame) and one PMC pass
# of k_project's instruction counts.  Each step under its own time limit; a failure ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ "${TESTS:-1}" = 1 ]; then
  timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
  rc=$?; echo "pytest rc=$rc: $(tail -n 1 gpurun_out/pytest_gpu.log)"
  [ $rc -eq 0 ] || { grep -E "^FAILED|Error|error" gpurun_out/pytest_gpu.log | head -20; grep -B5 -A40 "^_____" gpurun_out/pytest_gpu.log | head -120; exit $rc; }
fi
CFGS=${CFGS:-cfg2_1m_sh3_1080p_f16 cfg3_5m_sh3_4k_f16} bash tools/kt.sh > gpurun_out/kt_summary.txt 2>&1 || { tail -20 gpurun_out/kt_summary.txt; exit 1; }
grep -E "cfg|k_project<|k_radix_down|k_tile_sort|k_blend|k_scatter|fps" gpurun_out/kt_summary.txt
rm -rf gpurun_out/pmc_proj
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE \
  --output-format csv -d gpurun_out/pmc_proj -o p -- python bench.py --steps 5 --warmup 2 --cpu-baseline 0 --parity 0 --orbit-steps 0 --inflight-steps 0 --virtual-ranks 0 \
  > gpurun_out/pmc_proj.log 2>&1 || { echo "pmc failed"; tail -5 gpurun_out/pmc_proj.log; exit 1; }
python3 tools/pmc_summary.py gpurun_out/pmc_proj | grep -A9 "k_project<true, 3>"
echo "=== done"
