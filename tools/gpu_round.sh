#!/bin/bash
# Round artefacts on one MI355X: GPU parity tests, smoke, bench lines (configs 2, 3, 5), the
# rocprofv3 kernel-trace summary of the default bench, PMC passes and the blend's HBM traffic.
# Everything lands in gpurun_out/round/; copy what is judged into profiles/ (tools/round_copy.sh).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/round
mkdir -p $OUT
export TMPDIR=/tmp
step() {  # name timeout cmd...   (stdout+stderr -> $OUT/name.log; crash/timeout ends the script)
  local name=$1 to=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "--- $name rc=$rc"; tail -n 3 "$OUT/$name.log"
  if [ $rc -ne 0 ]; then echo "ABORT after $name (rc=$rc)"; exit $rc; fi
}
step pytest_gpu 600 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
CMD="python bench.py --steps 10 --warmup 3 --cpu-baseline 0 --parity 0"
i=0
for set in "FETCH_SIZE" "WRITE_SIZE" \
           "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM"; do
  i=$((i+1))
  step pmc$i 120 rocprofv3 --pmc $set --output-format csv -d $OUT/pmc/p$i -o p$i -- $CMD
done
python tools/pmc_summary.py $OUT/pmc > $OUT/pmc_summary.txt
python tools/traffic.py $OUT/pmc > $OUT/traffic.json
cat $OUT/traffic.json
step bench_cfg2 600 python bench.py --traffic-json $OUT/traffic.json
step bench_cfg3 600 python bench.py --traffic-json $OUT/traffic.json --config cfg3_5m_sh3_4k_f16 --steps 30 --warmup 3
step bench_cfg5 600 python bench.py --traffic-json $OUT/traffic.json --config cfg5_1m_sh2_stereo_2x1440x1600_f16 --steps 30 --warmup 3
step bench_cfg5_global 600 python bench.py --traffic-json $OUT/traffic.json --config cfg5_1m_sh2_stereo_2x1440x1600_f16 --steps 30 --warmup 3 --stereo-path global --cpu-baseline 0
step kernel_trace_cfg5 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt5 -o run -- \
     python bench.py --config cfg5_1m_sh2_stereo_2x1440x1600_f16 --steps 30 --warmup 5 --cpu-baseline 0 --parity 0
step kernel_trace 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o run -- \
     python bench.py --traffic-json $OUT/traffic.json --steps 50 --warmup 5 --cpu-baseline 0 --parity 0
echo "=== done"
