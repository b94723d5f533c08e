#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/dbg_adv_diff.py f32 20000 640 360 16 5 > gpurun_out/dbg_adv.txt 2>&1; echo rc=$?
cat gpurun_out/dbg_adv.txt | tail -40
