#!/bin/bash
# r05: uncached exchange memory diagnosis: each memory kind in its own process, then
# uncached followed by fine-grained in one process; with DIAG_KEEP=1 no allocation is freed (no reuse of a
# virtual address range).  (tools/exp/mg_uncached_diag.py; pixel checks against the oracle only)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/uc; mkdir -p $O; export TMPDIR=/tmp
for k in ${KINDS:-uc uc_own uc,fine}; do
  t=${k/,/_then_}_keep${DIAG_KEEP:-0}
  timeout -k 10 ${TO:-150} python -u tools/exp/mg_uncached_diag.py ${ROUNDS:-3} $k > $O/$t.log 2>&1
  rc=$?; echo "== $k keep=${DIAG_KEEP:-0} rc=$rc"; grep -v amdgpu.ids $O/$t.log | tail -n 18
  [ $rc -eq 0 ] || exit $rc
done
