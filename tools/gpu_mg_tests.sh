# The multi-GPU GPU tests alone (processes on one GPU, virtual ranks, RCCL set-up).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${OUT:-mgt}
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_multigpu_ipc.py tests/test_multigpu_rccl.py > $O/pytest_mg.log 2>&1 || { tail -40 $O/pytest_mg.log | cut -c1-300; exit 1; }
tail -1 $O/pytest_mg.log
