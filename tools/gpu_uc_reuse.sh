set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for i in 1 2; do
  timeout -k 10 240 python -u tests/mg_uc_reuse.py gpurun_out/uc_$i.json > gpurun_out/uc_$i.log 2>&1 || { echo "run $i failed rc=$?"; tail -20 gpurun_out/uc_$i.log; exit 1; }
  echo "run $i"; grep '^{' gpurun_out/uc_$i.log
done
