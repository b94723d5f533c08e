set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for a in "2632483 28" "2632483 32" "13000000 30" "1000000 16"; do
  timeout -k 10 120 ./tools/exp/rocprim_sort_probe $a >> gpurun_out/rocprim_probe.log 2>&1; rc=$?; echo "probe $a rc=$rc"
  [ $rc -eq 0 ] || exit $rc
done
cat gpurun_out/rocprim_probe.log
