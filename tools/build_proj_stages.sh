#!/bin/bash
# Builds the GSM_PROJ_STOP variants of libgsm_amd.so (gsm-renderer_amd/lib_ps<k>) from the default build's
# objects: only gsm_kernels.hip is recompiled per variant.
set -eu
cd "$(dirname "$0")/../gsm-renderer_amd"
# the stop macros live in a patch (not in the product): git apply tools/exp/proj_stop.patch first
grep -q GSM_PROJ_STOP csrc/gsm_kernels.hip || { echo "apply tools/exp/proj_stop.patch first (git apply)"; exit 1; }
make -s -j8
for k in ${STOPS:-1 2 3 4 5 6 7 8}; do
  rm -rf build_ps$k lib_ps$k; mkdir -p build_ps$k
  cp -p build/*.o build_ps$k/; rm build_ps$k/gsm_kernels.o
  make -s BUILD=build_ps$k LIB=lib_ps$k EXTRA=-DGSM_PROJ_STOP=$k &
done
wait
ls -la lib_ps*/libgsm_amd.so
