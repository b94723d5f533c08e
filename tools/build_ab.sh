#!/bin/bash
# A/B builds of libgsm_amd.so: `bash tools/build_ab.sh name1="-DX=1" name2="-DY=0" [head]` builds each named
# variant of the working tree into gsm-renderer_amd/lib_ab_<name> (only $ABSRC, default gsm_kernels gsm_sort,
# recompiled), and
# `head` the committed tree (git HEAD) into lib_ab_head.  Run the variants with GSM_AMD_LIB=<dir>/libgsm_amd.so.
set -eu
cd "$(dirname "$0")/../gsm-renderer_amd"
make -s -j8
for arg in "$@"; do
  if [ "$arg" = head ]; then
    t=$(mktemp -d); (cd .. && git archive HEAD include gsm-renderer_amd/Makefile gsm-renderer_amd/csrc) | tar -x -C "$t"
    make -s -C "$t/gsm-renderer_amd" -j8 && rm -rf lib_ab_head && mkdir -p lib_ab_head && cp "$t/gsm-renderer_amd/lib/libgsm_amd.so" lib_ab_head/
    rm -rf "$t"; continue
  fi
  name=${arg%%=*}; extra=${arg#*=}
  rm -rf build_ab_$name lib_ab_$name; mkdir -p build_ab_$name
  cp -p build/*.o build_ab_$name/; for f in ${ABSRC:-gsm_kernels gsm_sort}; do rm -f build_ab_$name/$f.o; done
  make -s BUILD=build_ab_$name LIB=lib_ab_$name EXTRA="$extra" &
done
wait
ls -la lib_ab_*/libgsm_amd.so
