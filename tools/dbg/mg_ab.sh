#!/bin/bash
# failure rate of the virtual-rank frame (tools/dbg/mg_dbg2.py) per library variant
for v in lib lib_pd lib_rd lib_bd; do
  echo "== $v"
  GSM_AMD_LIB=$PWD/gsm-renderer_amd/$v/libgsm_amd.so timeout -k 10 200 python tools/dbg/mg_dbg2.py 6 2>&1 | grep -c BAD
done
