#!/bin/bash
# failure rate of the virtual-rank frame (tools/dbg/mg_dbg2.py: 6 rounds x 3 cases x 2 frames) per
# exchange-memory kind (GSM_MG_MEM, create-time)
for m in fine uncached cached; do
  echo "== $m: bad frames of 36"
  GSM_MG_MEM=$m timeout -k 10 200 python tools/dbg/mg_dbg2.py 6 2>&1 | grep -c BAD
done
exit 0
