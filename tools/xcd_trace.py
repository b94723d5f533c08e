"""Per-XCD summary of a blend trace (tools/blend_trace.py output): units, walked entries, busy time
and last end per XCC id."""
import sys

import numpy as np

tr = np.load(sys.argv[1])["trace"].astype(np.int64)
t0 = tr[:, 0].min()
start = (tr[:, 0] - t0) * 10.0 / 1e3
end = (tr[:, 1] - t0) * 10.0 / 1e3
walked = tr[:, 2] & 0xFFFFFFFF
xcc = (tr[:, 3] >> 48) & 0xFF
for x in range(8):
    m = xcc == x
    print(f"xcc {x}: units {m.sum():5d} walked {walked[m].sum():9d} busy_us {(end - start)[m].sum():9.1f} "
          f"first_start {start[m].min():6.1f} last_end {end[m].max():6.1f}")
