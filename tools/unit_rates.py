"""Walk rates of the longest blend units in per-unit traces (exp_virtual_ranks.py --trace-rank npz):
duration, entries walked and ns per entry of the longest units and of the static (first) units.

usage: python tools/unit_rates.py TRACE.npz [TRACE2.npz ...]
"""
import sys

import numpy as np

for f in sys.argv[1:]:
    tr = np.load(f)["trace"].astype(np.int64)
    t0 = tr[:, 0].min()
    start = (tr[:, 0] - t0) * 10.0 / 1e3
    end = (tr[:, 1] - t0) * 10.0 / 1e3
    dur = end - start
    walked = tr[:, 2] & 0xFFFFFFFF
    order = np.argsort(-dur)
    print(f, "units", len(dur), "span", round(float(end.max()), 1))
    for i in order[:8]:
        print(f"  unit {i:6d} start {start[i]:6.1f} dur {dur[i]:6.1f} us walked {walked[i]:5d} "
              f"{1e3 * dur[i] / max(walked[i], 1):6.1f} ns/entry")
    st = start < 1.0
    print("  static units", int(st.sum()), "mean ns/entry", round(float(1e3 * dur[st].sum() / max(walked[st].sum(), 1)), 1),
          "others", round(float(1e3 * dur[~st].sum() / max(walked[~st].sum(), 1)), 1))
