"""Entry throughput over time from a blend trace (tools/blend_trace.py output)."""
import sys
import numpy as np

for path in sys.argv[1:]:
    tr = np.load(path)["trace"].astype(np.int64)
    t0 = tr[:, 0].min()
    s = (tr[:, 0] - t0) * 10 / 1000
    e = (tr[:, 1] - t0) * 10 / 1000
    w = tr[:, 2] & 0xFFFFFFFF
    d = e - s
    print(path)
    step = max(5.0, e.max() / 30)
    for a in np.arange(0, e.max(), step):
        b = a + step
        ov = np.clip(np.minimum(e, b) - np.maximum(s, a), 0, None)
        frac = np.where(d > 0, ov / np.maximum(d, 1e-9), 0)
        ent = (frac * w).sum()
        occ = ov.sum() / step
        print("  t=%6.0f occ=%6.0f entries/us=%7.0f per-wave entries/ms=%6.1f" % (a, occ, ent / step, ent / step / max(occ, 1) * 1000))
    o = np.argsort(-d)[:5]
    for i in o:
        print(f"  long unit {i} start {s[i]:.1f} dur {d[i]:.1f} walked {w[i]} count {tr[i,2]>>32}")
