"""Per-frame GPU timeline from a rocprofv3 kernel trace of bench.py: frames start at each projection
launch (k_project / k_records_in / k_project_part); for the median frame prints every kernel's
start offset and duration, the sum of kernel time and the idle gaps between launches.
usage: python tools/timeline.py <kernel_trace.csv>"""
import csv
import statistics
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
frames, cur = [], []
for r in rows:
    name = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("gsm::", "")
    if name.startswith("k_project") and not name.startswith("k_project_part") and cur:
        frames.append(cur)
        cur = []
    cur.append((name, int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
if cur:
    frames.append(cur)
frames = [f for f in frames if any(n.startswith("k_blend") for n, _, _ in f)]
spans = []
for f in frames:
    t0, t1 = f[0][1], max(e for _, _, e in f)
    busy = sum(e - s for _, s, e in f)
    spans.append((t1 - t0, busy, f))
spans.sort(key=lambda x: x[0])
span, busy, f = spans[len(spans) // 2]
print(f"frames {len(spans)}; median span {span/1e3:.1f} us, kernel time {busy/1e3:.1f} us, gaps {(span-busy)/1e3:.1f} us")
t0 = f[0][1]
prev_end = t0
for n, s, e in f:
    print(f"  {(s - t0)/1e3:7.1f} +{(e - s)/1e3:6.1f}  gap {(s - prev_end)/1e3:5.1f}  {n[:60]}")
    prev_end = max(prev_end, e)
