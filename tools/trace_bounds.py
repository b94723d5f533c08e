"""Bounds of a blend from its per-unit trace (tools/blend_trace.py's npz): the span, the longest unit,
the work bound (sum of unit durations over the wave slots), the LPT makespan of the measured unit
durations on that many identical slots, the slot occupancy over time and how the span splits into the
static phase, the dynamic phase and the tail (fewer than half the slots busy).

usage: python tools/trace_bounds.py gpurun_out/blend_trace_cfg2_1m_sh3_1080p_f16_0.npz [slots]
"""
import heapq
import json
import sys

import numpy as np


def main():
    tr = np.load(sys.argv[1])["trace"].astype(np.int64)
    slots = int(sys.argv[2]) if len(sys.argv) > 2 else 3072
    t0 = tr[:, 0].min()
    start = (tr[:, 0] - t0) * 10.0 / 1e3  # us
    end = (tr[:, 1] - t0) * 10.0 / 1e3
    dur = end - start
    walked = tr[:, 2] & 0xFFFFFFFF
    span = end.max()
    work = dur.sum() / slots
    # LPT on identical slots over the measured durations
    heap = [0.0] * slots
    for d in np.sort(dur)[::-1]:
        t = heapq.heappop(heap)
        heapq.heappush(heap, t + d)
    lpt = max(heap)
    grid = np.linspace(0, span, 401)
    occ = np.array([((start <= x) & (end > x)).sum() for x in grid[:-1]])
    half = np.nonzero(occ < slots // 2)[0]
    tail_start = grid[half[0]] if len(half) else span
    order = np.argsort(-dur)
    out = {
        "units": int(len(dur)), "span_us": round(float(span), 1), "longest_unit_us": round(float(dur.max()), 1),
        "longest_walk": int(walked[order[0]]), "work_bound_us": round(float(work), 1), "lpt_us": round(float(lpt), 1),
        "busy_frac": round(float(dur.sum() / (span * slots)), 3),
        "tail_start_us (occupancy < half)": round(float(tail_start), 1),
        "occupancy_deciles": [int(occ[i]) for i in range(0, 400, 40)],
        "ns_per_entry_longest10": [round(float(dur[i] * 1e3 / max(1, walked[i])), 1) for i in order[:10]],
        "walks_longest10": [int(walked[i]) for i in order[:10]],
        "start_of_longest10_us": [round(float(start[i]), 1) for i in order[:10]],
        "units_ending_last10": [(round(float(start[i]), 1), round(float(dur[i]), 1), int(walked[i]))
                                for i in np.argsort(-end)[:10]],
    }
    print(json.dumps(out))


if __name__ == "__main__":
    main()
