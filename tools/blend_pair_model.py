"""Cost model of walking two blend units per wave (8 pixels per lane = one 4x2 group per lane, the two
units' groups on the two half-waves), against the measured per-unit alive curves of the current kernel
(tools/blend_curves.py, GSM_BLEND_ZSTATS=2 build).

Per walked entry, wave-instructions of the three lane layouts (ISA of k_blend_px):
  8 px / lane (64 groups):  quadratic form 25, table addressing 8, joins 4, alpha 12, blend 24, break 5 = 78
  4 px / lane (32 groups):  42.6 (the current half-tile walk)
  2 px / lane (16 groups):  38   (the current compacted walk)
Current: each unit alone, 4 px / lane until the checkpoint (every 16 entries) where at most 16 of its 32
groups live, then 2 px / lane.  Pairs: units paired in longest-first order (the schedule's), 8 px / lane
while more than 32 of the pair's 64 groups live, 4 px / lane while more than 16, then 2 px / lane; the
`--singles` longest units run alone as now.  Prints the total wave-instructions of both, the longest job.

usage: python tools/blend_pair_model.py gpurun_out/blend_curves_cfg2_1m_sh3_1080p_f16_0.npz [--singles 1024]
"""
import argparse
import json

import numpy as np

C8, C4, C2 = 78.0, 42.6, 38.0


def alive_at(thr_e, thresholds, e):
    """groups alive after entry e (step function from the threshold crossings; 32 before the first)"""
    a = 32
    for t, ee in zip(thresholds, thr_e):
        if ee <= e:
            a = min(a, t)
    return a


def unit_checkpoints(walk):
    return list(range(16, walk + 16, 16))


def cost_single(w, thr_e, thresholds):
    c, comp = 0.0, False
    for cp in unit_checkpoints(w):
        c += 16 * (C2 if comp else C4)
        if not comp and alive_at(thr_e, thresholds, cp - 1) <= 16:
            comp = True
    return c


def cost_pair(wu, tu, wv, tv, thresholds):
    w = max(wu, wv)
    c, layout = 0.0, 8
    for cp in unit_checkpoints(w):
        c += 16 * {8: C8, 4: C4, 2: C2}[layout]
        a = (alive_at(tu, thresholds, cp - 1) if cp <= wu else 0) + (alive_at(tv, thresholds, cp - 1) if cp <= wv else 0)
        if layout == 8 and a <= 32:
            layout = 4
        if layout == 4 and a <= 16:
            layout = 2
    return c


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("npz")
    ap.add_argument("--singles", type=int, default=1024)
    args = ap.parse_args()
    d = np.load(args.npz)
    walked, thr, thresholds = d["walked"], d["thr"], list(d["thresholds"])
    order = np.argsort(-walked, kind="stable")
    cur = [cost_single(int(walked[i]), thr[i], thresholds) for i in range(len(walked))]
    total_cur = float(np.sum(cur))
    new, jobs = 0.0, []
    for i in order[:args.singles]:
        new += cur[i]
        jobs.append(cur[i])
    rest = order[args.singles:]
    for k in range(0, len(rest), 2):
        u = rest[k]
        if k + 1 < len(rest):
            v = rest[k + 1]
            c = cost_pair(int(walked[u]), thr[u], int(walked[v]), thr[v], thresholds)
        else:
            c = cur[u]
        new += c
        jobs.append(c)
    print(json.dumps({"units": int(len(walked)), "walked": int(walked.sum()), "current_Minst": round(total_cur / 1e6, 2),
                      "pairs_Minst": round(new / 1e6, 2), "ratio": round(new / total_cur, 3),
                      "singles": args.singles, "jobs": len(jobs),
                      "longest_job_current_kinst": round(max(cur) / 1e3, 1),
                      "longest_pair_job_kinst": round(max(jobs[args.singles:] or [0]) / 1e3, 1)}))


if __name__ == "__main__":
    main()
