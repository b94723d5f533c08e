"""Load balance of the multi-GPU tile-row split (SURVEY.md 8e leaves contiguous vs interleaved row
blocks to measurement): per tile row, the oracle's assignments (sort + scatter work) and blend
group iterations (`group_iters`, the walk lengths of the reference's 4x2 groups: blend work), summed
over the rows each of W ranks would own under three splits --
  contiguous : rank r owns rows [r * ceil(T / W), ...) (the product's split, gsm_multigpu.h)
  interleaved: rank r owns rows r, r + W, r + 2W, ...
  adaptive   : contiguous blocks cut where the cumulative load of the previous frame crosses k / W
and reports max / mean over ranks (1.0 = perfect balance) for a uniform scene (BASELINE config 2's
generator) on the orbit camera path and for a non-uniform one (the same cloud with most gaussians
squeezed into the lower third of the view).  CPU only (the C oracle).

    python tools/slab_balance.py [--count N] [--out profiles/r03_slab_balance.json]
"""
import argparse
import json
import math
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gsm-renderer_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle as O  # noqa: E402
from gsm_amd import scenes  # noqa: E402


def row_loads(fr):
    tx, ty = fr["tiles_x"], fr["tiles_y"]
    assign = fr["headers"][:, 1].astype(np.int64).reshape(ty, tx).sum(1)
    blend = fr["group_iters"].astype(np.int64).reshape(ty, tx, -1).sum((1, 2))
    return assign, blend


def splits(ty, w, prev_load):
    per = math.ceil(ty / w)
    contiguous = [list(range(r * per, min(ty, (r + 1) * per))) for r in range(w)]
    interleaved = [list(range(r, ty, w)) for r in range(w)]
    cyclic = {b: [[y for y in range(ty) if (y // b) % w == r] for r in range(w)] for b in (2, 4)}
    cum = np.cumsum(prev_load) / max(prev_load.sum(), 1)
    cuts = [0] + [int(np.searchsorted(cum, k / w)) + 1 for k in range(1, w)] + [ty]
    cuts = np.maximum.accumulate(np.minimum(cuts, ty))
    adaptive = [list(range(cuts[r], cuts[r + 1])) for r in range(w)]
    return {"contiguous": contiguous, "interleaved": interleaved, "cyclic2": cyclic[2], "cyclic4": cyclic[4],
            "adaptive": adaptive}


def records(fr, parts):
    """(gaussian, rank) records the exchange moves: a gaussian with tiles goes to every rank owning a
    row of its rect (the rect rows bound the rows its tile tests hit)"""
    b = fr["bounds"]
    live = fr["tile_counts"] > 0
    y0, y1 = b[live, 2], b[live, 3]
    owner = np.full(fr["tiles_y"], -1)
    for r, rows in enumerate(parts):
        owner[rows] = r
    tot = 0
    for r in range(len(parts)):
        mine = np.zeros(fr["tiles_y"] + 1, np.int64)
        mine[1:] = np.cumsum(owner == r)
        tot += int(np.count_nonzero(mine[y1 + 1] - mine[y0] > 0))
    return tot


def imbalance(load, parts):
    s = np.array([load[p].sum() if p else 0 for p in parts], np.float64)
    return round(float(s.max() / max(s.mean(), 1e-9)), 3)


def skewed_scene(n, w, h, seed):
    world, harm, cam = scenes.gen_scene(n, w, h, 16, 1, seed)
    rng = np.random.default_rng(seed + 1)
    z = world["pz"].astype(np.float32)
    # 80 % of the cloud in the lower third of the view (screen y grows downwards: world y > 0 here
    # maps below the centre with this projection), the rest uniform
    sel = rng.random(n) < 0.8
    world["py"][sel] = (rng.uniform(0.2, 0.6, sel.sum()) * z[sel]).astype(np.float32)
    return world, harm, cam


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--count", type=int, default=1_000_000)
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    n, W, H = a.count, a.width, a.height
    out = {"count": n, "width": W, "height": H, "note": __doc__.split("\n\n")[0].replace("\n", " "), "cases": []}
    scenes_ = {"uniform": scenes.gen_scene(n, W, H, 16, 1, 42), "lower_third": skewed_scene(n, W, H, 42)}
    for sname, (world, harm, _) in scenes_.items():
        prev = None
        for ang in (0.0, 0.25, 13.75, 30.0):
            cam = scenes.orbit_camera(W, H, ang)
            fr = O.render(world, harm, 16, cam, W, H, max_gaussians=n)
            assign, blend = row_loads(fr)
            ref = prev if prev is not None else blend  # the adaptive cut uses the previous view's blend load
            case = {"scene": sname, "orbit_deg": ang, "assignments": int(assign.sum()), "by_world": {}}
            for w in (2, 4, 8):
                sp = splits(fr["tiles_y"], w, ref)
                case["by_world"][w] = {k: {"assign": imbalance(assign, v), "blend": imbalance(blend, v),
                                           "records": records(fr, v)} for k, v in sp.items()}
            out["cases"].append(case)
            print(json.dumps(case))
            prev = blend
    if a.out:
        with open(a.out, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
