"""Debug: repeat the virtual-rank product frame and report mismatching rows/pixels."""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "gsm-renderer_amd")]
import torch
import gsm_amd as gsm
import oracle as O
from gsm_amd import scenes
from test_multigpu_ipc import _virtual_frame
O.build()
cases = [(2, 40_000, 640, 360, 1), (3, 60_000, 1280, 720, 1), (8, 50_000, 640, 360, 0)]
refs = {}
for it in range(int(sys.argv[1]) if len(sys.argv) > 1 else 4):
    for world, n, w, h, prec in cases:
        sh = 16 if prec else 4
        cams = [scenes.make_camera(w, h), scenes.orbit_camera(w, h, 5.0)]
        frames, counts, timeouts = _virtual_frame(gsm, torch, world, n, w, h, sh, prec, 78, cams)
        key = (world, n, w, h, prec)
        if key not in refs:
            wn, hn, _ = scenes.gen_scene(n, w, h, sh, prec, seed=78)
            refs[key] = [O.render(wn, hn, sh, c, w, h, max_gaussians=n)["color"] for c in cams]
        for i, got in enumerate(frames):
            ref = refs[key][i]
            badpx = np.any(got != ref, axis=2)
            rows = np.nonzero(badpx.any(axis=1))[0]
            msg = ""
            if len(rows):
                ys, xs = np.nonzero(badpx)
                msg = (f" rows {rows.min()}-{rows.max()} ({len(rows)}), px {len(ys)}, cols {xs.min()}-{xs.max()},"
                       f" sample got {got[ys[0], xs[0]].tolist()} ref {ref[ys[0], xs[0]].tolist()}")
            print(it, key, "frame", i, "timeouts", sum(timeouts), "OK" if not len(rows) else "BAD" + msg, flush=True)
