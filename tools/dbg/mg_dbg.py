"""Debug: which rows / slabs of the virtual-rank multi-GPU frame differ from the oracle."""
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
for world, n, w, h, prec, seed in [(8, 50_000, 640, 360, 0, 78), (8, 50_000, 640, 360, 1, 78), (4, 50_000, 640, 360, 0, 78), (8, 20_000, 640, 360, 0, 5)]:
    sh = 16 if prec else 4
    cams = [scenes.make_camera(w, h), scenes.orbit_camera(w, h, 5.0)]
    frames, counts, timeouts = _virtual_frame(gsm, torch, world, n, w, h, sh, prec, seed, cams)
    wn, hn, _ = scenes.gen_scene(n, w, h, sh, prec, seed=seed)
    for i, (got, cam) in enumerate(zip(frames, cams)):
        ref = O.render(wn, hn, sh, cam, w, h, max_gaussians=n)
        bad = np.nonzero(np.any(got != ref["color"], axis=(1, 2)))[0]
        print(world, prec, seed, "cam", i, "timeouts", timeouts, "bad rows", len(bad), bad[:20], bad[-5:] if len(bad) else "", flush=True)
