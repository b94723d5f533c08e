"""A/B of the multi-GPU exchange memory kind: the virtual-rank product frame
(tests/test_multigpu_ipc.py _virtual_frame: W renderers of one process, the product kernels, barriers
and gather into rank 0's frame) repeated `rounds` times over three cases and two cameras, each frame
compared with the oracle (colour and gathered depth).  The exchange memory kind comes from the
environment at prepare: GSM_MG_MEM=fine (default) | cached | uncached-ab (uncached memory; the product
refuses GSM_MG_MEM=uncached).

usage: GSM_MG_MEM=uncached-ab python tools/exp/mg_memkind_ab.py [rounds]   -> one line per frame, then
       "bad frames: B of F" (the r03 log profiles/r03_mg_exchange_memory_ab.log came from its predecessor)"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "gsm-renderer_amd")]
import torch  # noqa: E402

import gsm_amd as gsm  # noqa: E402
import oracle as O  # noqa: E402  (checker only)
from gsm_amd import scenes  # noqa: E402
from test_multigpu_ipc import _virtual_frame  # noqa: E402

O.build()
cases = [(2, 40_000, 640, 360, 1), (3, 60_000, 1280, 720, 1), (8, 50_000, 640, 360, 0)]
refs, bad, total = {}, 0, 0
for it in range(int(sys.argv[1]) if len(sys.argv) > 1 else 4):
    for world, n, w, h, prec in cases:
        sh = 16 if prec else 4
        cams = [scenes.make_camera(w, h), scenes.orbit_camera(w, h, 5.0)]
        try:
            frames, counts, timeouts, depths = _virtual_frame(gsm, torch, world, n, w, h, sh, prec, 78, cams)
        except gsm.RendererError as e:  # e.g. a memory kind refused at prepare
            print("refused:", e, flush=True)
            sys.exit(0)
        key = (world, n, w, h, prec)
        if key not in refs:
            wn, hn, _ = scenes.gen_scene(n, w, h, sh, prec, seed=78)
            refs[key] = [O.render(wn, hn, sh, c, w, h, max_gaussians=n) for c in cams]
        for i, (got, gd) in enumerate(zip(frames, depths)):
            ref = refs[key][i]
            rows = np.nonzero(np.any(got != ref["color"], axis=(1, 2)) | np.any(gd != ref["depth"], axis=1))[0]
            total += 1
            bad += bool(len(rows))
            print(it, key, "frame", i, "timeouts", sum(timeouts),
                  "OK" if not len(rows) else f"BAD rows {rows.min()}-{rows.max()} ({len(rows)})", flush=True)
print(f"bad frames: {bad} of {total} (GSM_MG_MEM={os.environ.get('GSM_MG_MEM', 'fine')})", flush=True)
