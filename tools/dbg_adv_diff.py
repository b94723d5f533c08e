"""Diagnostic (r06): an adversarial scene of tests/test_gpu_parity.py rendered on the GPU and by the oracle;
the first gaussians whose render data / bounds / tile counts differ, with their inputs.
usage: python tools/dbg_adv_diff.py KIND N W H SH SEED"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "gsm-renderer_amd")]
import torch  # noqa: E402

import adversarial  # noqa: E402
import gsm_amd as gsm  # noqa: E402
import oracle as O  # noqa: E402
from test_gpu_parity import gpu_render, oracle_render  # noqa: E402

kind, n, w, h, sh, seed = sys.argv[1], *map(int, sys.argv[2:7])
O.build()
case = adversarial.scene(kind, n, w, h, sh, seed, False)
r = oracle_render(O, case)
g = gpu_render(gsm, torch, case)
print("assignments gpu", g["counters"]["total_assignments"], "oracle", r["total_assignments"])
for name in ("bounds", "tile_counts", "render_data"):
    a = np.asarray(g[name]).reshape(len(case["world"]), -1) if name != "render_data" else None
    if name == "render_data":
        vis = r["mask"].astype(bool)
        ga = g["render_data"][vis].view(np.uint8).reshape(int(vis.sum()), -1)
        ra = r["render_data"][vis].view(np.uint8).reshape(int(vis.sum()), -1)
        ids = np.nonzero(vis)[0]
        bad = np.nonzero(np.any(ga != ra, axis=1))[0]
        print("render_data: differing gaussians", len(bad))
        for i in bad[:6]:
            print("  gid", int(ids[i]), "gpu", ga[i].view(np.uint16).tolist(), "oracle", ra[i].view(np.uint16).tolist())
            print("    world", case["world"][ids[i]])
        continue
    ra = np.asarray(r[name]).reshape(len(case["world"]), -1)
    bad = np.nonzero(np.any(a != ra, axis=1))[0]
    print(name, ": differing gaussians", len(bad))
    for i in bad[:6]:
        print("  gid", int(i), "gpu", a[i].tolist(), "oracle", ra[i].tolist(), "world", case["world"][i])
