"""Regenerate the committed golden fixtures under tests/golden/.

* radix_kat_seed42.npz / radix_kat_seed123.npz -- the key sets of the reference's
  own radix-sort known-answer tests (Tests/RendererTests/GlobalUnitTests.swift:23-178),
  regenerated from glibc drand48 exactly as the Swift test does
  (tile = UInt32(drand48()*T), depth = Float(drand48()*100) -> Float16 bits ^ 0x8000).
* oracle_digests.json -- sha256 digests of every intermediate and output of the C
  oracle on small scenes (the reference's generateVisibleGaussians/generateGridGaussians
  fixtures and seeded synthetic scenes).  They pin the oracle against regressions and
  are what the GPU parity tests compare against.

Run: python tests/golden/make_golden.py
"""
import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "gsm-renderer_amd"))
import oracle as O  # noqa: E402
from gsm_amd import scenes  # noqa: E402


def radix_keys(seed: int, count: int, tiles: int):
    L = O.lib()
    L.og_srand48(seed)
    keys = np.zeros(count, np.uint32)
    for i in range(count):
        tile = int(L.og_drand48() * tiles)
        depth = np.float32(L.og_drand48() * 100.0)
        keys[i] = L.og_sort_key(tile, L.og_f2h(float(depth)))
    return keys


def digest(a: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def scene(name: str):
    """Inputs for each golden case (shared with tests/test_gpu_parity.py)."""
    if name == "ref_visible_50k_640x360_sh0_f32":
        w, h = O.gen_visible_gaussians(50_000, 42)
        return dict(world=w, harm=h, sh=1, cam=O.make_camera(640, 360), width=640, height=360,
                    max_gaussians=50_000, color_space=0)
    if name == "ref_grid_4096_640x360_sh0_f32":
        w, h = O.gen_grid_gaussians(4096, 42)
        return dict(world=w, harm=h, sh=1, cam=O.make_camera(640, 360), width=640, height=360,
                    max_gaussians=4096, color_space=0)
    if name == "synth_20k_640x360_sh3_f16":
        w, h, cam = scenes.gen_scene(20_000, 640, 360, 16, 1, seed=7)
        return dict(world=w, harm=h, sh=16, cam=cam, width=640, height=360, max_gaussians=20_000,
                    color_space=0)
    if name == "synth_20k_640x360_sh2_f16_srgb":
        w, h, cam = scenes.gen_scene(20_000, 640, 360, 9, 1, seed=8)
        return dict(world=w, harm=h, sh=9, cam=cam, width=640, height=360, max_gaussians=20_000,
                    color_space=1)
    if name == "synth_20k_640x360_sh1_f32":
        w, h, cam = scenes.gen_scene(20_000, 640, 360, 4, 0, seed=9, scale_px=1.5)
        return dict(world=w, harm=h, sh=4, cam=cam, width=640, height=360, max_gaussians=20_000,
                    color_space=0)
    raise KeyError(name)


CASES = ["ref_visible_50k_640x360_sh0_f32", "ref_grid_4096_640x360_sh0_f32",
         "synth_20k_640x360_sh3_f16", "synth_20k_640x360_sh2_f16_srgb", "synth_20k_640x360_sh1_f32"]


def render(name: str) -> dict:
    s = scene(name)
    return O.render(s["world"], s["harm"], s["sh"], s["cam"], s["width"], s["height"],
                    max_gaussians=s["max_gaussians"], color_space=s["color_space"])


def frame_digests(r: dict) -> dict:
    vis = r["mask"].astype(bool)
    return {
        "visible": int(r["visible"]), "total_assignments": int(r["total_assignments"]),
        "overflow": int(r["overflow"]), "active_tiles": int(r["active_tiles"]),
        "render_data_visible": digest(r["render_data"][vis]), "bounds": digest(r["bounds"]),
        "tile_counts": digest(r["tile_counts"]), "keys": digest(r["keys"]),
        "values": digest(r["values"]), "sorted_keys": digest(r["sorted_keys"]),
        "sorted_values": digest(r["sorted_values"]), "headers": digest(r["headers"]),
        "color": digest(r["color"]), "depth": digest(r["depth"]),
    }


def main():
    k42 = radix_keys(42, 1024, 10)
    np.savez_compressed(os.path.join(HERE, "radix_kat_seed42.npz"), keys=k42)
    k123 = radix_keys(123, 50_000, 100)
    np.savez_compressed(os.path.join(HERE, "radix_kat_seed123.npz"), keys=k123)
    out = {}
    for name in CASES:
        out[name] = frame_digests(render(name))
        print(name, out[name]["visible"], out[name]["total_assignments"], out[name]["overflow"])
    with open(os.path.join(HERE, "oracle_digests.json"), "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
