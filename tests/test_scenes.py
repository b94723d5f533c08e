"""Synthetic scene generator used by the benchmark."""
import numpy as np

from gsm_amd import scenes
from gsm_amd.types import WORLD16, WORLD32


def test_scene_layouts_and_determinism():
    w, h, cam = scenes.gen_scene(1000, 1920, 1080, 16, 1, seed=3)
    assert w.dtype == WORLD16 and w.dtype.itemsize == 32
    assert h.dtype == np.uint16 and h.size == 1000 * 16 * 3
    w2, h2, _ = scenes.gen_scene(1000, 1920, 1080, 16, 1, seed=3)
    assert w.tobytes() == w2.tobytes() and h.tobytes() == h2.tobytes()
    w, h, cam = scenes.gen_scene(500, 640, 360, 1, 0, seed=3)
    assert w.dtype == WORLD32 and w.dtype.itemsize == 48 and h.dtype == np.float32
    assert cam["proj"].shape == (16,) and cam["proj"][11] == 1.0


def test_scene_density_stays_inside_capacity(oracle):
    w, h, cam = scenes.gen_scene(30_000, 1920, 1080, 16, 1, seed=5)
    r = oracle.render(w, h, 16, cam, 1920, 1080, max_gaussians=30_000)
    assert r["overflow"] == 0
    assert 2.0 < r["total_assignments"] / 30_000 < 3.5
