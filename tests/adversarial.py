"""Adversarial splat scenes for the GPU parity tests (test_adversarial_scenes_bit_exact): ordinary
gaussians mixed with the inputs the projection, the tile tests, the sort and the blend have edge
paths for -- extreme and zero scales, zero / huge / tiny quaternions, positions at the camera, on the
near plane, behind it, past fp16's depth range, inf and NaN coordinates, opacities at and around the
cull threshold or outside [0, 1] or NaN, huge / negative / NaN SH coefficients.  The oracle is the
judge of what each should produce; the GPU must match it bit for bit.  (Test data only.)"""
import numpy as np


def scene(kind, n, width, height, sh, seed, overflow=False):
    import sys
    import os
    here = os.path.dirname(os.path.abspath(__file__))
    root = os.path.dirname(here)
    for p in (root, os.path.join(root, "oracle"), os.path.join(root, "gsm-renderer_amd")):
        if p not in sys.path:
            sys.path.insert(0, p)
    from gsm_amd import scenes
    from gsm_amd.types import WORLD32, WORLD16
    prec = 1 if kind == "f16" else 0
    w, h, cam = scenes.gen_scene(n, width, height, sh, prec, seed=seed)
    rng = np.random.default_rng(seed + 1000)
    k = max(sh, 1)
    m = n // 4  # a quarter of the gaussians get an edge value (one field each, a few fields per gaussian)
    idx = rng.choice(n, m, replace=False)
    f32 = lambda v: np.asarray(v, np.float32)
    pos_vals = f32([0.0, 1e-7, 0.1, 0.1000001, -1.0, 5e4, 7e4, 1e6, 1e30, np.inf, -np.inf, np.nan])
    scale_vals = f32([0.0, 1e-7, 5e-4, 4.9e-4, 1e-3, 2.0, 50.0, 1e3, 6e4, 1e6, np.inf, np.nan, -0.5])
    rot_vals = f32([0.0, 1e-20, 1e-9, 1e6, -3.0, np.nan, np.inf])
    op_vals = f32([0.0, 0.005, 0.004999, 0.0051, 1.0, 1.5, 255.0, -0.5, np.nan])
    harm_vals = f32([0.0, -5.0, 1e3, 6e4, 1e8, np.inf, np.nan])
    h = h.reshape(n, -1)
    for j, g in enumerate(idx):
        r = rng.integers(0, 6)
        if r == 0:  # position: z (near plane 0.1 in make_camera), x, y
            axis = ["px", "py", "pz"][rng.integers(0, 3)]
            v = pos_vals[rng.integers(0, len(pos_vals))]
            w[axis][g] = v if axis != "pz" or rng.random() < 0.5 else np.float32(abs(v)) if np.isfinite(v) else v
        elif r == 1:  # scale (values >= 2 -- rects of hundreds or thousands of tiles -- for 1 in 50)
            big = rng.random() < 0.02
            for axis in ("sx", "sy", "sz"):
                if rng.random() < 0.5:
                    v = scale_vals[rng.integers(0, len(scale_vals))]
                    if not big and np.isfinite(v) and v >= 2.0:
                        v = np.float32(v * 1e-4)
                    w[axis][g] = v if prec == 0 else np.float16(v).view(np.uint16)
        elif r == 2:  # rotation
            if prec == 0:
                q = w["rot"][g].copy()
                q[rng.integers(0, 4)] = rot_vals[rng.integers(0, len(rot_vals))]
                if rng.random() < 0.3:
                    q[:] = 0.0
                w["rot"][g] = q
            else:
                for axis in ("rx", "ry", "rz", "rw"):
                    if rng.random() < 0.4:
                        w[axis][g] = np.float16(rot_vals[rng.integers(0, len(rot_vals))]).view(np.uint16)
        elif r == 3:  # opacity
            v = op_vals[rng.integers(0, len(op_vals))]
            w["opacity"][g] = v if prec == 0 else np.float16(v).view(np.uint16)
        elif r == 4:  # SH coefficients
            c = rng.integers(0, h.shape[1])
            v = harm_vals[rng.integers(0, len(harm_vals))]
            h[g, c] = v if prec == 0 else np.float16(v).view(np.uint16)
        elif rng.random() < 0.05:  # a large, close, opaque gaussian (huge tile rects, long lists)
            w["pz"][g] = np.float32(rng.uniform(0.3, 1.0))
            for axis in ("sx", "sy", "sz"):
                v = np.float32(rng.uniform(0.005, 0.03))
                w[axis][g] = v if prec == 0 else np.float16(v).view(np.uint16)
    # overflow=False: room for every assignment (max_gaussians sets the 4x cap); True: the reference's cap
    return dict(world=w, harm=h.reshape(-1), sh=sh, cam=cam, width=width, height=height,
                max_gaussians=n if overflow else 4 * n)
