"""Synthetic Gaussian clouds and cameras for the benchmark configs.

Modelled on the reference's fixture generator generateVisibleGaussians
(Tests/RendererTests/TestUtils.swift:189-231: z ~ U[1.5, 9.5], x,y ~ U[-1,1]*0.6z,
opacity ~ U[0.5,1]) and camera makeProjectionMatrix/makeCameraParams
(TestUtils.swift:37-94: 60 deg fov, near 0.1, far 10, OpenCV +Z forward, identity
view).  The scale is changed for density: log-uniform scales tuned so a
frame has ~2.6 tile assignments per gaussian at every resolution (measured with the
oracle: scale_px 0.8/1.0/1.2/1.5 -> A/N 1.99/2.30/2.62/3.13), inside the reference's
4*N assignment capacity and its 16.78M radix-sort limit at 5M/4K.  Quaternions are random unit vectors, SH DC ~ U[0,1] and
higher bands ~ N(0, 0.1) clipped to +-0.3.  numpy PCG64, seeded.
"""
from __future__ import annotations

import math

import numpy as np

from .types import WORLD16, WORLD32


def projection_matrix(width: int, height: int, near: float = 0.1, far: float = 10.0,
                      fov_degrees: float = 60.0) -> np.ndarray:
    """makeProjectionMatrix, OpenCV convention (TestUtils.swift:37-71), column-major flat."""
    aspect = np.float32(width) / np.float32(height)
    fov = np.float32(fov_degrees) * np.float32(math.pi) / np.float32(180.0)
    f = np.float32(1.0) / np.float32(math.tan(float(fov) / 2.0))
    P = np.zeros(16, np.float32)
    P[0] = f / aspect
    P[5] = f
    P[10] = np.float32(far) / (np.float32(far) - np.float32(near))
    P[11] = 1.0
    P[14] = -(np.float32(far) * np.float32(near)) / (np.float32(far) - np.float32(near))
    return P


def make_camera(width: int, height: int, eye_offset_x: float = 0.0) -> dict:
    """makeCameraParams (TestUtils.swift:74-94); eye_offset_x shifts the camera for stereo."""
    P = projection_matrix(width, height)
    V = np.eye(4, dtype=np.float32).reshape(-1)  # column-major identity
    V[12] = -np.float32(eye_offset_x)            # translation column (view = T(-eye))
    aspect = width / height
    f = float(P[5])
    return {"view": V, "proj": P, "position": np.array([eye_offset_x, 0.0, 0.0], np.float32),
            "focal_x": width * f / (2 * aspect), "focal_y": height * f / 2, "near": 0.1, "far": 10.0}


def orbit_camera(width: int, height: int, angle_deg: float, pivot_z: float = 5.5) -> dict:
    """make_camera's camera moved on a circle about the y axis through (0, 0, pivot_z), still looking
    at that point: angle 0 is make_camera itself.  Used for the moving-camera benchmark (bench.py
    --camera-path orbit), where every frame sees a slightly different view."""
    a = math.radians(angle_deg)
    c, s = np.float32(math.cos(a)), np.float32(math.sin(a))
    R = np.array([[c, 0, s], [0, 1, 0], [-s, 0, c]], np.float32)        # camera-to-world rotation
    pos = np.array([0, 0, pivot_z], np.float32) + R @ np.array([0, 0, -pivot_z], np.float32)
    Rt = R.T
    t = -(Rt @ pos)
    V = np.eye(4, dtype=np.float32)
    V[:3, :3] = Rt
    V[:3, 3] = t
    cam = make_camera(width, height)
    cam["view"] = V.T.reshape(-1).astype(np.float32)  # column-major flat
    cam["position"] = pos.astype(np.float32)
    return cam


def _f16_bits(x: np.ndarray) -> np.ndarray:
    return np.asarray(x, np.float32).astype(np.float16).view(np.uint16)


def gen_scene(count: int, width: int, height: int, sh_components: int, precision: int,
              seed: int = 42, scale_px: float = 1.2, spread: float = 0.6):
    """Returns (world structured array, harmonics array (float32 or fp16 bits), camera dict).

    precision: 0 -> PackedWorldGaussian + f32 SH, 1 -> PackedWorldGaussianHalf + f16 SH."""
    rng = np.random.default_rng(seed)
    z = rng.uniform(1.5, 9.5, count).astype(np.float32)
    x = (rng.uniform(-1.0, 1.0, count) * spread * z).astype(np.float32)
    y = (rng.uniform(-1.0, 1.0, count) * spread * z).astype(np.float32)
    f_px = (height / 2.0) / math.tan(math.radians(30.0))
    s_med = scale_px * 5.5 / f_px
    s = (s_med * np.exp(rng.uniform(-1.0, 1.0, (count, 3)) * 0.6)).astype(np.float32)
    q = rng.normal(size=(count, 4)).astype(np.float32)
    q /= np.linalg.norm(q, axis=1, keepdims=True)
    op = rng.uniform(0.5, 1.0, count).astype(np.float32)
    k = max(int(sh_components), 1)
    harm = np.zeros((count, 3, k), np.float32)
    harm[:, :, 0] = rng.uniform(0.0, 1.0, (count, 3))
    if k > 1:
        harm[:, :, 1:] = np.clip(rng.normal(0.0, 0.1, (count, 3, k - 1)), -0.3, 0.3)
    harm = harm.reshape(-1)  # planar per gaussian: [R0..Rk-1, G0.., B0..]
    if precision == 0:
        w = np.zeros(count, WORLD32)
        w["px"], w["py"], w["pz"] = x, y, z
        w["opacity"] = op
        w["sx"], w["sy"], w["sz"] = s[:, 0], s[:, 1], s[:, 2]
        w["rot"] = q
        h = harm
    else:
        w = np.zeros(count, WORLD16)
        w["px"], w["py"], w["pz"] = x, y, z
        w["opacity"] = _f16_bits(op)
        w["sx"], w["sy"], w["sz"] = _f16_bits(s[:, 0]), _f16_bits(s[:, 1]), _f16_bits(s[:, 2])
        w["rx"], w["ry"], w["rz"], w["rw"] = (_f16_bits(q[:, i]) for i in range(4))
        h = _f16_bits(harm)
    return w, h, make_camera(width, height)


# Benchmark / parity configurations (BASELINE.json "configs")
CONFIGS = {
    "cfg1_50k_sh0_640x360_f32": dict(count=50_000, width=640, height=360, sh=1, precision=0),
    "cfg2_1m_sh3_1080p_f16": dict(count=1_000_000, width=1920, height=1080, sh=16, precision=1),
    "cfg3_5m_sh3_4k_f16": dict(count=5_000_000, width=3840, height=2160, sh=16, precision=1),
    # config 5: two eyes of 1440x1600 side by side (width = per eye), +-32 mm x offsets
    "cfg5_1m_sh2_stereo_2x1440x1600_f16": dict(count=1_000_000, width=1440, height=1600, sh=9, precision=1,
                                               stereo=0.032),
}
