"""ctypes binding for the C oracle (TEST INFRASTRUCTURE ONLY).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import
this module; the product path (gsm-renderer_amd/) never does.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "libgsm_oracle.so")

WORLD32 = np.dtype([("px", "<f4"), ("py", "<f4"), ("pz", "<f4"), ("opacity", "<f4"),
                    ("sx", "<f4"), ("sy", "<f4"), ("sz", "<f4"), ("pad0", "<f4"),
                    ("rot", "<f4", (4,))])
WORLD16 = np.dtype([("px", "<f4"), ("py", "<f4"), ("pz", "<f4"), ("opacity", "<u2"),
                    ("sx", "<u2"), ("sy", "<u2"), ("sz", "<u2"), ("rx", "<u2"), ("ry", "<u2"),
                    ("rz", "<u2"), ("rw", "<u2"), ("pad0", "<u2"), ("pad1", "<u2")])
RENDER_DATA = np.dtype([("meanX", "<u2"), ("meanY", "<u2"), ("theta", "<u2"), ("sigma1", "<u2"),
                        ("sigma2", "<u2"), ("depth", "<u2"), ("colorR", "u1"), ("colorG", "u1"),
                        ("colorB", "u1"), ("opacity", "u1")])
STEREO_RENDER_DATA = np.dtype([(f, "<u2") for f in (
    "leftMeanX", "leftMeanY", "leftCxx", "leftCyy", "leftCxy2", "leftDepth",
    "rightMeanX", "rightMeanY", "rightCxx", "rightCyy", "rightCxy2", "rightDepth")] +
    [("colorR", "u1"), ("colorG", "u1"), ("colorB", "u1"), ("opacity", "u1"),
     ("centerDepth", "<u2"), ("pad0", "<u2")])
assert WORLD32.itemsize == 48 and WORLD16.itemsize == 32 and RENDER_DATA.itemsize == 16
assert STEREO_RENDER_DATA.itemsize == 32


class OgCamera(C.Structure):
    _fields_ = [("view", C.c_float * 16), ("proj", C.c_float * 16), ("position", C.c_float * 3),
                ("focal_x", C.c_float), ("focal_y", C.c_float),
                ("near_plane", C.c_float), ("far_plane", C.c_float)]


class OgConfig(C.Structure):
    _fields_ = [("max_gaussians", C.c_uint32), ("max_width", C.c_uint32),
                ("max_height", C.c_uint32), ("precision", C.c_uint32),
                ("color_space", C.c_uint32)]


class OgFrame(C.Structure):
    _fields_ = [("count", C.c_uint32), ("width", C.c_uint32), ("height", C.c_uint32),
                ("tiles_x", C.c_uint32), ("tiles_y", C.c_uint32), ("tile_count", C.c_uint32),
                ("max_assignments", C.c_uint32), ("total_assignments", C.c_uint32),
                ("overflow", C.c_uint32), ("visible", C.c_uint32), ("active_tiles", C.c_uint32),
                ("render_data", C.c_void_p), ("bounds", C.c_void_p), ("mask", C.c_void_p),
                ("tile_counts", C.c_void_p), ("keys", C.c_void_p), ("values", C.c_void_p),
                ("sorted_keys", C.c_void_p), ("sorted_values", C.c_void_p),
                ("headers", C.c_void_p), ("color", C.c_void_p), ("depth", C.c_void_p),
                ("group_iters", C.c_void_p),
                ("t_project", C.c_double), ("t_assign", C.c_double), ("t_sort", C.c_double),
                ("t_headers", C.c_double), ("t_blend", C.c_double)]


class OgDfFrame(C.Structure):
    _fields_ = [("count", C.c_uint32), ("width", C.c_uint32), ("height", C.c_uint32),
                ("tiles_x", C.c_uint32), ("tiles_y", C.c_uint32), ("tile_count", C.c_uint32),
                ("max_instances", C.c_uint32), ("visible", C.c_uint32),
                ("total_instances", C.c_uint32), ("overflow", C.c_uint32),
                ("active_tiles", C.c_uint32),
                ("render_data", C.c_void_p), ("bounds", C.c_void_p), ("touched", C.c_void_p),
                ("depth_keys", C.c_void_p), ("depth_order", C.c_void_p),
                ("inst_tiles", C.c_void_p), ("inst_gids", C.c_void_p), ("headers", C.c_void_p),
                ("eye_color", C.c_void_p), ("color", C.c_void_p),
                ("t_project", C.c_double), ("t_sort", C.c_double), ("t_blend", C.c_double)]


def build(force: bool = False) -> str:
    """Compile the oracle with gcc (oracle/Makefile)."""
    src = os.path.join(_HERE, "gsm_oracle.c")
    if force or not os.path.exists(_LIB_PATH) or os.path.getmtime(_LIB_PATH) < max(
            os.path.getmtime(os.path.join(_HERE, f)) for f in
            ("gsm_oracle.c", "gsm_oracle.h", "gsm_oracle_math.h")):
        subprocess.run(["make", "-s", "-C", _HERE], check=True)
    assert os.path.exists(src)
    return _LIB_PATH


_lib = None


def lib():
    global _lib
    if _lib is None:
        build()
        L = C.CDLL(_LIB_PATH)
        L.og_render.argtypes = [C.POINTER(OgConfig), C.c_void_p, C.c_void_p, C.c_uint32, C.c_uint32,
                                C.POINTER(OgCamera), C.c_uint32, C.c_uint32, C.c_int,
                                C.POINTER(C.POINTER(OgFrame))]
        L.og_render.restype = C.c_int
        L.og_frame_free.argtypes = [C.POINTER(OgFrame)]
        L.og_sort_key.argtypes = [C.c_uint32, C.c_uint16]
        L.og_sort_key.restype = C.c_uint32
        L.og_radix_sort_pairs.argtypes = [C.c_void_p, C.c_void_p, C.c_uint32]
        L.og_f2h.argtypes = [C.c_float]
        L.og_f2h.restype = C.c_uint16
        L.og_h2f.argtypes = [C.c_uint16]
        L.og_h2f.restype = C.c_float
        L.og_d2h.argtypes = [C.c_double]
        L.og_d2h.restype = C.c_uint16
        L.og_exp_h.argtypes = [C.c_uint16]
        L.og_exp_h.restype = C.c_uint16
        L.og_hfma.argtypes = [C.c_uint16, C.c_uint16, C.c_uint16]
        L.og_hfma.restype = C.c_uint16
        for name in ("og_atan2f",):
            getattr(L, name).argtypes = [C.c_float, C.c_float]
            getattr(L, name).restype = C.c_float
        for name in ("og_log2f", "og_exp2f"):
            getattr(L, name).argtypes = [C.c_float]
            getattr(L, name).restype = C.c_float
        L.og_convert_color.argtypes = [C.c_void_p, C.c_size_t, C.c_int, C.c_void_p]
        L.og_convert_color.restype = C.c_int
        L.og_srand48.argtypes = [C.c_long]
        L.og_drand48.restype = C.c_double
        L.og_gen_visible_gaussians.argtypes = [C.c_uint32, C.c_long, C.c_void_p, C.c_void_p]
        L.og_gen_grid_gaussians.argtypes = [C.c_uint32, C.c_long, C.c_void_p, C.c_void_p]
        L.og_make_camera.argtypes = [C.c_uint32, C.c_uint32, C.POINTER(OgCamera)]
        L.og_df_render_stereo.argtypes = [C.POINTER(OgConfig), C.c_void_p, C.c_void_p, C.c_uint32,
                                          C.c_uint32, C.POINTER(OgCamera), C.POINTER(OgCamera),
                                          C.c_void_p, C.c_uint32, C.c_uint32, C.c_int,
                                          C.POINTER(C.POINTER(OgDfFrame))]
        L.og_df_render_stereo.restype = C.c_int
        L.og_df_frame_free.argtypes = [C.POINTER(OgDfFrame)]
        L.og_sincos_theta.argtypes = [C.c_float, C.POINTER(C.c_float), C.POINTER(C.c_float)]
        L.og_float_to_sortable.argtypes = [C.c_float]
        L.og_float_to_sortable.restype = C.c_uint32
        _lib = L
    return _lib


def drand48_sequence(seed: int, n: int) -> np.ndarray:
    L = lib()
    L.og_srand48(seed)
    return np.array([L.og_drand48() for _ in range(n)], dtype=np.float64)


def make_camera(width: int, height: int) -> dict:
    cam = OgCamera()
    lib().og_make_camera(width, height, C.byref(cam))
    return camera_to_dict(cam)


def camera_to_dict(cam: OgCamera) -> dict:
    return {"view": np.array(cam.view[:], np.float32), "proj": np.array(cam.proj[:], np.float32),
            "position": np.array(cam.position[:], np.float32), "focal_x": cam.focal_x,
            "focal_y": cam.focal_y, "near": cam.near_plane, "far": cam.far_plane}


def dict_to_camera(d: dict) -> OgCamera:
    cam = OgCamera()
    cam.view[:] = [float(v) for v in np.asarray(d["view"], np.float32).reshape(-1)]
    cam.proj[:] = [float(v) for v in np.asarray(d["proj"], np.float32).reshape(-1)]
    cam.position[:] = [float(v) for v in np.asarray(d["position"], np.float32).reshape(-1)]
    cam.focal_x = float(d.get("focal_x", 0.0))
    cam.focal_y = float(d.get("focal_y", 0.0))
    cam.near_plane = float(d.get("near", 0.1))
    cam.far_plane = float(d.get("far", 10.0))
    return cam


def gen_visible_gaussians(count: int, seed: int = 42):
    world = np.zeros(count, WORLD32)
    harm = np.zeros(count * 3, np.float32)
    lib().og_gen_visible_gaussians(count, seed, world.ctypes.data, harm.ctypes.data)
    return world, harm


def gen_grid_gaussians(count: int, seed: int = 42):
    world = np.zeros(count, WORLD32)
    harm = np.zeros(count * 3, np.float32)
    lib().og_gen_grid_gaussians(count, seed, world.ctypes.data, harm.ctypes.data)
    return world, harm


def convert_color(color_u16: np.ndarray, fmt: int) -> np.ndarray:
    """The frame's rgba16f colour (uint16 bits, [..., 4]) in target pixel format `fmt`
    (include/gsm_renderer.h gsm_color_format): uint16 [..., 4], float32 [..., 4] or uint8 [..., 4]."""
    src = np.ascontiguousarray(color_u16, np.uint16)
    n = src.size // 4
    shape = src.shape
    if fmt == 0:
        return src.copy()
    out = np.zeros(shape, np.float32) if fmt == 1 else np.zeros(shape, np.uint8)
    if lib().og_convert_color(src.ctypes.data, n, int(fmt), out.ctypes.data) == 0:
        raise ValueError(f"unknown colour format {fmt}")
    return out


def radix_sort_pairs(keys: np.ndarray, values: np.ndarray):
    k = np.ascontiguousarray(keys, np.uint32).copy()
    v = np.ascontiguousarray(values, np.int32).copy()
    lib().og_radix_sort_pairs(k.ctypes.data, v.ctypes.data, k.size)
    return k, v


def _arr(ptr, dtype, n):
    if n == 0 or not ptr:
        return np.zeros(0, dtype)
    buf = (C.c_char * (n * np.dtype(dtype).itemsize)).from_address(ptr)
    return np.frombuffer(bytes(buf), dtype=dtype, count=n)


def render(world: np.ndarray, harmonics: np.ndarray, sh_components: int, camera: dict,
           width: int, height: int, max_gaussians: int | None = None,
           max_width: int | None = None, max_height: int | None = None,
           precision: int | None = None, color_space: int = 0, nthreads: int = 0,
           count: int | None = None) -> dict:
    """Render one frame with the oracle; returns every intermediate as numpy arrays."""
    L = lib()
    if nthreads <= 0:  # the GPU box exports OMP_NUM_THREADS=16 (its CPU share per GPU)
        nthreads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or min(16, os.cpu_count() or 1)
    if precision is None:
        precision = 1 if world.dtype == WORLD16 else 0
    n = len(world) if count is None else count
    cfg = OgConfig(max_gaussians if max_gaussians is not None else max(n, 1),
                   max_width or width, max_height or height, precision, color_space)
    cam = dict_to_camera(camera)
    world = np.ascontiguousarray(world)
    harmonics = np.ascontiguousarray(harmonics)
    out = C.POINTER(OgFrame)()
    rc = L.og_render(C.byref(cfg), world.ctypes.data if world.size else None,
                     harmonics.ctypes.data if harmonics.size else None, n, sh_components,
                     C.byref(cam), width, height, nthreads, C.byref(out))
    if rc != 0:
        return {"status": rc}
    f = out.contents
    try:
        tot = f.total_assignments
        res = {
            "status": 0, "count": f.count, "tiles_x": f.tiles_x, "tiles_y": f.tiles_y,
            "tile_count": f.tile_count, "max_assignments": f.max_assignments,
            "total_assignments": tot, "overflow": f.overflow, "visible": f.visible,
            "active_tiles": f.active_tiles,
            "render_data": _arr(f.render_data, RENDER_DATA, f.count),
            "bounds": _arr(f.bounds, np.int32, f.count * 4).reshape(-1, 4),
            "mask": _arr(f.mask, np.uint8, f.count),
            "tile_counts": _arr(f.tile_counts, np.uint32, f.count),
            "keys": _arr(f.keys, np.uint32, tot), "values": _arr(f.values, np.int32, tot),
            "sorted_keys": _arr(f.sorted_keys, np.uint32, tot),
            "sorted_values": _arr(f.sorted_values, np.int32, tot),
            "headers": _arr(f.headers, np.uint32, f.tile_count * 2).reshape(-1, 2),
            "color": _arr(f.color, np.uint16, width * height * 4).reshape(height, width, 4),
            "depth": _arr(f.depth, np.uint16, width * height).reshape(height, width),
            "group_iters": _arr(f.group_iters, np.uint32, f.tile_count * 64).reshape(-1, 8, 8),
            "times": {"project": f.t_project, "assign": f.t_assign, "sort": f.t_sort,
                      "headers": f.t_headers, "blend": f.t_blend},
        }
    finally:
        L.og_frame_free(out)
    return res


def _nthreads(nthreads: int) -> int:
    if nthreads > 0:
        return nthreads
    return int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or min(16, os.cpu_count() or 1)


def sincos_theta(theta: float):
    s, c = C.c_float(), C.c_float()
    lib().og_sincos_theta(float(theta), C.byref(s), C.byref(c))
    return s.value, c.value


def df_render_stereo(world: np.ndarray, harmonics: np.ndarray, sh_components: int, left: dict,
                     right: dict, width: int, height: int, scene_transform=None,
                     max_gaussians: int | None = None, max_width: int | None = None,
                     max_height: int | None = None, precision: int | None = None,
                     color_space: int = 0, nthreads: int = 0, count: int | None = None) -> dict:
    """DepthFirst stereo side-by-side frame (og_df_render_stereo); width/height per eye.
    "color" is the [height, 2*width, 4] side-by-side target, "eye_color" the two
    intermediate slices [2, height, width, 4] before the copy's vertical flip."""
    L = lib()
    if precision is None:
        precision = 1 if world.dtype == WORLD16 else 0
    n = len(world) if count is None else count
    cfg = OgConfig(max_gaussians if max_gaussians is not None else max(n, 1),
                   max_width or width, max_height or height, precision, color_space)
    cl, cr = dict_to_camera(left), dict_to_camera(right)
    world = np.ascontiguousarray(world)
    harmonics = np.ascontiguousarray(harmonics)
    st = None
    if scene_transform is not None:
        st = np.ascontiguousarray(np.asarray(scene_transform, np.float32).reshape(16))
    out = C.POINTER(OgDfFrame)()
    rc = L.og_df_render_stereo(C.byref(cfg), world.ctypes.data if world.size else None,
                               harmonics.ctypes.data if harmonics.size else None, n, sh_components,
                               C.byref(cl), C.byref(cr), st.ctypes.data if st is not None else None,
                               width, height, _nthreads(nthreads), C.byref(out))
    if rc != 0:
        return {"status": rc}
    f = out.contents
    try:
        tot, V = f.total_instances, f.visible
        res = {
            "status": 0, "count": f.count, "tiles_x": f.tiles_x, "tiles_y": f.tiles_y,
            "tile_count": f.tile_count, "max_instances": f.max_instances, "visible": V,
            "total_instances": tot, "overflow": f.overflow, "active_tiles": f.active_tiles,
            "render_data": _arr(f.render_data, STEREO_RENDER_DATA, f.count),
            "bounds": _arr(f.bounds, np.int32, f.count * 4).reshape(-1, 4),
            "touched": _arr(f.touched, np.uint32, f.count),
            "depth_keys": _arr(f.depth_keys, np.uint32, f.count),
            "depth_order": _arr(f.depth_order, np.int32, V),
            "inst_tiles": _arr(f.inst_tiles, np.uint32, tot),
            "inst_gids": _arr(f.inst_gids, np.int32, tot),
            "headers": _arr(f.headers, np.uint32, f.tile_count * 2).reshape(-1, 2),
            "eye_color": _arr(f.eye_color, np.uint16, 2 * width * height * 4).reshape(2, height, width, 4),
            "color": _arr(f.color, np.uint16, 2 * width * height * 4).reshape(height, 2 * width, 4),
            "times": {"project": f.t_project, "sort": f.t_sort, "blend": f.t_blend},
        }
    finally:
        L.og_df_frame_free(out)
    return res
