"""PLY ingestion (include/gsm_ply.h): the reference's PLYLoader.load and GaussianSceneBuilder
(Sources/Renderer/Utils/PLYLoader.swift, Scene.swift) over the C ABI of libgsm_amd.so.

    ds = gsm_amd.ply.load("scene.ply")          # GaussianDataset: records + planar harmonics
    world, harm = ds.pack(precision=1)          # GaussianInput buffers (PackedWorldGaussianHalf, fp16 SH)

The loader runs on the host (file parsing and per-vertex conversion); `pack` gives the bytes
the renderer's GaussianInput expects, ready to copy to the device.
"""
from __future__ import annotations

import ctypes as C
import enum
from dataclasses import dataclass

import numpy as np

from .types import WORLD16, WORLD32


class PLYStatus(enum.IntEnum):
    """PLYLoaderError (PLYLoader.swift:220-247) and PLYHeader.DecodeError (:91-113)."""
    OK = 0
    IO = 1
    INVALID_HEADER = 2
    UNSUPPORTED_FORMAT = 3
    MISSING_VERTEX_ELEMENT = 4
    MISSING_REQUIRED_PROPERTIES = 5
    LIST_PROPERTIES_NOT_SUPPORTED = 6
    INSUFFICIENT_DATA = 7
    MISSING_CHUNK_ELEMENT = 8
    HEADER_FORMAT_MISSING = 9
    HEADER_INVALID_CHARACTERS = 10
    HEADER_UNKNOWN_KEYWORD = 11
    HEADER_UNEXPECTED_KEYWORD = 12
    HEADER_INVALID_LINE = 13
    HEADER_INVALID_FORMAT_TYPE = 14
    HEADER_UNKNOWN_PROPERTY_TYPE = 15
    INVALID_ARGUMENT = 16


class PLYLoaderError(RuntimeError):
    def __init__(self, status: int, message: str):
        self.status = PLYStatus(status)
        super().__init__(f"{self.status.name}: {message}")


_SIG = {
    "gsm_ply_load": ([C.c_char_p, C.POINTER(C.c_void_p)], C.c_int),
    "gsm_ply_load_memory": ([C.c_void_p, C.c_size_t, C.POINTER(C.c_void_p)], C.c_int),
    "gsm_ply_last_error": ([], C.c_char_p),
    "gsm_ply_status_string": ([C.c_int], C.c_char_p),
    "gsm_ply_free": ([C.c_void_p], None),
    "gsm_ply_count": ([C.c_void_p], C.c_uint32),
    "gsm_ply_sh_components": ([C.c_void_p], C.c_uint32),
    "gsm_ply_is_compressed": ([C.c_void_p], C.c_int),
    "gsm_ply_records": ([C.c_void_p] + [C.c_void_p] * 5, C.c_int),
    "gsm_ply_bounds": ([C.c_void_p, C.c_void_p, C.POINTER(C.c_float)], C.c_int),
    "gsm_ply_sort_morton": ([C.c_void_p], C.c_int),
    "gsm_ply_packed_sizes": ([C.c_void_p, C.c_int, C.POINTER(C.c_size_t), C.POINTER(C.c_size_t)], C.c_int),
    "gsm_ply_pack": ([C.c_void_p, C.c_int, C.c_void_p, C.c_size_t, C.c_void_p, C.c_size_t], C.c_int),
}
_BOUND = False


def _l():
    global _BOUND
    from . import _lib
    L = _lib()
    if not _BOUND:
        for name, (args, res) in _SIG.items():
            fn = getattr(L, name)
            fn.argtypes = args
            fn.restype = res
        _BOUND = True
    return L


def _check(st: int):
    if st != 0:
        raise PLYLoaderError(st, _l().gsm_ply_last_error().decode())


@dataclass
class GaussianDataset:
    """GaussianDataset (Scene.swift:141-158) as numpy arrays.  rotations are (x, y, z, w)."""
    positions: np.ndarray    # [n, 3] f32 (recentred)
    scales: np.ndarray       # [n, 3] f32 (linear)
    rotations: np.ndarray    # [n, 4] f32, normalised quaternion (x, y, z, w)
    opacities: np.ndarray    # [n] f32 (linear)
    harmonics: np.ndarray    # [n * 3 * sh_components] f32, planar per gaussian
    sh_components: int
    compressed: bool
    _handle: C.c_void_p = None

    @property
    def count(self) -> int:
        return int(self.positions.shape[0])

    def bounds(self):
        """GaussianSceneBuilder.bounds(of:) (Scene.swift:172-196) -> (center[3], radius)."""
        c = np.zeros(3, np.float32)
        r = C.c_float(0.0)
        _check(_l().gsm_ply_bounds(self._handle, c.ctypes.data, C.byref(r)))
        return c, float(r.value)

    def pack(self, precision: int = 1):
        """GaussianInput buffers: (world structured array, harmonics array).  precision 1 ->
        PackedWorldGaussianHalf + fp16 SH bits (uint16), 0 -> PackedWorldGaussian + f32 SH."""
        L = _l()
        gb, hb = C.c_size_t(0), C.c_size_t(0)
        _check(L.gsm_ply_packed_sizes(self._handle, precision, C.byref(gb), C.byref(hb)))
        world = np.zeros(self.count, WORLD16 if precision else WORLD32)
        harm = np.zeros(hb.value // (2 if precision else 4), np.uint16 if precision else np.float32)
        _check(L.gsm_ply_pack(self._handle, precision, world.ctypes.data, world.nbytes,
                              harm.ctypes.data if harm.size else None, harm.nbytes))
        return world, harm

    def sort_morton(self) -> "GaussianDataset":
        """GaussianSceneBuilder.sortByMortonCode (Scene.swift:74-138), in place (stable ties)."""
        _check(_l().gsm_ply_sort_morton(self._handle))
        self._refresh()
        return self

    def _refresh(self):
        L = _l()
        n = int(L.gsm_ply_count(self._handle))
        k = int(L.gsm_ply_sh_components(self._handle))
        hb = C.c_size_t(0)
        gb = C.c_size_t(0)
        _check(L.gsm_ply_packed_sizes(self._handle, 0, C.byref(gb), C.byref(hb)))
        self.positions = np.zeros((n, 3), np.float32)
        self.scales = np.zeros((n, 3), np.float32)
        self.rotations = np.zeros((n, 4), np.float32)
        self.opacities = np.zeros(n, np.float32)
        self.harmonics = np.zeros(hb.value // 4, np.float32)
        _check(L.gsm_ply_records(self._handle, self.positions.ctypes.data, self.scales.ctypes.data,
                                 self.rotations.ctypes.data, self.opacities.ctypes.data,
                                 self.harmonics.ctypes.data if self.harmonics.size else None))
        self.sh_components = k
        self.compressed = bool(L.gsm_ply_is_compressed(self._handle))

    def __del__(self):
        if self._handle:
            try:
                _l().gsm_ply_free(self._handle)
            except Exception:
                pass
            self._handle = None


def _wrap(h: C.c_void_p) -> GaussianDataset:
    e = np.zeros(0, np.float32)
    ds = GaussianDataset(e, e, e, e, e, 0, False, h)
    ds._refresh()
    return ds


def load(path: str) -> GaussianDataset:
    """PLYLoader.load(url:) (PLYLoader.swift:254-287)."""
    h = C.c_void_p()
    _check(_l().gsm_ply_load(str(path).encode(), C.byref(h)))
    return _wrap(h)


def load_bytes(data: bytes) -> GaussianDataset:
    h = C.c_void_p()
    buf = C.create_string_buffer(bytes(data), len(data))
    _check(_l().gsm_ply_load_memory(buf, len(data), C.byref(h)))
    return _wrap(h)
