"""gsm_amd -- Python mirror of the reference's GlobalRenderer operator surface over the
MI355X C ABI (include/gsm_renderer.h, include/gsm_debug.h).

Mirrors Sources/Renderer/Shared/GaussianRendererProtocol.swift (RendererConfig,
GaussianInput, CameraParams, RendererError) and GlobalRenderer.swift (init, render,
renderStereo, debugReadTotalAssignments, lastGPUTime).  Device buffers are torch
tensors on a ROCm device (PyTorch is plumbing: memory, streams, torch.distributed);
every frame runs in the hand-written gfx950 kernels of libgsm_amd.so.  There is no
CPU fallback: if the library is missing, importing a renderer raises.
"""
from __future__ import annotations

import ctypes as C
import enum
import os
from dataclasses import dataclass, field
from typing import Optional

import numpy as np

try:  # load torch's HIP runtime first so libgsm_amd.so binds to the same one
    import torch  # noqa: F401
except Exception:  # pragma: no cover - torch is always present in this image
    torch = None

from .types import RENDER_DATA, WORLD16, WORLD32  # noqa: F401

_PKG_DIR = os.path.dirname(os.path.abspath(__file__))
# GSM_AMD_LIB: another in-tree build of the same library (A/B experiments, tools/); default lib/
LIB_PATH = os.environ.get("GSM_AMD_LIB") or os.path.join(os.path.dirname(_PKG_DIR), "lib", "libgsm_amd.so")
INCLUDE_DIR = os.path.join(os.path.dirname(os.path.dirname(_PKG_DIR)), "include")


class Status(enum.IntEnum):
    """RendererError cases (GaussianRendererProtocol.swift:274-292) as C status codes."""
    OK = 0
    DEVICE_NOT_AVAILABLE = 1
    FAILED_TO_CREATE_LIBRARY = 2
    FAILED_TO_CREATE_PIPELINE = 3
    FAILED_TO_ALLOCATE_BUFFER = 4
    FAILED_TO_ALLOCATE_TEXTURE = 5
    INVALID_GAUSSIAN_COUNT = 6
    INVALID_DIMENSIONS = 7
    INVALID_BUFFER_SIZE = 8
    INVALID_TILE_COUNT = 9
    INVALID_ASSIGNMENT_CAPACITY = 10
    RENDER_FAILED = 11
    ENCODER_CREATION_FAILED = 12
    MISSING_REQUIRED_BUFFER = 13
    INVALID_ARGUMENT = 14
    UNSUPPORTED = 15
    PHASE_ORDER = 16


class RendererError(RuntimeError):
    def __init__(self, status: int, what: str = ""):
        self.status = Status(status)
        msg = _lib().gsm_status_string(int(status)).decode() if _LIB is not None else self.status.name
        super().__init__(f"{self.status.name}: {msg}{(' (' + what + ')') if what else ''}")


class RenderPrecision(enum.IntEnum):  # GaussianRendererProtocol.swift:4-7
    FLOAT32 = 0
    FLOAT16 = 1


class GaussianColorSpace(enum.IntEnum):  # GaussianRendererProtocol.swift:196-201
    LINEAR = 0
    SRGB = 1


class ColorFormat(enum.IntEnum):
    """Colour target pixel format (RendererConfig.colorFormat, GaussianRendererProtocol.swift:207;
    include/gsm_renderer.h gsm_color_format has the conversion rules)."""
    RGBA16F = 0
    RGBA32F = 1
    RGBA8_UNORM = 2
    RGBA8_UNORM_SRGB = 3
    BGRA8_UNORM = 4
    BGRA8_UNORM_SRGB = 5

    @property
    def bytes_per_pixel(self) -> int:
        return 8 if self == ColorFormat.RGBA16F else (16 if self == ColorFormat.RGBA32F else 4)


class BufferId(enum.IntEnum):  # include/gsm_debug.h gsm_buffer_id
    RENDER_DATA = 0
    BOUNDS = 1
    TILE_COUNTS = 2
    KEYS = 3
    VALUES = 4
    SORTED_KEYS = 5
    SORTED_VALUES = 6
    HEADERS = 7
    EXP_TABLE = 8
    BLEND_TRACE = 9


STAGES = ("project", "scan", "scatter", "sort", "headers", "blend")
# gsm_blend_kernel (include/gsm_debug.h) -> the kernel's name in rocprofv3 traces
BLEND_KERNELS = {0: None, 1: "k_blend_px", 2: "k_blend_px", 3: "k_blend_pw"}


@dataclass
class RendererConfig:
    """RendererConfig (GaussianRendererProtocol.swift:195-228) with the same defaults."""
    max_gaussians: int = 6_000_000
    max_width: int = 1920
    max_height: int = 1080
    precision: RenderPrecision = RenderPrecision.FLOAT16
    color_format: int = 0
    gaussian_color_space: GaussianColorSpace = GaussianColorSpace.SRGB
    back_to_front: bool = False


@dataclass
class GaussianInput:
    """GaussianInput (GaussianRendererProtocol.swift:9-26): device buffers + counts."""
    gaussians: "torch.Tensor"
    harmonics: "torch.Tensor"
    gaussian_count: int
    shComponents: int = 0

    @property
    def sh_components(self) -> int:
        return self.shComponents


@dataclass
class CameraParams:
    """CameraParams (GaussianRendererProtocol.swift:28-54).  view/proj are 16 floats in
    simd_float4x4 (column-major) memory order."""
    view: np.ndarray
    proj: np.ndarray
    position: np.ndarray = field(default_factory=lambda: np.zeros(3, np.float32))
    focal_x: float = 0.0
    focal_y: float = 0.0
    near: float = 0.1
    far: float = 10.0

    @staticmethod
    def from_dict(d: dict) -> "CameraParams":
        return CameraParams(np.asarray(d["view"], np.float32).reshape(16),
                            np.asarray(d["proj"], np.float32).reshape(16),
                            np.asarray(d.get("position", np.zeros(3)), np.float32).reshape(3),
                            float(d.get("focal_x", 0.0)), float(d.get("focal_y", 0.0)),
                            float(d.get("near", 0.1)), float(d.get("far", 10.0)))

    def to_dict(self) -> dict:
        return {"view": np.asarray(self.view, np.float32), "proj": np.asarray(self.proj, np.float32),
                "position": np.asarray(self.position, np.float32), "focal_x": self.focal_x,
                "focal_y": self.focal_y, "near": self.near, "far": self.far}


# ---------------------------------------------------------------------------
# ctypes layer
# ---------------------------------------------------------------------------
class _Config(C.Structure):
    _fields_ = [("max_gaussians", C.c_uint32), ("max_width", C.c_uint32), ("max_height", C.c_uint32),
                ("precision", C.c_uint32), ("color_format", C.c_uint32),
                ("gaussian_color_space", C.c_uint32), ("back_to_front", C.c_uint32)]


class _Input(C.Structure):
    _fields_ = [("gaussians", C.c_void_p), ("harmonics", C.c_void_p),
                ("gaussian_count", C.c_uint32), ("sh_components", C.c_uint32)]


class _Camera(C.Structure):
    _fields_ = [("view", C.c_float * 16), ("proj", C.c_float * 16), ("position", C.c_float * 3),
                ("focal_x", C.c_float), ("focal_y", C.c_float),
                ("near_plane", C.c_float), ("far_plane", C.c_float)]


class _Counters(C.Structure):
    _fields_ = [("total_assignments", C.c_uint32), ("max_capacity", C.c_uint32),
                ("padded_count", C.c_uint32), ("overflow", C.c_uint32), ("tiles_x", C.c_uint32),
                ("tiles_y", C.c_uint32), ("tile_count", C.c_uint32), ("gaussian_count", C.c_uint32)]


class _DfCounters(C.Structure):
    _fields_ = [("gaussian_count", C.c_uint32), ("visible", C.c_uint32), ("total_instances", C.c_uint32),
                ("max_instances", C.c_uint32), ("overflow", C.c_uint32), ("tiles_x", C.c_uint32),
                ("tiles_y", C.c_uint32), ("tile_count", C.c_uint32)]


_LIB = None

# every function include/gsm_renderer.h and include/gsm_debug.h declare, with ctypes signature
_SIGNATURES = {
    "gsm_abi_version": ([], C.c_int),
    "gsm_status_string": ([C.c_int], C.c_char_p),
    "gsm_renderer_config_default": ([C.POINTER(_Config)], None),
    "gsm_camera_params_init": ([C.POINTER(_Camera), C.c_void_p, C.c_void_p, C.c_void_p, C.c_float,
                                C.c_float], None),
    "gsm_global_create": ([C.POINTER(_Config), C.c_int, C.POINTER(C.c_void_p)], C.c_int),
    "gsm_global_destroy": ([C.c_void_p], None),
    "gsm_global_render": ([C.c_void_p, C.c_void_p, C.POINTER(_Input), C.POINTER(_Camera), C.c_uint32,
                           C.c_uint32, C.c_void_p, C.c_size_t, C.c_void_p, C.c_size_t], C.c_int),
    "gsm_global_render_stereo": ([C.c_void_p, C.c_void_p, C.POINTER(_Input), C.POINTER(_Camera),
                                  C.POINTER(_Camera), C.c_uint32, C.c_uint32, C.c_void_p, C.c_size_t,
                                  C.c_void_p, C.c_size_t], C.c_int),
    "gsm_global_render_stereo_sbs": ([C.c_void_p, C.c_void_p, C.POINTER(_Input), C.POINTER(_Camera),
                                      C.POINTER(_Camera), C.c_uint32, C.c_uint32, C.c_void_p, C.c_size_t,
                                      C.c_void_p, C.c_size_t], C.c_int),
    "gsm_global_debug_read_total_assignments": ([C.c_void_p], C.c_uint32),
    "gsm_global_last_gpu_time": ([C.c_void_p, C.POINTER(C.c_double)], C.c_int),
    "gsm_global_debug_counters": ([C.c_void_p, C.POINTER(_Counters)], C.c_int),
    "gsm_global_debug_blend_kernel": ([C.c_void_p, C.POINTER(C.c_int)], C.c_int),
    "gsm_debug_sort_workspace_bytes": ([C.c_uint32], C.c_size_t),
    "gsm_debug_sort_plan_fits": ([C.c_uint32, C.c_uint32, C.c_int, C.c_size_t], C.c_int),
    "gsm_global_debug_copy": ([C.c_void_p, C.c_int, C.c_void_p, C.c_size_t, C.POINTER(C.c_size_t)],
                              C.c_int),
    "gsm_global_set_profiling": ([C.c_void_p, C.c_int], C.c_int),
    "gsm_global_stage_times": ([C.c_void_p, C.POINTER(C.c_float), C.c_int], C.c_int),
    "gsm_global_set_tile_rows": ([C.c_void_p, C.c_uint32, C.c_uint32], C.c_int),
    "gsm_sort_pairs_u32": ([C.c_void_p, C.c_void_p, C.c_uint32, C.c_uint32, C.c_void_p], C.c_int),
    # include/gsm_multigpu.h
    "gsm_global_project_partition": ([C.c_void_p, C.c_void_p, C.POINTER(_Input), C.POINTER(_Camera),
                                      C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32,
                                      C.POINTER(C.c_uint32), C.c_uint32, C.c_void_p, C.c_uint64,
                                      C.c_void_p], C.c_int),
    "gsm_global_render_records": ([C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint32, C.c_uint32, C.c_uint32,
                                   C.c_void_p, C.c_size_t, C.c_void_p, C.c_size_t], C.c_int),
    # include/gsm_depthfirst.h
    "gsm_depthfirst_create": ([C.POINTER(_Config), C.c_int, C.POINTER(C.c_void_p)], C.c_int),
    "gsm_depthfirst_destroy": ([C.c_void_p], None),
    "gsm_depthfirst_render_stereo_sbs": ([C.c_void_p, C.c_void_p, C.POINTER(_Input), C.POINTER(_Camera),
                                          C.POINTER(_Camera), C.c_void_p, C.c_uint32, C.c_uint32, C.c_void_p,
                                          C.c_size_t], C.c_int),
    "gsm_depthfirst_debug_counters": ([C.c_void_p, C.POINTER(_DfCounters)], C.c_int),
    "gsm_depthfirst_debug_copy": ([C.c_void_p, C.c_int, C.c_void_p, C.c_size_t, C.POINTER(C.c_size_t)],
                                  C.c_int),
    "gsm_depthfirst_set_profiling": ([C.c_void_p, C.c_int], C.c_int),
    "gsm_depthfirst_stage_times": ([C.c_void_p, C.POINTER(C.c_float), C.c_int], C.c_int),
    "gsm_depthfirst_last_gpu_time": ([C.c_void_p, C.POINTER(C.c_double)], C.c_int),
    "gsm_debug_sort_rank_probe": ([C.c_int, C.POINTER(C.c_int)], C.c_int),
    "gsm_debug_partition_counts": ([C.c_void_p, C.c_void_p, C.POINTER(_Input), C.POINTER(_Camera), C.c_uint32,
                                    C.c_uint32, C.c_uint32, C.c_uint32, C.POINTER(C.c_uint32), C.c_uint32,
                                    C.c_void_p], C.c_int),
    "gsm_debug_partition_push": ([C.c_void_p, C.c_void_p, C.c_uint32, C.c_uint32, C.c_void_p,
                                  C.POINTER(C.c_void_p), C.c_void_p], C.c_int),
    "gsm_debug_render_records_device_count": ([C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint32, C.c_void_p,
                                               C.c_uint32, C.c_uint32, C.c_void_p, C.c_size_t, C.c_void_p,
                                               C.c_size_t], C.c_int),
    "gsm_multigpu_create": ([C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.POINTER(C.c_void_p)], C.c_int),
    # (options structs passed as pointers: _MgOptions, gsm_multigpu_options)
    "gsm_multigpu_default_options": ([C.c_void_p], None),
    "gsm_multigpu_prepare_with_options": ([C.c_void_p, C.c_int, C.c_int, C.c_void_p, C.POINTER(C.c_void_p),
                                           C.c_void_p], C.c_int),
    "gsm_multigpu_create_with_options": ([C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_void_p,
                                          C.POINTER(C.c_void_p)], C.c_int),
    "gsm_multigpu_destroy": ([C.c_void_p], None),
    "gsm_multigpu_render": ([C.c_void_p, C.c_void_p, C.POINTER(_Input), C.POINTER(_Camera), C.c_uint32,
                             C.c_uint32, C.c_void_p, C.c_size_t, C.c_void_p, C.c_size_t, C.c_void_p], C.c_int),
    "gsm_multigpu_debug_counts": ([C.c_void_p, C.POINTER(C.c_uint32)], C.c_int),
    "gsm_multigpu_prepare": ([C.c_void_p, C.c_int, C.c_int, C.POINTER(C.c_void_p), C.c_void_p], C.c_int),
    "gsm_multigpu_connect": ([C.c_void_p, C.c_void_p], C.c_int),
    "gsm_multigpu_render_phase": ([C.c_void_p, C.c_int, C.c_void_p, C.POINTER(_Input), C.POINTER(_Camera),
                                   C.c_uint32, C.c_uint32, C.c_void_p, C.c_size_t, C.c_void_p, C.c_size_t,
                                   C.c_void_p], C.c_int),
    "gsm_multigpu_frame": ([C.c_void_p, C.POINTER(C.c_void_p), C.POINTER(C.c_size_t)], C.c_int),
    "gsm_multigpu_status": ([C.c_void_p, C.POINTER(C.c_uint32), C.c_int], C.c_int),
    "gsm_multigpu_set_timeout_ms": ([C.c_void_p, C.c_uint32], C.c_int),
    "gsm_multigpu_debug_copy_exchange": ([C.c_void_p, C.c_void_p, C.c_size_t], C.c_int),
    "gsm_multigpu_debug_copy_frame": ([C.c_void_p, C.c_void_p, C.c_size_t, C.c_uint32, C.c_uint32], C.c_int),
    "gsm_multigpu_debug_copy_depth": ([C.c_void_p, C.c_void_p, C.c_size_t, C.c_uint32, C.c_uint32], C.c_int),
    "gsm_multigpu_frame_depth": ([C.c_void_p, C.POINTER(C.c_void_p), C.POINTER(C.c_size_t)], C.c_int),
    "gsm_multigpu_errors": ([C.c_void_p, C.POINTER(C.c_uint32), C.POINTER(C.c_uint32), C.c_int], C.c_int),
    "gsm_multigpu_finish_frame": ([C.c_void_p, C.c_void_p], C.c_int),
    "gsm_multigpu_wait_event": ([C.c_void_p, C.c_void_p], C.c_int),
    "gsm_multigpu_debug_set_epoch": ([C.c_void_p, C.c_uint32], C.c_int),
}

SPLAT_RECORD_BYTES = 48  # include/gsm_multigpu.h GSM_SPLAT_RECORD_BYTES
MAX_SLABS = 16
MULTIGPU_HANDLE_BYTES = 256  # GSM_MULTIGPU_HANDLE_BYTES


def _lib():
    """Load libgsm_amd.so (built in-tree by __graft_entry__.build / make).  Raises if absent:
    there is deliberately no fallback path."""
    global _LIB
    if _LIB is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"libgsm_amd.so not built: {LIB_PATH} (run `make -C gsm-renderer_amd`)")
        L = C.CDLL(LIB_PATH)
        for name, (args, res) in _SIGNATURES.items():
            fn = getattr(L, name)
            fn.argtypes = args
            fn.restype = res
        _LIB = L
    return _LIB


def library_path() -> str:
    return LIB_PATH


def _check(st: int, what: str = ""):
    if st != 0:
        raise RendererError(st, what)


def _ptr(t) -> Optional[int]:
    if t is None:
        return None
    if isinstance(t, int):
        return t
    return int(t.data_ptr())


def _camera_struct(cam: CameraParams) -> _Camera:
    c = _Camera()
    c.view[:] = [float(v) for v in np.asarray(cam.view, np.float32).reshape(16)]
    c.proj[:] = [float(v) for v in np.asarray(cam.proj, np.float32).reshape(16)]
    c.position[:] = [float(v) for v in np.asarray(cam.position, np.float32).reshape(3)]
    c.focal_x, c.focal_y = float(cam.focal_x), float(cam.focal_y)
    c.near_plane, c.far_plane = float(cam.near), float(cam.far)
    return c


def _stream_handle(stream) -> Optional[int]:
    if stream is None:
        if torch is not None and torch.cuda.is_available():
            return int(torch.cuda.current_stream().cuda_stream)
        return None
    if isinstance(stream, int):
        return stream
    return int(stream.cuda_stream)


class GlobalRenderer:
    """GlobalRenderer (GlobalRenderer.swift:72-572) on one HIP device."""

    def __init__(self, device: Optional[int] = None, config: RendererConfig = RendererConfig()):
        L = _lib()
        self.config = config
        cfg = _Config(int(config.max_gaussians), int(config.max_width), int(config.max_height),
                      int(config.precision), int(config.color_format),
                      int(config.gaussian_color_space), int(bool(config.back_to_front)))
        h = C.c_void_p()
        dev = -1 if device is None else int(device)
        _check(L.gsm_global_create(C.byref(cfg), dev, C.byref(h)), "gsm_global_create")
        self._h = h
        self.device = dev
        self._bpp = ColorFormat(int(config.color_format)).bytes_per_pixel

    def close(self):
        if getattr(self, "_h", None) and self._h.value:
            _lib().gsm_global_destroy(self._h)
            self._h = C.c_void_p()

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass

    # -- GlobalRenderer.render (GlobalRenderer.swift:201-238) --
    def render(self, color_texture, depth_texture, input: GaussianInput, camera: CameraParams,
               width: int, height: int, stream=None, color_pitch: Optional[int] = None,
               depth_pitch: Optional[int] = None):
        inp = _Input(_ptr(input.gaussians), _ptr(input.harmonics), int(input.gaussian_count),
                     int(input.sh_components))
        cam = _camera_struct(camera)
        cp = color_pitch if color_pitch is not None else int(width) * self._bpp
        dp = depth_pitch if depth_pitch is not None else int(width) * 2
        st = _lib().gsm_global_render(self._h, _stream_handle(stream), C.byref(inp), C.byref(cam),
                                      int(width), int(height), _ptr(color_texture), cp,
                                      _ptr(depth_texture), dp)
        _check(st, "gsm_global_render")

    def project_partition(self, input: GaussianInput, camera: CameraParams, width: int, height: int,
                          first: int, count: int, slab_rows, send, send_capacity: int, send_counts,
                          stream=None):
        """gsm_global_project_partition: records of ids [first, first+count) per tile-row slab
        (slab_rows: num_slabs + 1 boundaries) into `send` (device, send_capacity records);
        `send_counts` (device, uint32 per slab) receives the record count of every slab."""
        inp = _Input(_ptr(input.gaussians), _ptr(input.harmonics), int(input.gaussian_count),
                     int(input.sh_components))
        cam = _camera_struct(camera)
        rows = (C.c_uint32 * len(slab_rows))(*[int(x) for x in slab_rows])
        st = _lib().gsm_global_project_partition(self._h, _stream_handle(stream), C.byref(inp), C.byref(cam),
                                                 int(width), int(height), int(first), int(count), rows,
                                                 len(slab_rows) - 1, _ptr(send), int(send_capacity),
                                                 _ptr(send_counts))
        _check(st, "gsm_global_project_partition")

    def render_records(self, color_texture, depth_texture, records, count: int, width: int, height: int,
                       stream=None, color_pitch: Optional[int] = None, depth_pitch: Optional[int] = None):
        """gsm_global_render_records: this renderer's tile rows from `count` received records."""
        cp = color_pitch if color_pitch is not None else int(width) * self._bpp
        dp = depth_pitch if depth_pitch is not None else int(width) * 2
        st = _lib().gsm_global_render_records(self._h, _stream_handle(stream), _ptr(records), int(count),
                                              int(width), int(height), _ptr(color_texture), cp,
                                              _ptr(depth_texture), dp)
        _check(st, "gsm_global_render_records")

    def debug_partition_counts(self, input: GaussianInput, camera: CameraParams, width: int, height: int,
                               first: int, count: int, slab_rows, send_counts, stream=None):
        """gsm_debug_partition_counts: the native multi-GPU frame's projection of ids
        [first, first+count) with per-slab record counts into `send_counts` (device uint32)."""
        inp = _Input(_ptr(input.gaussians), _ptr(input.harmonics), int(input.gaussian_count),
                     int(input.sh_components))
        cam = _camera_struct(camera)
        rows = (C.c_uint32 * len(slab_rows))(*[int(x) for x in slab_rows])
        _check(_lib().gsm_debug_partition_counts(self._h, _stream_handle(stream), C.byref(inp), C.byref(cam),
                                                 int(width), int(height), int(first), int(count), rows,
                                                 len(slab_rows) - 1, _ptr(send_counts)),
               "gsm_debug_partition_counts")

    def debug_partition_push(self, world: int, rank: int, counts, recv_buffers, recv_count, stream=None):
        """gsm_debug_partition_push: the last partition's records written into their slab owners'
        receive buffers (device tensors, one per rank) at the offsets of the device count matrix."""
        bufs = (C.c_void_p * len(recv_buffers))(*[_ptr(b) for b in recv_buffers])
        _check(_lib().gsm_debug_partition_push(self._h, _stream_handle(stream), int(world), int(rank),
                                               _ptr(counts), bufs, _ptr(recv_count)),
               "gsm_debug_partition_push")

    def debug_render_records_device_count(self, color_texture, depth_texture, records, capacity: int, count,
                                          width: int, height: int, stream=None):
        """gsm_debug_render_records_device_count: render_records with the count read on the device."""
        _check(_lib().gsm_debug_render_records_device_count(self._h, _stream_handle(stream), _ptr(records),
                                                            int(capacity), _ptr(count), int(width), int(height),
                                                            _ptr(color_texture), int(width) * self._bpp,
                                                            _ptr(depth_texture), int(width) * 2),
               "gsm_debug_render_records_device_count")

    def render_stereo(self, color_texture, depth_texture, input: GaussianInput, left: CameraParams,
                      right: CameraParams, width: int, height: int, stream=None):
        inp = _Input(_ptr(input.gaussians), _ptr(input.harmonics), int(input.gaussian_count),
                     int(input.sh_components))
        cl, cr = _camera_struct(left), _camera_struct(right)
        st = _lib().gsm_global_render_stereo(self._h, _stream_handle(stream), C.byref(inp), C.byref(cl),
                                             C.byref(cr), int(width), int(height), _ptr(color_texture),
                                             int(width) * 16, _ptr(depth_texture), int(width) * 4)
        _check(st, "gsm_global_render_stereo")

    def render_stereo_sbs(self, color_texture, depth_texture, input: GaussianInput, left: CameraParams,
                          right: CameraParams, width_per_eye: int, height: int, stream=None,
                          color_pitch: Optional[int] = None, depth_pitch: Optional[int] = None):
        """gsm_global_render_stereo_sbs: both eyes into one side-by-side target (config 5)."""
        inp = _Input(_ptr(input.gaussians), _ptr(input.harmonics), int(input.gaussian_count),
                     int(input.sh_components))
        cl, cr = _camera_struct(left), _camera_struct(right)
        cp = color_pitch if color_pitch is not None else 2 * int(width_per_eye) * self._bpp
        dp = depth_pitch if depth_pitch is not None else 2 * int(width_per_eye) * 2
        st = _lib().gsm_global_render_stereo_sbs(self._h, _stream_handle(stream), C.byref(inp), C.byref(cl),
                                                 C.byref(cr), int(width_per_eye), int(height),
                                                 _ptr(color_texture), cp, _ptr(depth_texture), dp)
        _check(st, "gsm_global_render_stereo_sbs")

    def debug_read_total_assignments(self) -> int:
        return int(_lib().gsm_global_debug_read_total_assignments(self._h))

    @property
    def last_gpu_time(self) -> Optional[float]:
        s = C.c_double()
        st = _lib().gsm_global_last_gpu_time(self._h, C.byref(s))
        return float(s.value) if st == 0 else None

    # -- introspection (include/gsm_debug.h) --
    def set_profiling(self, stage_events: bool = True, keep_unsorted: bool = False,
                      blend_trace: bool = False, blend_events: bool = False, blend_event_period: int = 1,
                      capture: bool = False):
        """blend_event_period > 1: with blend_events, bracket the blend on every period-th frame only.
        capture (implied by keep_unsorted): keep the render data and the sorted keys / values for
        copy_buffer (include/gsm_debug.h); the product path writes neither."""
        flags = (1 if stage_events else 0) | (2 if keep_unsorted else 0) | (4 if blend_trace else 0) | \
            (8 if blend_events else 0) | (16 if capture else 0) | \
            ((max(1, min(255, int(blend_event_period))) & 0xFF) << 8)
        _check(_lib().gsm_global_set_profiling(self._h, flags), "gsm_global_set_profiling")

    def stage_times_ms(self) -> dict:
        arr = (C.c_float * len(STAGES))()
        _check(_lib().gsm_global_stage_times(self._h, arr, len(STAGES)), "gsm_global_stage_times")
        return {k: float(v) for k, v in zip(STAGES, arr)}

    def set_tile_rows(self, begin: int, end: int):
        _check(_lib().gsm_global_set_tile_rows(self._h, int(begin), int(end)), "gsm_global_set_tile_rows")

    def blend_kernel(self) -> str:
        """The blend kernel the last enqueued frame launched (gsm_global_debug_blend_kernel)."""
        k = C.c_int(0)
        _check(_lib().gsm_global_debug_blend_kernel(self._h, C.byref(k)), "gsm_global_debug_blend_kernel")
        return BLEND_KERNELS[k.value]

    def counters(self) -> dict:
        c = _Counters()
        _check(_lib().gsm_global_debug_counters(self._h, C.byref(c)), "gsm_global_debug_counters")
        return {name: int(getattr(c, name)) for name, _ in _Counters._fields_}

    def copy_buffer(self, which: BufferId) -> np.ndarray:
        L = _lib()
        need = C.c_size_t()
        _check(L.gsm_global_debug_copy(self._h, int(which), None, 0, C.byref(need)), "debug_copy")
        n = int(need.value)
        raw = np.zeros(max(n, 1), np.uint8)
        if n:
            _check(L.gsm_global_debug_copy(self._h, int(which), raw.ctypes.data, n, None), "debug_copy")
        raw = raw[:n]
        if which == BufferId.RENDER_DATA:
            return raw.view(RENDER_DATA)
        if which == BufferId.BOUNDS:
            return raw.view(np.int32).reshape(-1, 4)
        if which in (BufferId.TILE_COUNTS, BufferId.KEYS, BufferId.SORTED_KEYS):
            return raw.view(np.uint32)
        if which in (BufferId.VALUES, BufferId.SORTED_VALUES):
            return raw.view(np.int32)
        if which == BufferId.HEADERS:
            return raw.view(np.uint32).reshape(-1, 2)
        if which == BufferId.BLEND_TRACE:
            return raw.view(np.uint64).reshape(-1, 4)
        if which == BufferId.EXP_TABLE:
            return raw.view(np.uint16)
        return raw


class DepthFirstBuffer(enum.IntEnum):  # include/gsm_depthfirst.h gsm_depthfirst_buffer
    RENDER_DATA = 0
    BOUNDS = 1
    TOUCHED = 2
    DEPTH_KEYS = 3
    DEPTH_ORDER = 4
    INSTANCE_TILES = 5
    INSTANCE_GAUSSIANS = 6
    HEADERS = 7
    BLEND_STATS = 8


DF_STAGES = ("project", "depth_sort", "instances", "tile_sort", "blend")  # gsm_depthfirst_stage

# StereoTiledRenderData (BridgingTypes.h:250-276), 32 B
STEREO_RENDER_DATA = np.dtype([(f, "<u2") for f in (
    "leftMeanX", "leftMeanY", "leftCxx", "leftCyy", "leftCxy2", "leftDepth",
    "rightMeanX", "rightMeanY", "rightCxx", "rightCyy", "rightCxy2", "rightDepth")] +
    [("colorR", "u1"), ("colorG", "u1"), ("colorB", "u1"), ("opacity", "u1"),
     ("centerDepth", "<u2"), ("pad0", "<u2")])


class DepthFirstRenderer:
    """DepthFirstRenderer (DepthFirstRenderer.swift:11-831) on one HIP device: the stereo
    side-by-side path (renderStereo(target: .sideBySide), :205-223, 469-512).  The mono
    render/renderStereo(.foveated) entry points of the reference are out of scope."""

    def __init__(self, device: Optional[int] = None, config: RendererConfig = RendererConfig()):
        L = _lib()
        self.config = config
        cfg = _Config(int(config.max_gaussians), int(config.max_width), int(config.max_height),
                      int(config.precision), int(config.color_format),
                      int(config.gaussian_color_space), int(bool(config.back_to_front)))
        h = C.c_void_p()
        dev = -1 if device is None else int(device)
        _check(L.gsm_depthfirst_create(C.byref(cfg), dev, C.byref(h)), "gsm_depthfirst_create")
        self._h = h
        self.device = dev
        self._bpp = ColorFormat(int(config.color_format)).bytes_per_pixel

    def close(self):
        if getattr(self, "_h", None) and self._h.value:
            _lib().gsm_depthfirst_destroy(self._h)
            self._h = C.c_void_p()

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass

    def render_stereo_sbs(self, color_texture, input: GaussianInput, left: CameraParams, right: CameraParams,
                          width_per_eye: int, height: int, scene_transform=None, stream=None,
                          color_pitch: Optional[int] = None):
        """Both eyes side by side into color_texture ([height, 2 * width_per_eye] of the
        config's colour format), as the reference's copy pass leaves them (rows flipped)."""
        inp = _Input(_ptr(input.gaussians), _ptr(input.harmonics), int(input.gaussian_count),
                     int(input.sh_components))
        cl, cr = _camera_struct(left), _camera_struct(right)
        st_arr = None
        if scene_transform is not None:
            st_arr = (C.c_float * 16)(*[float(v) for v in np.asarray(scene_transform, np.float32).reshape(16)])
        cp = color_pitch if color_pitch is not None else 2 * int(width_per_eye) * self._bpp
        st = _lib().gsm_depthfirst_render_stereo_sbs(self._h, _stream_handle(stream), C.byref(inp), C.byref(cl),
                                                     C.byref(cr), st_arr, int(width_per_eye), int(height),
                                                     _ptr(color_texture), cp)
        _check(st, "gsm_depthfirst_render_stereo_sbs")

    @property
    def last_gpu_time(self) -> Optional[float]:
        s = C.c_double()
        st = _lib().gsm_depthfirst_last_gpu_time(self._h, C.byref(s))
        return float(s.value) if st == 0 else None

    def set_profiling(self, stage_events: bool = True, blend_events: bool = False, blend_stats: bool = False,
                      blend_event_period: int = 1):
        flags = (1 if stage_events else 0) | (2 if blend_stats else 0) | (8 if blend_events else 0) | \
            ((max(1, min(255, int(blend_event_period))) & 0xFF) << 8)
        _check(_lib().gsm_depthfirst_set_profiling(self._h, flags), "set_profiling")

    def stage_times_ms(self) -> dict:
        arr = (C.c_float * len(DF_STAGES))()
        _check(_lib().gsm_depthfirst_stage_times(self._h, arr, len(DF_STAGES)), "gsm_depthfirst_stage_times")
        return {k: float(v) for k, v in zip(DF_STAGES, arr)}

    def counters(self) -> dict:
        c = _DfCounters()
        _check(_lib().gsm_depthfirst_debug_counters(self._h, C.byref(c)), "gsm_depthfirst_debug_counters")
        return {name: int(getattr(c, name)) for name, _ in _DfCounters._fields_}

    def copy_buffer(self, which: DepthFirstBuffer) -> np.ndarray:
        L = _lib()
        need = C.c_size_t()
        _check(L.gsm_depthfirst_debug_copy(self._h, int(which), None, 0, C.byref(need)), "debug_copy")
        n = int(need.value)
        raw = np.zeros(max(n, 1), np.uint8)
        if n:
            _check(L.gsm_depthfirst_debug_copy(self._h, int(which), raw.ctypes.data, n, None), "debug_copy")
        raw = raw[:n]
        if which == DepthFirstBuffer.RENDER_DATA:
            return raw.view(STEREO_RENDER_DATA)
        if which == DepthFirstBuffer.BOUNDS:
            return raw.view(np.int32).reshape(-1, 4)
        if which == DepthFirstBuffer.HEADERS:
            return raw.view(np.uint32).reshape(-1, 2)
        if which in (DepthFirstBuffer.DEPTH_ORDER, DepthFirstBuffer.INSTANCE_GAUSSIANS):
            return raw.view(np.int32)
        if which == DepthFirstBuffer.BLEND_STATS:
            return raw.view(np.uint64)
        return raw.view(np.uint32)


def sort_pairs_u32(keys, values, key_bits: int = 32, stream=None):
    """Stable device radix sort of uint32 (key, value) pairs in place (torch int32 tensors)."""
    n = int(keys.numel())
    _check(_lib().gsm_sort_pairs_u32(_ptr(keys), _ptr(values), n, int(key_bits), _stream_handle(stream)),
           "gsm_sort_pairs_u32")


class _MgOptions(C.Structure):
    _fields_ = [("struct_bytes", C.c_uint32), ("rows", C.c_int32), ("pipelined", C.c_int32),
                ("transport", C.c_int32), ("timeout_ms", C.c_uint32), ("reserved", C.c_uint32),
                ("nccl_comm", C.c_void_p)]


MG_ROWS = {"contiguous": 0, "interleaved": 1}
MG_TRANSPORT = {"peer_stores": 0, "rccl": 1}


@dataclass
class MultiGpuOptions:
    """gsm_multigpu_options (include/gsm_multigpu.h): row layout, pipelining, transport, barrier
    timeout, and the RCCL transport's communicator (ncclComm_t as an int)."""
    rows: str = "contiguous"
    pipelined: bool = False
    transport: str = "peer_stores"
    timeout_ms: int = 10000
    nccl_comm: Optional[int] = None

    def _c(self) -> "_MgOptions":
        o = _MgOptions()
        _lib().gsm_multigpu_default_options(C.byref(o))
        o.rows = MG_ROWS[self.rows]
        o.pipelined = 1 if self.pipelined else 0
        o.transport = MG_TRANSPORT[self.transport]
        o.timeout_ms = int(self.timeout_ms)
        o.nccl_comm = C.c_void_p(int(self.nccl_comm)) if self.nccl_comm else None
        return o


class MultiGpuRenderer:
    """gsm_multigpu_* (include/gsm_multigpu.h): one frame of a GlobalRenderer split by tile-row slab
    across the ranks of a node -- counts, records and slab pixels written straight into the owners'
    exchange memory (peer mappings over xGMI), ordered by device-side flag barriers, the bands
    gathered on rank 0 -- all inside libgsm_amd.so, no host round trip and no collective in a frame.

    Two ways to set up (both collective):
      MultiGpuRenderer(renderer, comm, rank, world)       handles exchanged over an RCCL
                                                          communicator (torch: _comm_ptr());
      MultiGpuRenderer.connect(renderer, rank, world, allgather)
                                                          handles exchanged by the caller:
                                                          allgather(bytes) -> list of every rank's
                                                          bytes (e.g. torch.distributed over gloo)."""

    def __init__(self, renderer: "GlobalRenderer", comm: Optional[int], rank: int, world_size: int, _handle=None,
                 options: Optional["MultiGpuOptions"] = None):
        """options None: gsm_multigpu_create (defaults + the environment's test overrides); otherwise
        gsm_multigpu_create_with_options."""
        self.renderer = renderer
        self.rank = int(rank)
        self.world_size = int(world_size)
        if _handle is not None:
            self._h = _handle
            return
        h = C.c_void_p()
        if options is None:
            _check(_lib().gsm_multigpu_create(renderer._h, C.c_void_p(int(comm)), int(rank), int(world_size),
                                              C.byref(h)), "gsm_multigpu_create")
        else:
            o = options._c()
            _check(_lib().gsm_multigpu_create_with_options(renderer._h, C.c_void_p(int(comm)), int(rank),
                                                           int(world_size), C.byref(o), C.byref(h)),
                   "gsm_multigpu_create_with_options")
        self._h = h

    @classmethod
    def prepare(cls, renderer: "GlobalRenderer", rank: int, world_size: int,
                options: Optional["MultiGpuOptions"] = None):
        """gsm_multigpu_prepare (options None) or gsm_multigpu_prepare_with_options: (unconnected
        renderer, this rank's handle bytes)."""
        h = C.c_void_p()
        buf = C.create_string_buffer(MULTIGPU_HANDLE_BYTES)
        if options is None:
            _check(_lib().gsm_multigpu_prepare(renderer._h, int(rank), int(world_size), C.byref(h), buf),
                   "gsm_multigpu_prepare")
        else:
            o = options._c()
            _check(_lib().gsm_multigpu_prepare_with_options(renderer._h, int(rank), int(world_size), C.byref(o),
                                                            C.byref(h), buf), "gsm_multigpu_prepare_with_options")
        return cls(renderer, None, rank, world_size, _handle=h), bytes(buf.raw)

    def connect_handles(self, handles):
        """gsm_multigpu_connect with every rank's handle bytes, in rank order."""
        blob = b"".join(bytes(x) for x in handles)
        if len(blob) != MULTIGPU_HANDLE_BYTES * self.world_size:
            raise ValueError("one handle per rank expected")
        _check(_lib().gsm_multigpu_connect(self._h, C.c_char_p(blob)), "gsm_multigpu_connect")
        return self

    @classmethod
    def connect(cls, renderer: "GlobalRenderer", rank: int, world_size: int, allgather,
                options: Optional["MultiGpuOptions"] = None):
        mg, mine = cls.prepare(renderer, rank, world_size, options)
        try:
            return mg.connect_handles(allgather(mine))
        except Exception:
            mg.close()
            raise

    @staticmethod
    def torch_allgather(data: bytes):
        """Every rank's bytes over torch.distributed's default group (any backend)."""
        import torch.distributed as dist
        out = [None] * dist.get_world_size()
        dist.all_gather_object(out, data)
        return out

    @staticmethod
    def torch_comm(device) -> int:
        """The ncclComm_t of torch.distributed's default NCCL process group on `device`."""
        import torch.distributed as dist
        return int(dist.group.WORLD._get_backend(torch.device("cuda", int(device)))._comm_ptr())

    def _args(self, input, camera, color_texture, depth_texture, width, color_pitch, depth_pitch):
        inp = _Input(_ptr(input.gaussians), _ptr(input.harmonics), int(input.gaussian_count),
                     int(input.sh_components))
        cam = _camera_struct(camera)
        cp = color_pitch if color_pitch is not None else int(width) * 8
        dp = depth_pitch if depth_pitch is not None else int(width) * 2
        return inp, cam, cp, dp

    def render(self, color_texture, depth_texture, input: GaussianInput, camera: CameraParams, width: int,
               height: int, gather: bool = True, stream=None, color_pitch: Optional[int] = None,
               depth_pitch: Optional[int] = None, gather_target=None, gather_depth: Optional[bool] = None):
        """One frame.  gather: rank 0 receives the whole frame -- in color_texture (a copy of the
        library frame), or, with gather_target = self.frame()[0], in the library frame itself; the
        other ranks' color_texture is then unused (may be None).  gather_depth (with gather): rank 0
        also receives the r16f depth -- in depth_texture (a copy) or, when depth_texture is None, in
        the library depth frame (self.frame_depth()); default: whether depth_texture is given (every
        rank must make the same choice: pass it explicitly when only rank 0 holds a depth texture)."""
        self.render_phases(range(4), color_texture, depth_texture, input, camera, width, height, gather, stream,
                           color_pitch, depth_pitch, gather_target, gather_depth)

    def render_phases(self, phases, color_texture, depth_texture, input: GaussianInput, camera: CameraParams,
                      width: int, height: int, gather: bool = True, stream=None, color_pitch: Optional[int] = None,
                      depth_pitch: Optional[int] = None, gather_target=None, gather_depth: Optional[bool] = None):
        """gsm_multigpu_render_phase for each phase in `phases` (virtual ranks: phase p of every rank
        before phase p + 1 of any, include/gsm_multigpu.h).  Every phase is issued even after one
        returned an error (the ranks stay in step); the first error is raised after the last.
        gather_depth as render's."""
        if gather_depth is None:
            gather_depth = depth_texture is not None
        inp, cam, cp, dp = self._args(input, camera, color_texture, depth_texture, width, color_pitch, depth_pitch)
        col = _ptr(color_texture)
        dep = _ptr(depth_texture)
        if gather:  # rank 0: the caller's target (a copy) or else the library frame; others: any non-NULL
            if gather_target is not None:
                g = _ptr(gather_target)
            elif self.rank == 0:
                g = col if col is not None else self.frame()[0]
            else:
                g = 1
            if not gather_depth:
                dep = None
            elif self.rank == 0:
                if dep is None:
                    dep, dp = self.frame_depth()
            else:
                dep = 1
        else:
            g = None
        first = None
        for p in phases:
            st = _lib().gsm_multigpu_render_phase(self._h, int(p), _stream_handle(stream), C.byref(inp), C.byref(cam),
                                                  int(width), int(height), col, cp, dep, dp, g)
            if st != 0 and first is None:
                first = (st, p)
        if first is not None:
            _check(first[0], f"gsm_multigpu_render_phase({first[1]})")

    def finish_frame(self, stream=None):
        """gsm_multigpu_finish_frame: the phases a caller left unfinished (barrier steps; the slab is
        abandoned from phase 2 on), so the ranks stay in step; a no-op when no frame is pending."""
        _check(_lib().gsm_multigpu_finish_frame(self._h, _stream_handle(stream)), "gsm_multigpu_finish_frame")

    def debug_set_epoch(self, epoch: int):
        """gsm_multigpu_debug_set_epoch (tests: reach the 2^31 epoch wrap in a few frames)."""
        _check(_lib().gsm_multigpu_debug_set_epoch(self._h, int(epoch) & 0xFFFFFFFF), "gsm_multigpu_debug_set_epoch")

    def wait_event(self, event):
        """gsm_multigpu_wait_event: the next frame's projection (phase 0) waits for `event` (a
        torch.cuda.Event recorded after the caller wrote this frame's gaussians / harmonics) -- needed
        when pipelined (GSM_MG_PIPELINE=1), where phase 0 runs on the library's own stream."""
        h = event.cuda_event if hasattr(event, "cuda_event") else int(event)
        _check(_lib().gsm_multigpu_wait_event(self._h, C.c_void_p(h)), "gsm_multigpu_wait_event")

    def frame(self):
        """(device pointer, pitch bytes) of rank 0's gathered frame; (None, 0) elsewhere."""
        p = C.c_void_p()
        pitch = C.c_size_t()
        _check(_lib().gsm_multigpu_frame(self._h, C.byref(p), C.byref(pitch)), "gsm_multigpu_frame")
        return p.value, int(pitch.value)

    def frame_depth(self):
        """(device pointer, pitch bytes) of rank 0's gathered r16f depth frame; (None, 0) elsewhere."""
        p = C.c_void_p()
        pitch = C.c_size_t()
        _check(_lib().gsm_multigpu_frame_depth(self._h, C.byref(p), C.byref(pitch)), "gsm_multigpu_frame_depth")
        return p.value, int(pitch.value)

    def copy_depth(self, width: int, height: int) -> np.ndarray:
        """Rank 0: the gathered r16f depth frame as uint16 bits [height, width] (synchronous)."""
        out = np.empty((int(height), int(width)), np.uint16)
        _check(_lib().gsm_multigpu_debug_copy_depth(self._h, out.ctypes.data_as(C.c_void_p), int(width) * 2,
                                                    int(width), int(height)), "gsm_multigpu_debug_copy_depth")
        return out

    def errors(self, clear: bool = False):
        """(barrier timeouts, failed peer arrivals) since create or the last clear."""
        t, f = C.c_uint32(0), C.c_uint32(0)
        _check(_lib().gsm_multigpu_errors(self._h, C.byref(t), C.byref(f), 1 if clear else 0), "gsm_multigpu_errors")
        return int(t.value), int(f.value)

    def copy_frame(self, width: int, height: int) -> np.ndarray:
        """Rank 0: the gathered rgba16f frame as uint16 bits [height, width, 4] (synchronous)."""
        out = np.empty((int(height), int(width), 4), np.uint16)
        _check(_lib().gsm_multigpu_debug_copy_frame(self._h, out.ctypes.data_as(C.c_void_p), int(width) * 8,
                                                    int(width), int(height)), "gsm_multigpu_debug_copy_frame")
        return out

    def copy_exchange(self, nbytes: int) -> np.ndarray:
        """The first nbytes of this rank's exchange memory (control, counts from byte 1024, records
        from byte 4096), synchronous."""
        out = np.empty(int(nbytes), np.uint8)
        _check(_lib().gsm_multigpu_debug_copy_exchange(self._h, out.ctypes.data_as(C.c_void_p), out.size),
               "gsm_multigpu_debug_copy_exchange")
        return out

    def status(self, clear: bool = False) -> int:
        """Barrier timeouts since create (0 on a healthy run)."""
        out = C.c_uint32(0)
        _check(_lib().gsm_multigpu_status(self._h, C.byref(out), 1 if clear else 0), "gsm_multigpu_status")
        return int(out.value)

    def set_timeout_ms(self, ms: int):
        _check(_lib().gsm_multigpu_set_timeout_ms(self._h, int(ms)), "gsm_multigpu_set_timeout_ms")

    def counts(self) -> np.ndarray:
        out = (C.c_uint32 * (self.world_size * self.world_size))()
        _check(_lib().gsm_multigpu_debug_counts(self._h, out), "gsm_multigpu_debug_counts")
        return np.array(out, np.uint32).reshape(self.world_size, self.world_size)

    def close(self):
        if getattr(self, "_h", None) and self._h.value:
            _lib().gsm_multigpu_destroy(self._h)
            self._h = C.c_void_p()

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass


def sort_rank_probe(device: int = 0) -> bool:
    """True when the device serves same-address LDS atomics of one wave in lane order (the sorts'
    default stable ranks); False -> the renderers rank by ballot matches."""
    out = C.c_int(0)
    _check(_lib().gsm_debug_sort_rank_probe(int(device), C.byref(out)), "gsm_debug_sort_rank_probe")
    return bool(out.value)


def abi_version() -> int:
    return int(_lib().gsm_abi_version())
