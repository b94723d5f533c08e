"""C-ABI surface of libgsm_amd.so: loads, exports every declared symbol, struct layouts
match the headers, and the host-side validation that needs no GPU."""
import ctypes as C
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADERS = [os.path.join(ROOT, "include", h) for h in ("gsm_renderer.h", "gsm_debug.h", "gsm_multigpu.h",
                                                            "gsm_depthfirst.h")]
PLY_HEADER = os.path.join(ROOT, "include", "gsm_ply.h")


def declared_functions(headers=HEADERS):
    names = set()
    for h in headers:
        src = open(h).read()
        src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
        for m in re.finditer(r"\b(gsm_[a-z0-9_]+)\s*\(", src):
            names.add(m.group(1))
    return sorted(names)


def test_library_exports_every_declared_symbol(gsm):
    L = gsm._lib()
    missing = [n for n in declared_functions() if not hasattr(L, n)]
    assert not missing, missing
    assert set(declared_functions()) == set(gsm._SIGNATURES), "binding must cover the headers"
    out = subprocess.run(["nm", "-D", "--defined-only", gsm.library_path()], capture_output=True,
                         text=True, check=True).stdout
    exported = set(re.findall(r" T (gsm_[a-z0-9_]+)", out))
    assert set(declared_functions()) <= exported


def test_ply_header_symbols_exported_and_bound(gsm):
    from gsm_amd import ply
    names = set(declared_functions([PLY_HEADER]))
    assert names == set(ply._SIG), "the ply binding must cover include/gsm_ply.h"
    out = subprocess.run(["nm", "-D", "--defined-only", gsm.library_path()], capture_output=True,
                         text=True, check=True).stdout
    assert names <= set(re.findall(r" T (gsm_[a-z0-9_]+)", out))


def test_library_has_no_unresolved_internal_symbols(gsm):
    """Every gsm:: function the library calls is defined in it (a lazily bound ctypes load
    would only fail at the first call, on the GPU box)."""
    out = subprocess.run(["nm", "-DC", "--undefined-only", gsm.library_path()], capture_output=True,
                         text=True, check=True).stdout
    assert not [l for l in out.splitlines() if "gsm::" in l or " gsm_" in l], out


def test_struct_sizes_match_headers(gsm, tmp_path):
    prog = tmp_path / "sizes.c"
    prog.write_text('#include "gsm_debug.h"\n#include <stdio.h>\n'
                    'int main(void){printf("%zu %zu %zu %zu\\n", sizeof(gsm_renderer_config),'
                    ' sizeof(gsm_gaussian_input), sizeof(gsm_camera_params),'
                    ' sizeof(gsm_debug_counters));return 0;}\n')
    exe = tmp_path / "sizes"
    subprocess.run(["gcc", "-I", os.path.join(ROOT, "include"), str(prog), "-o", str(exe)], check=True)
    sizes = [int(x) for x in subprocess.run([str(exe)], capture_output=True, text=True,
                                            check=True).stdout.split()]
    assert sizes == [C.sizeof(gsm._Config), C.sizeof(gsm._Input), C.sizeof(gsm._Camera),
                     C.sizeof(gsm._Counters)]


def test_multigpu_options_layout_and_defaults(gsm, tmp_path):
    """gsm_multigpu_options (include/gsm_multigpu.h, r06): the C struct and the ctypes mirror agree, and
    gsm_multigpu_default_options (host only) fills the defaults the mirror relies on."""
    prog = tmp_path / "mgo.c"
    prog.write_text('#include "gsm_multigpu.h"\n#include <stdio.h>\n#include <stddef.h>\n'
                    'int main(void){printf("%zu %zu %zu\\n", sizeof(gsm_multigpu_options),'
                    ' offsetof(gsm_multigpu_options, timeout_ms), offsetof(gsm_multigpu_options, nccl_comm));return 0;}\n')
    exe = tmp_path / "mgo"
    subprocess.run(["gcc", "-I", os.path.join(ROOT, "include"), str(prog), "-o", str(exe)], check=True)
    sizes = [int(x) for x in subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.split()]
    assert sizes == [C.sizeof(gsm._MgOptions), gsm._MgOptions.timeout_ms.offset, gsm._MgOptions.nccl_comm.offset]
    o = gsm._MgOptions()
    gsm._lib().gsm_multigpu_default_options(C.byref(o))
    assert (o.struct_bytes, o.rows, o.pipelined, o.transport, o.timeout_ms) == (C.sizeof(o), 0, 0, 0, 10000)
    assert not o.nccl_comm
    c = gsm.MultiGpuOptions(rows="interleaved", transport="rccl", timeout_ms=5)._c()
    assert (c.rows, c.transport, c.timeout_ms) == (1, 1, 5)


def test_status_strings_and_defaults(gsm):
    L = gsm._lib()
    assert L.gsm_abi_version() == 1
    for s in gsm.Status:
        assert L.gsm_status_string(int(s))
    cfg = gsm._Config()
    L.gsm_renderer_config_default(C.byref(cfg))
    # RendererConfig() defaults (GaussianRendererProtocol.swift:211-219)
    assert (cfg.max_gaussians, cfg.max_width, cfg.max_height) == (6_000_000, 1920, 1080)
    assert cfg.precision == gsm.RenderPrecision.FLOAT16
    assert cfg.gaussian_color_space == gsm.GaussianColorSpace.SRGB
    cam = gsm._Camera()
    L.gsm_camera_params_init(C.byref(cam), None, None, None, 1.0, 2.0)
    assert abs(cam.near_plane - 0.1) < 1e-7 and cam.far_plane == 10.0


def test_create_rejects_too_many_gaussians_without_touching_the_gpu(gsm):
    # GlobalRenderer.init guard: maxGaussians <= 30_000_000 (GlobalRenderer.swift:111-113)
    with pytest.raises(gsm.RendererError) as e:
        gsm.GlobalRenderer(config=gsm.RendererConfig(max_gaussians=30_000_001))
    assert e.value.status == gsm.Status.INVALID_GAUSSIAN_COUNT


def test_create_rejects_unknown_color_format_without_touching_the_gpu(gsm):
    # gsm_color_format: RGBA16F .. BGRA8_UNORM_SRGB (include/gsm_renderer.h)
    with pytest.raises(gsm.RendererError) as e:
        gsm.GlobalRenderer(config=gsm.RendererConfig(max_gaussians=1000, color_format=6))
    assert e.value.status == gsm.Status.INVALID_ARGUMENT
    assert [f.bytes_per_pixel for f in gsm.ColorFormat] == [8, 16, 4, 4, 4, 4]


def test_create_without_device_reports_device_not_available(gsm):
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is visible")
    with pytest.raises(gsm.RendererError) as e:
        gsm.GlobalRenderer(config=gsm.RendererConfig(max_gaussians=1000))
    assert e.value.status == gsm.Status.DEVICE_NOT_AVAILABLE


def test_null_handle_arguments(gsm):
    L = gsm._lib()
    assert L.gsm_global_render(None, None, None, None, 1, 1, None, 0, None, 0) == gsm.Status.INVALID_ARGUMENT
    assert L.gsm_global_render_stereo(None, None, None, None, None, 1, 1, None, 0, None, 0) == \
        gsm.Status.INVALID_ARGUMENT
    assert L.gsm_global_debug_read_total_assignments(None) == 0
    L.gsm_global_destroy(None)


@pytest.mark.parametrize("capacity", [1, 4096, 4096 * 1024 + 1, 4_000_000, 20_000_000, 24_000_000])
def test_sort_workspace_guard(gsm, capacity):
    """every pass a sort plans is checked against its digit-count workspace before
    anything launches.  The renderers' own allocation (gsm_debug_sort_workspace_bytes) fits every plan
    they make -- 32-bit depth keys in 3 wide or 4 narrow passes, the 16-bit tile field in 2 narrow
    passes, one 9..11-bit wide pass -- and a workspace one word short of the widest pass is refused
    with GSM_ERR_INVALID_ASSIGNMENT_CAPACITY (host only: no GPU)."""
    L = gsm._lib()
    ws = L.gsm_debug_sort_workspace_bytes(capacity)
    plans = [(32, 1), (32, 0), (16, 0), (12, 0), (11, 1), (9, 1), (8, 0)]
    for bits, wide in plans:
        assert L.gsm_debug_sort_plan_fits(capacity, bits, wide, ws) == 0, (bits, wide)
    # the widest pass of this capacity is the one radix_workspace_bytes was sized for
    short = [L.gsm_debug_sort_plan_fits(capacity, bits, wide, ws - 4) for bits, wide in plans]
    assert gsm.Status.INVALID_ASSIGNMENT_CAPACITY in short
    for bits, wide in plans:
        assert L.gsm_debug_sort_plan_fits(capacity, bits, wide, 0) == gsm.Status.INVALID_ASSIGNMENT_CAPACITY
    assert L.gsm_debug_sort_plan_fits(capacity, 0, 0, ws) == gsm.Status.INVALID_ARGUMENT
