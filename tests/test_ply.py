"""PLY ingestion (include/gsm_ply.h): the product loader
(gsm-renderer_amd/csrc/gsm_ply.cpp) against the numpy restatement oracle/ply_oracle.py of
PLYLoader.swift / Scene.swift, on files written by tests/ply_util.py.  Parity against the
reference itself is unpinned (no PLY fixture or test vector ships with it).  Exact where
both sides do the same float32 operations; exp / 1/(1+exp) / quaternion normalisation within
4 ulp (C library vs numpy transcendental implementations)."""
import os
import sys

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path[:0] = [HERE, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "gsm-renderer_amd")]
import ply_oracle as PO  # noqa: E402
import ply_util as PU  # noqa: E402

ply = pytest.importorskip("gsm_amd.ply")


def ulps(a, b):
    a = np.asarray(a, np.float32).reshape(-1)
    b = np.asarray(b, np.float32).reshape(-1)
    ai = a.view(np.int32).astype(np.int64)
    bi = b.view(np.int32).astype(np.int64)
    ai = np.where(ai < 0, -(ai & 0x7FFFFFFF), ai)
    bi = np.where(bi < 0, -(bi & 0x7FFFFFFF), bi)
    return int(np.abs(ai - bi).max()) if a.size else 0


def check(ds, ref, tol=4):
    assert ds.count == len(ref["pos"])
    assert ds.sh_components == ref["sh"] and ds.compressed == ref["compressed"]
    np.testing.assert_array_equal(ds.positions, ref["pos"])
    np.testing.assert_array_equal(ds.harmonics, ref["harmonics"])
    assert ulps(ds.scales, ref["scale"]) <= tol
    assert ulps(ds.opacities, ref["opacity"]) <= tol
    assert ulps(ds.rotations, ref["rot"]) <= tol


@pytest.mark.parametrize("log_scale,logit,sh", [(True, True, 16), (False, False, 9), (True, False, 4), (False, True, 1)])
def test_standard_matches_restatement(tmp_path, log_scale, logit, sh):
    rng = np.random.default_rng(7 + sh)
    data = PU.standard(PU.gaussian_columns(rng, 3000, sh, log_scale, logit, shuffle=True))
    p = tmp_path / "s.ply"
    p.write_bytes(data)
    ds = ply.load(str(p))
    check(ds, PO.load(data))
    # detection took the branch the data was written for
    if not log_scale:
        np.testing.assert_array_less(ds.scales, 0.25)
    assert ds.sh_components == sh


def test_placeholders_types_aliases_and_crlf():
    rng = np.random.default_rng(3)
    n = 500
    s = rng.uniform(-5, -1, (n, 3))
    op = rng.normal(0, 2, n)
    s[::7] = 2.0  # placeholder vertices (PLYLoader.swift:655-657)
    op[::7] = 4.8402
    cols = [("PX", "double", rng.normal(0, 1, n)), ("py", "float", rng.normal(0, 1, n)),
            ("position_z", "short", rng.integers(-50, 50, n)), ("sx", "float", s[:, 0]), ("scale1", "float", s[:, 1]),
            ("scale_z", "float", s[:, 2]), ("qw", "float", rng.normal(0, 1, n)), ("rotation_x", "float", rng.normal(0, 1, n)),
            ("rot2", "float", rng.normal(0, 1, n)), ("qz", "int", rng.integers(-3, 3, n)), ("alpha", "float", op),
            ("sh_2", "float", rng.normal(0, 1, n)), ("sh_0", "float", rng.normal(0, 1, n)), ("sh_1", "float", rng.normal(0, 1, n)),
            ("red", "uchar", rng.integers(0, 255, n))]
    data = PU.standard(cols, eol="\r\n", extra_header=("obj_info generated",))
    ds = ply.load_bytes(data)
    ref = PO.load(data)
    assert ds.count == n - len(range(0, n, 7))
    check(ds, ref)


def test_uint8_opacity_is_normalised_and_sh_stride_not_multiple_of_3():
    rng = np.random.default_rng(5)
    n = 200
    cols = [("x", "float", rng.normal(0, 1, n)), ("y", "float", rng.normal(0, 1, n)), ("z", "float", rng.normal(0, 1, n)),
            ("opacity", "uchar", rng.integers(0, 256, n))] + [(f"f_dc_{i}", "float", rng.normal(0, 1, n)) for i in range(3)] \
        + [("f_rest_0", "float", rng.normal(0, 1, n))]
    data = PU.standard(cols)
    ds = ply.load_bytes(data)
    check(ds, PO.load(data))
    assert ds.harmonics.size == n * 4  # dataset.harmonics keeps the file's coefficient stride


def test_compressed_matches_restatement():
    rng = np.random.default_rng(11)
    for n, sh in ((1000, True), (256, False), (1, True)):
        data = PU.compressed(rng, n, with_sh=sh)
        ds = ply.load_bytes(data)
        assert ds.compressed and ds.sh_components == 1
        check(ds, PO.load(data), tol=4)


def test_bounds_morton_and_pack():
    rng = np.random.default_rng(2)
    data = PU.standard(PU.gaussian_columns(rng, 5000, 16))
    ds = ply.load_bytes(data)
    ref = PO.load(data)
    c, r = ds.bounds()
    rc, rr = PO.bounds(ref["pos"], ref["scale"])
    np.testing.assert_array_equal(c, rc)
    assert abs(r - rr) <= 1e-5 * max(1.0, rr)
    order = PO.morton_order(ds.positions.copy())
    pos0, harm0 = ds.positions.copy(), ds.harmonics.reshape(ds.count, -1).copy()
    ds.sort_morton()
    np.testing.assert_array_equal(ds.positions, pos0[order])
    np.testing.assert_array_equal(ds.harmonics.reshape(ds.count, -1), harm0[order])
    w32, h32 = ds.pack(0)
    np.testing.assert_array_equal(w32["px"], ds.positions[:, 0])
    np.testing.assert_array_equal(w32["rot"], ds.rotations)
    np.testing.assert_array_equal(w32["sx"], ds.scales[:, 0])
    np.testing.assert_array_equal(h32, ds.harmonics)
    w16, h16 = ds.pack(1)
    np.testing.assert_array_equal(w16["opacity"], ds.opacities.astype(np.float16).view(np.uint16))
    np.testing.assert_array_equal(w16["rw"], ds.rotations[:, 3].astype(np.float16).view(np.uint16))
    np.testing.assert_array_equal(w16["sz"], ds.scales[:, 2].astype(np.float16).view(np.uint16))
    np.testing.assert_array_equal(h16, ds.harmonics.astype(np.float16).view(np.uint16))


BAD = [
    (b"ply\nformat binary_little_endian 1.0\nelement vertex 1\nproperty float x\n", "INVALID_HEADER"),
    (b"ply\nformat ascii 1.0\nelement vertex 0\nproperty float x\nend_header\n", "UNSUPPORTED_FORMAT"),
    (b"ply\nformat binary_big_endian 1.0\nelement vertex 0\nproperty float x\nend_header\n", "UNSUPPORTED_FORMAT"),
    (b"ply\nformat binary_little_endian 1.0\nelement face 0\nproperty float x\nend_header\n", "MISSING_VERTEX_ELEMENT"),
    (b"ply\nformat binary_little_endian 1.0\nelement vertex 0\nproperty float x\nproperty float y\nend_header\n",
     "MISSING_REQUIRED_PROPERTIES"),
    (b"ply\nformat binary_little_endian 1.0\nelement vertex 0\nproperty float x\nproperty float y\nproperty float z\n"
     b"property list uchar int idx\nend_header\n", "LIST_PROPERTIES_NOT_SUPPORTED"),
    (b"ply\nformat binary_little_endian 1.0\nelement vertex 2\nproperty float x\nproperty float y\nproperty float z\n"
     b"end_header\n" + b"\0" * 20, "INSUFFICIENT_DATA"),
    (b"ply\nformat binary_little_endian 1.0\nelement vertex 0\nbogus 1\nend_header\n", "HEADER_UNKNOWN_KEYWORD"),
    (b"ply\nelement vertex 0\nend_header\n", "HEADER_UNEXPECTED_KEYWORD"),
    (b"ply\nformat binary_little_endian 1.0\nformat binary_little_endian 1.0\nend_header\n", "HEADER_UNEXPECTED_KEYWORD"),
    (b"ply\nformat binary_little_endian 1.0\nproperty float x\nend_header\n", "HEADER_UNEXPECTED_KEYWORD"),
    (b"ply\nformat binary_little_endian\nend_header\n", "HEADER_INVALID_LINE"),
    (b"ply\nformat binary_little_endian 1.0\nelement vertex 1x\nend_header\n", "HEADER_INVALID_LINE"),
    (b"ply\nformat binary_little_endian 1.0 \nend_header\n", "HEADER_INVALID_LINE"),
    (b"ply\nformat binary_middle_endian 1.0\nend_header\n", "HEADER_INVALID_FORMAT_TYPE"),
    (b"ply\nformat binary_little_endian 1.0\nelement vertex 0\nproperty half x\nend_header\n", "HEADER_UNKNOWN_PROPERTY_TYPE"),
    (b"ply\ncomment only\nend_header\n", "HEADER_FORMAT_MISSING"),
    (b"ply\ncomment \xc3\xa9\nformat binary_little_endian 1.0\nend_header\n", "HEADER_INVALID_CHARACTERS"),
    (b"ply\nformat binary_little_endian 1.0\nelement chunk 1\nproperty float min_x\nelement vertex 300\n"
     b"property uint packed_position\nproperty uint packed_rotation\nproperty uint packed_scale\nproperty uint packed_color\n"
     b"end_header\n" + b"\0" * (4 + 300 * 16), "INSUFFICIENT_DATA"),
    # a property read as 4 bytes but declared narrower, last in its element: the read would run past
    # the end of the file (the reference reads it unchecked, PLYLoader.swift:318-334)
    (b"ply\nformat binary_little_endian 1.0\nelement chunk 1\nproperty float min_y\nproperty ushort min_x\n"
     b"element vertex 1\nproperty uint packed_position\nproperty uint packed_rotation\nproperty uint packed_scale\n"
     b"property uint packed_color\nend_header\n" + b"\0" * (6 + 16), "INSUFFICIENT_DATA"),
    (b"ply\nformat binary_little_endian 1.0\nelement chunk 1\nproperty float min_x\n"
     b"element vertex 1\nproperty uint packed_position\nproperty uint packed_rotation\nproperty uint packed_scale\n"
     b"property uchar packed_color\nend_header\n" + b"\0" * (4 + 13), "INSUFFICIENT_DATA"),
]


@pytest.mark.parametrize("data,status", BAD)
def test_errors_like_the_reference(data, status):
    with pytest.raises(ply.PLYLoaderError) as e:
        ply.load_bytes(data)
    assert e.value.status.name == status


def test_missing_file():
    with pytest.raises(ply.PLYLoaderError) as e:
        ply.load("/nonexistent/scene.ply")
    assert e.value.status == ply.PLYStatus.IO


@pytest.mark.gpu
def test_ply_scene_renders_bit_exact(tmp_path):
    """PLY -> GaussianInput (PackedWorldGaussianHalf + fp16 SH3) -> GPU frame == oracle frame."""
    import torch
    import gsm_amd
    import oracle as O
    from gsm_amd import scenes
    rng = np.random.default_rng(9)
    n, W, H = 20000, 640, 360
    cols = PU.gaussian_columns(rng, n, 16)
    # place the cloud in front of the default camera (z ~ 3..8) with visible sizes
    cols[0] = ("x", "float", rng.uniform(-2, 2, n))
    cols[1] = ("y", "float", rng.uniform(-1.2, 1.2, n))
    cols[2] = ("z", "float", rng.uniform(3, 8, n))
    data = PU.standard(cols)
    ds = ply.load_bytes(data)
    ds.positions  # recentred by the loader; shift back in front of the camera via the view matrix
    world, harm = ds.pack(1)
    cam = scenes.make_camera(W, H)
    cam["view"] = cam["view"].copy()
    cam["view"][14] = np.float32(5.5)  # translate the recentred cloud to z ~ 5.5
    r = gsm_amd.GlobalRenderer(config=gsm_amd.RendererConfig(max_gaussians=ds.count, max_width=W, max_height=H,
                                                             precision=1, gaussian_color_space=0))
    dev = torch.device("cuda", 0)
    wt = torch.from_numpy(world.view(np.uint8).copy()).to(dev)
    ht = torch.from_numpy(harm.view(np.uint8).copy()).to(dev)
    color = torch.full((H, W, 4), float("nan"), dtype=torch.float16, device=dev)
    depth = torch.full((H, W), float("nan"), dtype=torch.float16, device=dev)
    r.render(color, depth, gsm_amd.GaussianInput(wt, ht, ds.count, ds.sh_components),
             gsm_amd.CameraParams.from_dict(cam), W, H)
    torch.cuda.synchronize()
    ref = O.render(world, harm, ds.sh_components, cam, W, H, max_gaussians=ds.count)
    assert ref["total_assignments"] > 10000
    np.testing.assert_array_equal(color.view(torch.int16).cpu().numpy().view(np.uint16), ref["color"])
    np.testing.assert_array_equal(depth.view(torch.int16).cpu().numpy().view(np.uint16), ref["depth"])
    r.close()
