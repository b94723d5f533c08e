"""DepthFirst stereo side-by-side path (include/gsm_depthfirst.h).

CPU (`-m "not gpu"`): the oracle's restatement of DepthFirstRenderer.renderStereo(.sideBySide)
checked for the properties the reference's pipeline guarantees -- stable 32-bit depth order
(DepthFirstShaders.metal:33-37, DepthRadixSortEncoder), instances of the union rect in depth order
then stably grouped by tile (:790-826, TileSortEncoder), tile ranges by binary search
(:1258-1313), the copy pass's row flip (DepthFirstStereoCopyEncoder.swift:70-98) -- plus the
reference's depth-sort known-answer test (DepthFirstUnitTests.swift:120-305).
GPU (`-m gpu`): the HIP path through the C ABI against the oracle, bit for bit, on every
intermediate buffer and the side-by-side target.  The reference has no image fixtures for this
path either, so, like the Global frame, parity is against the restatement.
"""
import numpy as np
import pytest

from test_gpu_parity import first_diff, to_dev


def _scene(n, w, h, sh, precision, seed, **kw):
    from gsm_amd import scenes
    world, harm, _ = scenes.gen_scene(n, w, h, sh, precision, seed=seed, **kw)
    return world, harm


def _cams(w, h, ipd=0.064):
    from gsm_amd import scenes
    return scenes.make_camera(w, h, -ipd / 2), scenes.make_camera(w, h, ipd / 2)


def _scene_transform():
    """Rotation about y by 0.2 rad, uniform scale 1.25, translation (0.1, -0.05, 0.3); column-major."""
    c, s, k = np.cos(0.2), np.sin(0.2), 1.25
    M = np.array([[c * k, 0, s * k, 0.1], [0, k, 0, -0.05], [-s * k, 0, c * k, 0.3], [0, 0, 0, 1]], np.float32)
    return M.T.reshape(-1).copy()  # column-major flat


# ---------------------------------------------------------------------------
# CPU: oracle properties
# ---------------------------------------------------------------------------
def test_oracle_depth_sort_kat(oracle):
    """DepthFirstUnitTests.testDepthSortSimple (:120-305): keys 10..1 with payload i*100 sort to
    payloads 900, 800, ..., 0.  The oracle's stable depth order restated in numpy terms: a stable
    argsort by the 32-bit key."""
    keys = np.arange(10, 0, -1, dtype=np.uint32)
    payload = np.arange(10, dtype=np.int32) * 100
    order = np.argsort(keys, kind="stable")
    assert payload[order].tolist() == [900, 800, 700, 600, 500, 400, 300, 200, 100, 0]
    # float_to_sortable_uint (DepthFirstShaders.metal:33-37) is monotone over signed floats
    vals = np.array([-5.0, -1.0, -0.0, 0.0, 1e-3, 0.1, 1.0, 9.5, 1e30], np.float32)
    ks = [oracle.lib().og_float_to_sortable(float(v)) for v in vals]
    assert ks == sorted(ks)


def test_oracle_sincos_theta_accuracy(oracle):
    """The numeric-contract sin/cos of the unquantised ellipse angle (gsm_oracle_math.h) is within
    one fp32 rounding of the true value on [0, pi)."""
    th = np.linspace(0, np.pi, 4001, dtype=np.float32)[:-1]
    for t in th[::7]:
        s, c = oracle.sincos_theta(float(t))
        assert abs(s - np.sin(np.float64(t))) <= 1.2e-7 and abs(c - np.cos(np.float64(t))) <= 1.2e-7


@pytest.fixture(scope="module")
def small_frame(oracle):
    n, w, h = 6000, 200, 150
    world, harm = _scene(n, w, h, 9, 1, 7)
    L, R = _cams(w, h)
    r = oracle.df_render_stereo(world, harm, 9, L, R, w, h)
    assert r["status"] == 0
    return r, world


def test_oracle_pipeline_invariants(small_frame):
    r, world = small_frame
    n = len(world)
    touched, keys, order = r["touched"], r["depth_keys"], r["depth_order"]
    vis = np.nonzero(touched > 0)[0]
    assert r["visible"] == len(vis) and 0 < len(vis) <= n
    # stable 32-bit depth order of the visible ids (ascending id among equal keys)
    np.testing.assert_array_equal(order, vis[np.argsort(keys[vis], kind="stable")])
    assert np.all(keys[touched == 0] == 0xFFFFFFFF)
    # union rect area == touched count
    b = r["bounds"]
    area = np.maximum(b[:, 1] - b[:, 0] + 1, 0) * np.maximum(b[:, 3] - b[:, 2] + 1, 0)
    np.testing.assert_array_equal(area[vis], touched[vis])
    assert r["overflow"] == 0 and r["total_instances"] == int(touched.sum())
    # instances: expansion in depth order (ty-major, tx-minor), then a stable tile sort
    tiles_x = r["tiles_x"]
    exp_t, exp_g = [], []
    for g in order:
        x0, x1, y0, y1 = b[g]
        for ty in range(y0, y1 + 1):
            for tx in range(x0, x1 + 1):
                exp_t.append(ty * tiles_x + tx)
                exp_g.append(g)
    exp_t, exp_g = np.array(exp_t), np.array(exp_g)
    srt = np.argsort(exp_t, kind="stable")
    np.testing.assert_array_equal(r["inst_tiles"], exp_t[srt])
    np.testing.assert_array_equal(r["inst_gids"], exp_g[srt])
    # headers: lower bound and count per tile
    t = np.arange(r["tile_count"])
    lo = np.searchsorted(r["inst_tiles"], t, side="left")
    hi = np.searchsorted(r["inst_tiles"], t, side="right")
    np.testing.assert_array_equal(r["headers"][:, 0], lo)
    np.testing.assert_array_equal(r["headers"][:, 1], hi - lo)


def test_oracle_copy_flips_rows(small_frame):
    r, _ = small_frame
    h, w2 = r["color"].shape[:2]
    w = w2 // 2
    for e in range(2):
        np.testing.assert_array_equal(r["color"][:, e * w:(e + 1) * w], r["eye_color"][e][::-1])


def test_oracle_identical_eyes_give_identical_halves(oracle):
    from gsm_amd import scenes
    n, w, h = 3000, 120, 96
    world, harm = _scene(n, w, h, 4, 1, 3)
    cam = scenes.make_camera(w, h, 0.0)
    r = oracle.df_render_stereo(world, harm, 4, cam, cam, w, h)
    np.testing.assert_array_equal(r["color"][:, :w], r["color"][:, w:])
    rd = r["render_data"][r["touched"] > 0]
    for f in ("MeanX", "MeanY", "Cxx", "Cyy", "Cxy2", "Depth"):
        np.testing.assert_array_equal(rd["left" + f], rd["right" + f])


def test_oracle_identity_scene_transform_is_default(oracle):
    n, w, h = 2000, 96, 80
    world, harm = _scene(n, w, h, 1, 0, 5)
    L, R = _cams(w, h)
    a = oracle.df_render_stereo(world, harm, 1, L, R, w, h)
    b = oracle.df_render_stereo(world, harm, 1, L, R, w, h, scene_transform=np.eye(4, dtype=np.float32))
    np.testing.assert_array_equal(a["color"], b["color"])
    c = oracle.df_render_stereo(world, harm, 1, L, R, w, h, scene_transform=_scene_transform())
    assert not np.array_equal(a["color"], c["color"])


def test_oracle_capacity_clamp(oracle):
    """More instances than 4 * max_gaussians: the depth order's tail loses its instances
    (createInstancesStereoKernel writes while writeOffset < maxAssignments) and overflow is set."""
    n, w, h = 3000, 160, 128
    world, harm = _scene(n, w, h, 1, 1, 9, scale_px=3.0)
    L, R = _cams(w, h)
    full = oracle.df_render_stereo(world, harm, 1, L, R, w, h, max_gaussians=4 * n)
    clamped = oracle.df_render_stereo(world, harm, 1, L, R, w, h, max_gaussians=n)
    assert full["overflow"] == 0 and full["total_instances"] > 4 * n
    assert clamped["overflow"] == 1 and clamped["total_instances"] == 4 * n


# ---------------------------------------------------------------------------
# GPU: HIP path through the C ABI, bit-exact against the oracle
# ---------------------------------------------------------------------------
def gpu_df(gsm, torch, world, harm, sh, L, R, w, h, max_gaussians=None, max_width=None, max_height=None,
           color_space=0, color_format=0, scene_transform=None, count=None, renderer=None):
    prec = 1 if world.dtype.itemsize == 32 else 0
    n = len(world) if count is None else count
    own = renderer is None
    if own:
        cfg = gsm.RendererConfig(max_gaussians=max_gaussians or max(n, 1), max_width=max_width or w,
                                 max_height=max_height or h, precision=prec, gaussian_color_space=color_space,
                                 color_format=color_format)
        renderer = gsm.DepthFirstRenderer(config=cfg)
    renderer.set_profiling(True)
    fmt = gsm.ColorFormat(color_format)
    dt = torch.float16 if fmt == gsm.ColorFormat.RGBA16F else (torch.float32 if fmt == gsm.ColorFormat.RGBA32F
                                                                else torch.uint8)
    color = torch.full((h, 2 * w, 4), 7, dtype=dt, device="cuda")
    if dt == torch.float16:
        color.fill_(float("nan"))
    inp = gsm.GaussianInput(to_dev(torch, world), to_dev(torch, harm), n, sh)
    renderer.render_stereo_sbs(color, inp, gsm.CameraParams.from_dict(L), gsm.CameraParams.from_dict(R), w, h,
                               scene_transform=scene_transform)
    torch.cuda.synchronize()
    B = gsm.DepthFirstBuffer
    out = {"counters": renderer.counters(), "stage_ms": renderer.stage_times_ms(), "renderer": renderer}
    c = color.cpu().numpy()
    out["color"] = c.view(np.uint16) if dt == torch.float16 else c
    for name, which in (("render_data", B.RENDER_DATA), ("bounds", B.BOUNDS), ("touched", B.TOUCHED),
                        ("depth_keys", B.DEPTH_KEYS), ("depth_order", B.DEPTH_ORDER),
                        ("inst_tiles", B.INSTANCE_TILES), ("inst_gids", B.INSTANCE_GAUSSIANS),
                        ("headers", B.HEADERS)):
        out[name] = renderer.copy_buffer(which)
    return out


def assert_df_equal(g, r):
    c = g["counters"]
    assert (c["visible"], c["total_instances"], c["overflow"]) == \
        (r["visible"], r["total_instances"], r["overflow"])
    assert (c["tiles_x"], c["tiles_y"]) == (r["tiles_x"], r["tiles_y"])
    np.testing.assert_array_equal(g["touched"], r["touched"], err_msg=first_diff(g["touched"], r["touched"]))
    np.testing.assert_array_equal(g["bounds"], r["bounds"])
    np.testing.assert_array_equal(g["depth_keys"], r["depth_keys"])
    vis = r["touched"] > 0
    grd = g["render_data"].view(np.uint8).reshape(-1, 32)[vis]
    ord_ = r["render_data"].view(np.uint8).reshape(-1, 32)[vis]
    if not np.array_equal(grd, ord_):
        bad = np.nonzero((grd != ord_).any(1))[0][:3]
        raise AssertionError(f"render_data differs at visible rows {bad}: {grd[bad]} vs {ord_[bad]}")
    np.testing.assert_array_equal(g["depth_order"], r["depth_order"])
    np.testing.assert_array_equal(g["inst_tiles"], r["inst_tiles"])
    np.testing.assert_array_equal(g["inst_gids"], r["inst_gids"])
    np.testing.assert_array_equal(g["headers"], r["headers"])
    assert np.array_equal(g["color"], r["color"]), first_diff(g["color"], r["color"])


DF_CASES = {
    # name: (n, w, h, sh, precision, color_space, seed, kwargs)
    "sh2_f16_config5_shape": (30000, 360, 400, 9, 1, 0, 11, {}),
    "sh0_f32_ragged": (12000, 250, 170, 1, 0, 0, 2, {}),
    "sh3_f16_srgb": (20000, 320, 240, 16, 1, 1, 4, {}),
    "sh1_f32_dense": (20000, 128, 96, 4, 0, 0, 8, {"spread": 0.05}),
}


@pytest.mark.gpu
@pytest.mark.parametrize("name", sorted(DF_CASES))
def test_df_bit_exact(gsm, cuda, oracle, name):
    n, w, h, sh, prec, cs, seed, kw = DF_CASES[name]
    world, harm = _scene(n, w, h, sh, prec, seed, **kw)
    L, R = _cams(w, h)
    r = oracle.df_render_stereo(world, harm, sh, L, R, w, h, color_space=cs)
    g = gpu_df(gsm, cuda, world, harm, sh, L, R, w, h, color_space=cs)
    assert_df_equal(g, r)
    g["renderer"].close()


@pytest.mark.gpu
@pytest.mark.parametrize("env", [{"GSM_SORT_WIDE": "0"}, {"GSM_SORT_RANK": "ballot"},
                                 {"GSM_SORT_WIDE": "0", "GSM_SORT_RANK": "ballot"}])
def test_df_sort_switches(gsm, cuda, oracle, monkeypatch, env):
    """The create-time sort switches (gsm_internal.h Tuning): narrow 4 x 8-bit depth passes and two
    tile passes instead of the wide ones (3 x 11/11/10 bits; one pass for this frame's 575 tiles),
    ballot ranks -- every intermediate stays bit-exact."""
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    n, w, h, sh, prec, cs, seed, kw = DF_CASES["sh2_f16_config5_shape"]
    world, harm = _scene(n, w, h, sh, prec, seed, **kw)
    L, R = _cams(w, h)
    r = oracle.df_render_stereo(world, harm, sh, L, R, w, h, color_space=cs)
    g = gpu_df(gsm, cuda, world, harm, sh, L, R, w, h, color_space=cs)
    assert_df_equal(g, r)
    g["renderer"].close()


@pytest.mark.gpu
@pytest.mark.parametrize("kind,n,w,h,sh,seed", [("f16", 30_000, 360, 400, 9, 21), ("f32", 20_000, 250, 170, 1, 22),
                                                 ("f16", 40_000, 640, 480, 16, 23)])
def test_df_adversarial_scenes_bit_exact(gsm, cuda, oracle, kind, n, w, h, sh, seed):
    """The Global path's adversarial inputs (tests/adversarial.py: zero / extreme / inf / NaN scales,
    positions and quaternions, opacities around the cull and outside [0, 1], huge / NaN SH) through the
    DepthFirst stereo frame: every intermediate and the side-by-side target bit for bit."""
    import adversarial
    case = adversarial.scene(kind, n, w, h, sh, seed)
    L, R = _cams(w, h)
    mg = case["max_gaussians"]  # (4 n: room for the large splats' instances, 4 x max_gaussians)
    r = oracle.df_render_stereo(case["world"], case["harm"], sh, L, R, w, h, max_gaussians=mg)
    assert r["status"] == 0 and r["overflow"] == 0
    g = gpu_df(gsm, cuda, case["world"], case["harm"], sh, L, R, w, h, max_gaussians=mg)
    assert_df_equal(g, r)
    g["renderer"].close()


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [31, 35, 37, 41])
def test_df_wide_baseline_ragged_frames(gsm, cuda, oracle, seed):
    """Eyes far apart (a baseline of 2-4 scene units instead of 0.064) on ragged frame sizes: many
    gaussians are on screen in one eye only, so the other eye's mean fails the reference's mean test
    (gMean.x >= -60000) and k_df_expand flags that eye for every instance -- the blend walks only the
    unflagged entries and takes their means as valid without testing them.  Every
    intermediate and the side-by-side target bit for bit."""
    rng = np.random.default_rng(seed)
    w, h = int(rng.integers(97, 400)), int(rng.integers(61, 300))
    n = int(rng.integers(8000, 25000))
    sh = int(rng.choice([1, 4, 9, 16]))
    prec = int(rng.integers(0, 2))
    world, harm = _scene(n, w, h, sh, prec, seed)
    L, R = _cams(w, h, ipd=float(rng.uniform(2.0, 4.0)))
    r = oracle.df_render_stereo(world, harm, sh, L, R, w, h, max_gaussians=4 * n)
    assert r["status"] == 0 and r["overflow"] == 0
    # one-eye gaussians exist (mean -1e10 -> fp16 -inf in the eye the gaussian misses)
    rd = r["render_data"].view(np.uint16).reshape(-1, 16)[r["touched"] > 0]
    assert ((rd[:, 0] == 0xFC00) != (rd[:, 6] == 0xFC00)).sum() > 100
    g = gpu_df(gsm, cuda, world, harm, sh, L, R, w, h, max_gaussians=4 * n)
    assert_df_equal(g, r)
    g["renderer"].close()


@pytest.mark.gpu
def test_df_scene_transform(gsm, cuda, oracle):
    n, w, h = 15000, 240, 200
    world, harm = _scene(n, w, h, 9, 1, 12)
    L, R = _cams(w, h)
    M = _scene_transform()
    r = oracle.df_render_stereo(world, harm, 9, L, R, w, h, scene_transform=M)
    g = gpu_df(gsm, cuda, world, harm, 9, L, R, w, h, scene_transform=M)
    assert_df_equal(g, r)
    g["renderer"].close()


@pytest.mark.gpu
def test_df_overflow_and_reuse(gsm, cuda, oracle):
    """Instance capacity clamp bit-exact, then the same handle renders a smaller frame inside its
    maxima (width/height < max, fewer gaussians than max) correctly."""
    n, w, h = 3000, 160, 128
    world, harm = _scene(n, w, h, 1, 1, 9, scale_px=3.0)
    L, R = _cams(w, h)
    r = oracle.df_render_stereo(world, harm, 1, L, R, w, h, max_gaussians=n)
    g = gpu_df(gsm, cuda, world, harm, 1, L, R, w, h, max_gaussians=n)
    assert r["overflow"] == 1
    assert_df_equal(g, r)
    rend = g["renderer"]
    w2, h2, n2 = 100, 72, 2000
    world2, harm2 = _scene(n2, w2, h2, 1, 1, 10)
    L2, R2 = _cams(w2, h2)
    r2 = oracle.df_render_stereo(world2, harm2, 1, L2, R2, w2, h2, max_gaussians=n, max_width=w, max_height=h)
    g2 = gpu_df(gsm, cuda, world2, harm2, 1, L2, R2, w2, h2, renderer=rend)
    assert_df_equal(g2, r2)
    rend.close()


@pytest.mark.gpu
def test_df_empty_frame_and_errors(gsm, cuda, oracle):
    w, h = 64, 48
    L, R = _cams(w, h)
    world = np.zeros(0, dtype=_scene(1, w, h, 1, 1, 0)[0].dtype)
    r = oracle.df_render_stereo(world, np.zeros(0, np.uint16), 1, L, R, w, h, max_gaussians=16)
    g = gpu_df(gsm, cuda, world, np.zeros(0, np.uint16), 1, L, R, w, h, max_gaussians=16)
    assert_df_equal(g, r)
    assert np.all(g["color"][..., 3] == 0x3C00) and np.all(g["color"][..., :3] == 0)
    rend = g["renderer"]
    x = cuda.zeros(16, dtype=cuda.uint8, device="cuda")
    cam = gsm.CameraParams.from_dict(L)
    with pytest.raises(gsm.RendererError) as e:
        rend.render_stereo_sbs(x, gsm.GaussianInput(x, x, 17, 1), cam, cam, w, h)
    assert e.value.status == gsm.Status.INVALID_GAUSSIAN_COUNT
    with pytest.raises(gsm.RendererError) as e:
        rend.render_stereo_sbs(x, gsm.GaussianInput(x, x, 1, 1), cam, cam, w + 1, h)
    assert e.value.status == gsm.Status.INVALID_DIMENSIONS
    with pytest.raises(gsm.RendererError) as e:
        rend.render_stereo_sbs(x, gsm.GaussianInput(x, x, 1, 1), cam, cam, w, h, color_pitch=2 * w * 8 - 8)
    assert e.value.status == gsm.Status.INVALID_BUFFER_SIZE
    rend.close()
    with pytest.raises(gsm.RendererError) as e:  # 16-bit tile ids: at most 65535 16x16 tiles
        gsm.DepthFirstRenderer(config=gsm.RendererConfig(max_gaussians=16, max_width=8192, max_height=8192))
    assert e.value.status == gsm.Status.INVALID_TILE_COUNT


@pytest.mark.gpu
@pytest.mark.parametrize("fmt", [1, 2, 3, 4, 5])
def test_df_color_formats(gsm, cuda, oracle, fmt):
    n, w, h = 8000, 160, 120
    world, harm = _scene(n, w, h, 4, 1, 13)
    L, R = _cams(w, h)
    r = oracle.df_render_stereo(world, harm, 4, L, R, w, h)
    want = oracle.convert_color(r["color"], fmt)
    g = gpu_df(gsm, cuda, world, harm, 4, L, R, w, h, color_format=fmt)
    if fmt == 1:
        np.testing.assert_array_equal(g["color"].view(np.uint32), want.view(np.uint32))
    else:
        np.testing.assert_array_equal(g["color"], want)
    g["renderer"].close()


@pytest.mark.gpu
def test_df_config5_full_size(gsm, cuda, oracle):
    """BASELINE configs[4] (1M, SH2, 2 x 1440x1600, fp16) end to end, with the reference's default
    RendererConfig.maxGaussians (6M, GaussianRendererProtocol.swift:212) so no instance is clamped."""
    from gsm_amd import scenes
    c = scenes.CONFIGS["cfg5_1m_sh2_stereo_2x1440x1600_f16"]
    n, w, h = c["count"], c["width"], c["height"]
    world, harm = _scene(n, w, h, c["sh"], c["precision"], 42)
    L, R = _cams(w, h)
    r = oracle.df_render_stereo(world, harm, c["sh"], L, R, w, h, max_gaussians=6_000_000)
    g = gpu_df(gsm, cuda, world, harm, c["sh"], L, R, w, h, max_gaussians=6_000_000)
    assert r["overflow"] == 0
    assert_df_equal(g, r)
    g["renderer"].close()


@pytest.mark.gpu
def test_df_wide_frame_and_schedule_independence(gsm, cuda, oracle):
    """Per-eye width 2100 (> 2048: fp16 pixel coordinates round, the blend's skip test must stand
    aside there) and three frames on one handle: the unit order of frames 2 and 3 comes from the
    previous frame's walk costs, the image must not change."""
    from gsm_amd import scenes
    n, w, h = 20000, 2100, 96
    world, harm = _scene(n, w, h, 4, 1, 17, spread=0.9)
    L, R = scenes.make_camera(w, h, -0.032), scenes.make_camera(w, h, 0.032)
    r = oracle.df_render_stereo(world, harm, 4, L, R, w, h)
    g = gpu_df(gsm, cuda, world, harm, 4, L, R, w, h)
    assert_df_equal(g, r)
    for _ in range(2):
        g2 = gpu_df(gsm, cuda, world, harm, 4, L, R, w, h, renderer=g["renderer"])
        assert np.array_equal(g2["color"], r["color"]), first_diff(g2["color"], r["color"])
    g["renderer"].close()
