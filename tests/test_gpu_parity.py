"""GPU parity: the HIP path (through the C ABI) against the C oracle, bit-exact.

Every intermediate of the reference's frame is compared: GaussianRenderData of the
visible gaussians, tile bounds, per-gaussian tile counts, unsorted and sorted keys /
indices, tile headers, and the rgba16f colour + r16f depth targets
(north star: headers/permutation bit-exact, colour within 1 fp16 ULP -- we require 0).
"""
import os
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from golden import make_golden as MG  # noqa: E402


def to_dev(torch, arr):
    a = np.ascontiguousarray(arr)
    if a.size == 0:
        return torch.zeros(16, dtype=torch.uint8, device="cuda")
    return torch.from_numpy(a.view(np.uint8).reshape(-1).copy()).cuda()


def gpu_render(gsm, torch, case, renderer=None, color_fill=None, keep=True, depth=True):
    w, h = case["width"], case["height"]
    maxw, maxh = case.get("max_width", w), case.get("max_height", h)
    prec = 1 if case["world"].dtype.itemsize == 32 else 0
    own = renderer is None
    if own:
        cfg = gsm.RendererConfig(max_gaussians=case["max_gaussians"], max_width=maxw, max_height=maxh,
                                 precision=prec, gaussian_color_space=case.get("color_space", 0))
        renderer = gsm.GlobalRenderer(config=cfg)
    renderer.set_profiling(stage_events=True, keep_unsorted=keep, capture=True)
    world = to_dev(torch, case["world"])
    harm = to_dev(torch, case["harm"])
    n = len(case["world"]) if case.get("count") is None else case["count"]
    color = torch.empty((h, w, 4), dtype=torch.float16, device="cuda")
    if color_fill is not None:
        color.fill_(color_fill)
    else:
        color.fill_(float("nan"))
    dep = torch.full((h, w), float("nan"), dtype=torch.float16, device="cuda") if depth else None
    inp = gsm.GaussianInput(world, harm, n, case["sh"])
    cam = gsm.CameraParams.from_dict(case["cam"])
    renderer.render(color, dep, inp, cam, w, h)
    torch.cuda.synchronize()
    out = {
        "color": color.view(torch.int16).cpu().numpy().view(np.uint16),
        "depth": dep.view(torch.int16).cpu().numpy().view(np.uint16) if depth else None,
        "counters": renderer.counters(),
        "render_data": renderer.copy_buffer(gsm.BufferId.RENDER_DATA),
        "bounds": renderer.copy_buffer(gsm.BufferId.BOUNDS),
        "tile_counts": renderer.copy_buffer(gsm.BufferId.TILE_COUNTS),
        "sorted_keys": renderer.copy_buffer(gsm.BufferId.SORTED_KEYS),
        "sorted_values": renderer.copy_buffer(gsm.BufferId.SORTED_VALUES),
        "headers": renderer.copy_buffer(gsm.BufferId.HEADERS),
        "stage_ms": renderer.stage_times_ms(),
        "renderer": renderer,
    }
    if keep:
        out["keys"] = renderer.copy_buffer(gsm.BufferId.KEYS)
        out["values"] = renderer.copy_buffer(gsm.BufferId.VALUES)
    return out


def oracle_render(oracle, case):
    return oracle.render(case["world"], case["harm"], case["sh"], case["cam"], case["width"],
                         case["height"], max_gaussians=case["max_gaussians"],
                         max_width=case.get("max_width"), max_height=case.get("max_height"),
                         color_space=case.get("color_space", 0), count=case.get("count"))


def first_diff(a, b):
    a = np.asarray(a).reshape(-1)
    b = np.asarray(b).reshape(-1)
    if a.shape != b.shape:
        return f"shape {a.shape} vs {b.shape}"
    idx = np.nonzero(a != b)[0]
    return f"{idx.size} diffs, first at {idx[:5].tolist()}: gpu {a[idx[:5]].tolist()} oracle {b[idx[:5]].tolist()}"


def assert_frame_equal(g, r, stages=True):
    c = g["counters"]
    assert c["total_assignments"] == r["total_assignments"]
    assert c["overflow"] == r["overflow"]
    if stages:
        vis = r["mask"].astype(bool)
        gv = g["render_data"][vis].view(np.uint8)
        rv = r["render_data"][vis].view(np.uint8)
        assert np.array_equal(gv, rv), "render data: " + first_diff(gv, rv)
        assert np.array_equal(g["bounds"], r["bounds"]), "bounds: " + first_diff(g["bounds"], r["bounds"])
        assert np.array_equal(g["tile_counts"], r["tile_counts"]), \
            "tile counts: " + first_diff(g["tile_counts"], r["tile_counts"])
        if "keys" in g:
            assert np.array_equal(g["keys"], r["keys"]), "keys: " + first_diff(g["keys"], r["keys"])
            assert np.array_equal(g["values"], r["values"]), "values: " + first_diff(g["values"], r["values"])
        assert np.array_equal(g["sorted_keys"], r["sorted_keys"]), \
            "sorted keys: " + first_diff(g["sorted_keys"], r["sorted_keys"])
        assert np.array_equal(g["sorted_values"], r["sorted_values"]), \
            "sorted values: " + first_diff(g["sorted_values"], r["sorted_values"])
        assert np.array_equal(g["headers"], r["headers"]), "headers: " + first_diff(g["headers"], r["headers"])
    assert np.array_equal(g["color"], r["color"]), "color: " + first_diff(g["color"], r["color"])
    if g["depth"] is not None:
        assert np.array_equal(g["depth"], r["depth"]), "depth: " + first_diff(g["depth"], r["depth"])


@pytest.mark.parametrize("name", MG.CASES)
def test_golden_cases_bit_exact(gsm, cuda, oracle, name):
    case = MG.scene(name)
    r = oracle_render(oracle, case)
    g = gpu_render(gsm, cuda, case)
    assert_frame_equal(g, r)
    g["renderer"].close()


def test_blend_exp_table_is_correctly_rounded(gsm, cuda):
    r = gsm.GlobalRenderer(config=gsm.RendererConfig(max_gaussians=16, max_width=64, max_height=32))
    tbl = r.copy_buffer(gsm.BufferId.EXP_TABLE)
    gold = np.load(os.path.join(HERE, "golden", "exp_h_table.npy"))
    # entry p = exp_h(fp16(-0.5 * p))
    p = np.arange(65536, dtype=np.uint32).astype(np.uint16).view(np.float16).astype(np.float32)
    arg = (np.float32(-0.5) * p).astype(np.float16).view(np.uint16)
    np.testing.assert_array_equal(tbl, gold[arg])
    r.close()


@pytest.mark.parametrize("seed,count,tiles", [(42, 1024, 10), (123, 50_000, 100)])
def test_radix_sort_kats(gsm, cuda, seed, count, tiles):
    """GlobalUnitTests.testRadixSortCorrectness / testRadixSortLargeScale on the HIP sort."""
    keys = np.load(os.path.join(HERE, "golden", f"radix_kat_seed{seed}.npz"))["keys"]
    assert keys.size == count
    k = cuda.from_numpy(keys.view(np.int32).copy()).cuda()
    v = cuda.arange(count, dtype=cuda.int32, device="cuda")
    gsm.sort_pairs_u32(k, v)
    ks = k.cpu().numpy().view(np.uint32)
    vs = v.cpu().numpy()
    assert np.all(ks[:-1] <= ks[1:])
    np.testing.assert_array_equal(ks, np.sort(keys))
    np.testing.assert_array_equal(vs, np.argsort(keys, kind="stable"))


def test_radix_sort_random_large(gsm, cuda):
    rng = np.random.default_rng(5)
    for n, bits in [(1, 32), (2047, 32), (2049, 16), (3_000_001, 32)]:
        keys = rng.integers(0, 2 ** bits, n, dtype=np.uint64).astype(np.uint32)
        keys[: n // 3] = keys[0]  # heavy duplicates: stability matters
        k = cuda.from_numpy(keys.view(np.int32).copy()).cuda()
        v = cuda.arange(n, dtype=cuda.int32, device="cuda")
        gsm.sort_pairs_u32(k, v, key_bits=bits)
        np.testing.assert_array_equal(k.cpu().numpy().view(np.uint32), np.sort(keys, kind="stable"))
        np.testing.assert_array_equal(v.cpu().numpy(), np.argsort(keys, kind="stable"))


def test_sort_rank_probe_reports_lane_order(gsm, cuda):
    """The create-time probe behind the default sort ranks (include/gsm_debug.h): on MI355X the
    lanes of one same-address ds_add_rtn_u32 are served in lane order (tools/exp/lds_atomic_order.hip);
    if a driver or firmware changed that, the renderers would switch to ballot ranks by themselves
    and this test names the change."""
    assert gsm.sort_rank_probe(0) is True


@pytest.mark.parametrize("variant", ["atomic", "ballot"])
def test_radix_sort_variants(gsm, cuda, variant, monkeypatch):
    """Both stable-rank forms (GSM_SORT_RANK, read at create / per stand-alone sort) give the stable
    order: lane-ordered LDS atomics (default when the probe passes) and ballot matches."""
    monkeypatch.setenv("GSM_SORT_RANK", variant)
    rng = np.random.default_rng(11)
    for n, bits in [(5, 32), (4096, 12), (4097, 32), (1_000_003, 32), (2_500_000, 14)]:
        keys = rng.integers(0, 2 ** bits, n, dtype=np.uint64).astype(np.uint32)
        keys[: n // 4] = keys[-1]
        for _ in range(2):  # a second sort reuses nothing stale from the first
            k = cuda.from_numpy(keys.view(np.int32).copy()).cuda()
            v = cuda.arange(n, dtype=cuda.int32, device="cuda")
            gsm.sort_pairs_u32(k, v, key_bits=bits)
            np.testing.assert_array_equal(k.cpu().numpy().view(np.uint32), np.sort(keys, kind="stable"))
            np.testing.assert_array_equal(v.cpu().numpy(), np.argsort(keys, kind="stable"))


@pytest.mark.parametrize("scan", ["none", "kernel"])
def test_radix_sort_scanless_and_scan_kernel(gsm, cuda, oracle, scan, monkeypatch):
    """Narrow passes with (GSM_SORT_SCAN=kernel) and without (default, r05) the k_radix_scan launch give
    the same stable order: stand-alone sorts of 1..4 digits (even digit counts take the alternating
    super-group row sets, odd ones the scan; repeated sorts find the rows zeroed again), and a 1080p
    frame (two narrow tile passes) rendered bit for bit three times on one renderer."""
    monkeypatch.setenv("GSM_SORT_SCAN", scan)
    rng = np.random.default_rng(17)
    for n, bits in [(3, 32), (4096, 8), (70_000, 16), (1_000_003, 24), (2_500_000, 32), (4_194_304, 32)]:
        keys = rng.integers(0, 2 ** bits, n, dtype=np.uint64).astype(np.uint32)
        keys[: n // 5] = keys[n // 2]
        for _ in range(2):
            k = cuda.from_numpy(keys.view(np.int32).copy()).cuda()
            v = cuda.arange(n, dtype=cuda.int32, device="cuda")
            gsm.sort_pairs_u32(k, v, key_bits=bits)
            np.testing.assert_array_equal(k.cpu().numpy().view(np.uint32), np.sort(keys, kind="stable"))
            np.testing.assert_array_equal(v.cpu().numpy(), np.argsort(keys, kind="stable"))
    case = _synth(200_000, 1920, 1080, 4, 1, 29)
    r = oracle_render(oracle, case)
    g = gpu_render(gsm, cuda, case, keep=False)
    monkeypatch.delenv("GSM_SORT_SCAN")
    assert_frame_equal(g, r)
    for _ in range(2):
        g2 = gpu_render(gsm, cuda, case, renderer=g["renderer"], keep=False)
        assert np.array_equal(g["color"], g2["color"])
        assert np.array_equal(g["depth"], g2["depth"])
    g["renderer"].close()


def _synth(n, w, h, sh, prec, seed, **kw):
    from gsm_amd import scenes
    world, harm, cam = scenes.gen_scene(n, w, h, sh, prec, seed=seed, **kw)
    return dict(world=world, harm=harm, sh=sh, cam=cam, width=w, height=h, max_gaussians=max(n, 1))


@pytest.mark.parametrize("w,h", [(320, 180), (1280, 720)])  # 120 tiles: one narrow pass; 1800: one wide pass
def test_empty_frame_is_clear(gsm, cuda, oracle, w, h):
    case = _synth(64, w, h, 1, 0, 1)
    case["count"] = 0
    g = gpu_render(gsm, cuda, case)
    r = oracle_render(oracle, case)
    assert r["total_assignments"] == 0
    assert_frame_equal(g, r, stages=False)
    col = g["color"].view(np.float16)
    assert np.all(col[..., :3] == 0) and np.all(col[..., 3] == 1)
    assert np.all(g["headers"] == 0)


def test_edge_cases(gsm, cuda, oracle):
    from gsm_amd.types import WORLD32
    w = np.zeros(5, WORLD32)
    w["rot"][:, 3] = 1.0
    # 0: huge gaussian covering the screen; 1: behind the camera; 2: tiny (scale cull);
    # 3: transparent (alpha cull); 4: off-screen
    w[0]["px"], w[0]["py"], w[0]["pz"], w[0]["opacity"] = 0.0, 0.0, 2.0, 0.9
    w[0]["sx"], w[0]["sy"], w[0]["sz"] = 1.5, 0.4, 0.2
    w[0]["rot"] = [0.2, 0.1, 0.3, 0.9]
    w[1]["pz"], w[1]["opacity"], w[1]["sx"], w[1]["sy"], w[1]["sz"] = -2.0, 0.9, 0.1, 0.1, 0.1
    w[2]["pz"], w[2]["opacity"], w[2]["sx"], w[2]["sy"], w[2]["sz"] = 3.0, 0.9, 1e-4, 1e-4, 1e-4
    w[3]["pz"], w[3]["opacity"], w[3]["sx"], w[3]["sy"], w[3]["sz"] = 3.0, 0.001, 0.1, 0.1, 0.1
    w[4]["px"], w[4]["pz"], w[4]["opacity"], w[4]["sx"], w[4]["sy"], w[4]["sz"] = 50.0, 3.0, 0.9, .1, .1, .1
    harm = np.tile(np.array([0.3, -0.2, 0.8], np.float32), 5)
    cam = oracle.make_camera(640, 360)
    case = dict(world=w, harm=harm, sh=1, cam=cam, width=640, height=360, max_gaussians=5)
    r = oracle_render(oracle, case)
    assert list(r["mask"]) == [1, 0, 0, 0, 0]
    g = gpu_render(gsm, cuda, case)
    assert_frame_equal(g, r)


@pytest.mark.parametrize("env", [{}, {"GSM_BLEND_WAVES": "16"}, {"GSM_BLEND_PAIRS": "0"}])
def test_far_gaussians_in_a_full_frame(gsm, cuda, oracle, monkeypatch, env):
    """test_far_gaussian_fp16_depth_overflow's record (fp16 depth inf) among 60k ordinary gaussians of a
    1080p frame: the half-tile walk and its compaction phase (k_blend_px), and at 16 waves the pair walk's
    three layouts (k_blend_pw), all switch to the exact depth test from the batch holding it."""
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    case = _synth(60_000, 1920, 1080, 1, 0, 7)
    far = np.zeros(4, case["world"].dtype)
    far["rot"][:, 3] = 1.0
    for i, (x, y) in enumerate([(0.0, 0.0), (30000.0, 9000.0), (-40000.0, -12000.0), (0.0, 20000.0)]):
        far[i]["px"], far[i]["py"], far[i]["pz"], far[i]["opacity"] = x, y, 80000.0 + 5000.0 * i, 0.8
        far[i]["sx"], far[i]["sy"], far[i]["sz"] = 3000.0, 2200.0, 3000.0
    case["world"] = np.concatenate([case["world"][:30_000], far, case["world"][30_000:]])
    h = case["harm"].reshape(-1, 3)
    case["harm"] = np.concatenate([h[:30_000], np.tile([[0.2, 0.1, -0.3]], (4, 1)).astype(h.dtype), h[30_000:]]).reshape(-1)
    case["max_gaussians"] = len(case["world"])
    r = oracle_render(oracle, case)
    assert all(r["mask"][30_000:30_004] == 1)
    g = gpu_render(gsm, cuda, case, keep=False)
    for k in env:
        monkeypatch.delenv(k)
    assert_frame_equal(g, r)
    g["renderer"].close()


@pytest.mark.parametrize("kind,n,w,h,sh,seed,env", [
    ("f32", 20_000, 640, 360, 16, 5, {}), ("f16", 20_000, 640, 360, 16, 6, {}),
    ("f32", 40_000, 1920, 1080, 1, 7, {}), ("f16", 60_000, 1920, 1080, 9, 8, {}),
    ("f16", 60_000, 1920, 1080, 16, 9, {"GSM_BLEND_WAVES": "16"}),
    ("f32", 30_000, 1280, 720, 4, 10, {"GSM_SORT_SCAN": "kernel"}),
    ("f16", 60_000, 1920, 1080, 9, 11, {"overflow": True}),
])
def test_adversarial_scenes_bit_exact(gsm, cuda, oracle, monkeypatch, kind, n, w, h, sh, seed, env):
    """Ordinary gaussians with a quarter of them given edge values (tests/adversarial.py: zero / extreme /
    inf / NaN scales, positions and quaternions, opacities around the 0.005 cull and outside [0, 1],
    huge / NaN SH coefficients, a few large close splats): every intermediate bit for bit."""
    import adversarial
    env = dict(env)
    overflow = env.pop("overflow", False)  # (max_gaussians = n: the assignments pass the 4 n cap)
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    case = adversarial.scene(kind, n, w, h, sh, seed, overflow)
    r = oracle_render(oracle, case)
    assert r["overflow"] == (1 if overflow else 0)
    g = gpu_render(gsm, cuda, case)
    for k in env:
        monkeypatch.delenv(k)
    assert_frame_equal(g, r)
    g["renderer"].close()


def _random_camera(w, h, seed):
    """make_camera's projection with a random orientation (QR of a normal matrix) at a random point
    within 8 units of the scene's centre (0, 0, 5.5) -- views from inside the cloud, from behind it,
    rolled, looking away."""
    from gsm_amd import scenes
    rng = np.random.default_rng(seed)
    pos = (np.array([0, 0, 5.5]) + rng.normal(size=3) * 3.0).astype(np.float32)
    if seed % 3 == 0:  # any orientation (often looking away from most of the cloud)
        q, r = np.linalg.qr(rng.normal(size=(3, 3)))
        R = q * np.sign(np.diag(r))
        if np.linalg.det(R) < 0:
            R[:, 0] = -R[:, 0]
    else:  # towards a point near the centre, rolled (camera looks along +z of its frame)
        fwd = np.array([0, 0, 5.5]) + rng.normal(size=3) * 1.5 - pos
        fwd /= np.linalg.norm(fwd)
        right = np.cross([0.0, 1.0, 0.0], fwd)
        right /= np.linalg.norm(right)
        up = np.cross(fwd, right)
        a = rng.uniform(-np.pi, np.pi)
        R = np.stack([np.cos(a) * right + np.sin(a) * up, -np.sin(a) * right + np.cos(a) * up, fwd], axis=1)
    R = R.astype(np.float32)
    V = np.eye(4, dtype=np.float32)
    V[:3, :3] = R.T
    V[:3, 3] = -(R.T @ pos)
    cam = scenes.make_camera(w, h)
    cam["view"] = V.T.reshape(-1).astype(np.float32)
    cam["position"] = pos
    return cam


@pytest.mark.parametrize("seed,w,h,maxw,maxh,sh,prec,cs", [
    (1, 1000, 555, 1024, 600, 16, 1, 0), (2, 333, 777, 333, 777, 9, 0, 1), (3, 1921, 1081, 1921, 1081, 4, 1, 1),
    (4, 97, 45, 640, 360, 1, 0, 0), (5, 1280, 720, 1920, 1080, 16, 1, 0), (6, 2000, 300, 2000, 300, 9, 1, 1),
])
def test_random_cameras_ragged_frames(gsm, cuda, oracle, seed, w, h, maxw, maxh, sh, prec, cs):
    """Random camera poses over ragged frame sizes (not multiples of the 32x16 tile, frames smaller than
    the renderer's maximum, 97x45 to 2000x300), every SH degree, both input precisions, sRGB input --
    every intermediate bit for bit."""
    case = _synth(80_000, w, h, sh, prec, 100 + seed, spread=1.5)
    case.update(cam=_random_camera(w, h, seed), max_width=maxw, max_height=maxh, color_space=cs)
    r = oracle_render(oracle, case)
    g = gpu_render(gsm, cuda, case)
    assert_frame_equal(g, r)
    g["renderer"].close()


@pytest.mark.parametrize("w,h", [
    (512, 256),    # 256 tiles: one narrow tile pass
    (544, 256),    # 272 tiles: two passes / one wide pass
    (2048, 512),   # 2048 tiles: the last quadrant-unit frame and the last one-wide-pass field
    (1600, 656),   # 2050 tiles: half-tile units, two narrow tile passes
    (2048, 768),   # 3072 tiles = 6144 half-tile units: the 12-wave blend's first frame
    (2016, 768),   # 3024 tiles: 8 waves
    (4096, 1536),  # 12288 tiles = 24576 units: the 16-wave pair-walk blend's first frame
])
def test_kernel_shape_thresholds(gsm, cuda, oracle, w, h):
    """Frames on both sides of every size rule that changes the kernels (one vs two narrow tile passes,
    the wide pass's 2048 tiles, quadrant vs half-tile blend units at 8 tiles per CU, 8 / 12 / 16 blend
    waves and the pair walk at 2 / 6 units per wave slot on 256 CUs): every intermediate bit for bit."""
    case = _synth(60_000, w, h, 4, 1, 43, spread=1.2)
    r = oracle_render(oracle, case)
    g = gpu_render(gsm, cuda, case, keep=False)
    assert_frame_equal(g, r)
    g["renderer"].close()


@pytest.mark.parametrize("n", [64 * 256, 64 * 256 + 1, 8192 * 256, 8192 * 256 + 1])
def test_fused_scan_threshold(gsm, cuda, oracle, n):
    """Frame sizes of 64 and 65 projection blocks (small fused scans), the last size whose block counts the
    scatter workgroups add up themselves (8192 blocks, kFusedScanMaxBlocks) and the first one that takes
    the k_scan_blocks launch: all bit-exact."""
    case = _synth(n, 320, 180, 1, 1, 41, scale_px=0.6)
    r = oracle_render(oracle, case)
    g = gpu_render(gsm, cuda, case, keep=False)
    assert_frame_equal(g, r)
    g["renderer"].close()


def test_far_gaussian_fp16_depth_overflow(gsm, cuda, oracle):
    """A gaussian whose view depth overflows fp16 (record depth +inf; the Global path has no far-plane
    cull): where its alphas are nonzero the reference's depth becomes inf / NaN (inf * 0), and a 4x2
    group whose alphas are all zero skips the entry (GlobalShaders.metal:1133) and keeps its depth."""
    from gsm_amd.types import WORLD32
    w = np.zeros(3, WORLD32)
    w["rot"][:, 3] = 1.0
    # 0: near, small; 1: at depth 80000 (fp16 inf), wide enough to cover ~60 px; 2: near, large
    w[0]["px"], w[0]["py"], w[0]["pz"], w[0]["opacity"] = 0.1, 0.05, 3.0, 0.6
    w[0]["sx"], w[0]["sy"], w[0]["sz"] = 0.05, 0.04, 0.05
    w[1]["px"], w[1]["py"], w[1]["pz"], w[1]["opacity"] = 0.0, 0.0, 80000.0, 0.9
    w[1]["sx"], w[1]["sy"], w[1]["sz"] = 3000.0, 2500.0, 3000.0
    w[2]["px"], w[2]["py"], w[2]["pz"], w[2]["opacity"] = -0.2, 0.1, 4.0, 0.3
    w[2]["sx"], w[2]["sy"], w[2]["sz"] = 0.5, 0.3, 0.2
    harm = np.tile(np.array([0.3, -0.2, 0.8], np.float32), 3)
    cam = oracle.make_camera(640, 360)
    case = dict(world=w, harm=harm, sh=1, cam=cam, width=640, height=360, max_gaussians=3)
    r = oracle_render(oracle, case)
    assert r["mask"][1] == 1
    g = gpu_render(gsm, cuda, case)
    assert_frame_equal(g, r)


def test_frame_smaller_than_max_and_reuse(gsm, cuda, oracle):
    """width/height < maxWidth/maxHeight (tile grid from the max dims, GlobalRenderer.swift:25-51),
    then a second, different frame on the same renderer (no stale state)."""
    a = _synth(20_000, 600, 300, 16, 1, 11)
    a.update(max_width=640, max_height=360, max_gaussians=30_000)
    ra = oracle_render(oracle, a)
    ga = gpu_render(gsm, cuda, a)
    assert_frame_equal(ga, ra)
    b = _synth(25_000, 640, 360, 9, 1, 12)
    b.update(max_width=640, max_height=360, max_gaussians=30_000)
    rb = oracle_render(oracle, b)
    gb = gpu_render(gsm, cuda, b, renderer=ga["renderer"])
    assert_frame_equal(gb, rb)
    ga["renderer"].close()


def test_null_depth_and_determinism(gsm, cuda, oracle):
    case = _synth(30_000, 640, 360, 16, 1, 21)
    r = oracle_render(oracle, case)
    g1 = gpu_render(gsm, cuda, case, depth=False, keep=False)
    assert_frame_equal(g1, r)
    g2 = gpu_render(gsm, cuda, case, renderer=g1["renderer"], depth=False, keep=False)
    assert np.array_equal(g1["color"], g2["color"])
    g1["renderer"].close()


def test_uncaptured_frame_keeps_only_what_the_blend_reads(gsm, cuda, oracle):
    """A frame rendered without capture (profiling bit 4 / keep_unsorted) writes neither the render
    data nor the sorted arrays (include/gsm_debug.h); their readback fails loudly, the image and the
    header counters still equal the oracle's, and a captured frame on the same renderer brings them back."""
    case = _synth(30_000, 640, 360, 16, 1, 23)
    r = oracle_render(oracle, case)
    g = gpu_render(gsm, cuda, case, keep=False)  # captured: every intermediate
    assert_frame_equal(g, r)
    rend = g["renderer"]
    rend.set_profiling(stage_events=False)
    w, h = case["width"], case["height"]
    color = cuda.empty((h, w, 4), dtype=cuda.float16, device="cuda")
    dep = cuda.empty((h, w), dtype=cuda.float16, device="cuda")
    inp = gsm.GaussianInput(to_dev(cuda, case["world"]), to_dev(cuda, case["harm"]), len(case["world"]), case["sh"])
    rend.render(color, dep, inp, gsm.CameraParams.from_dict(case["cam"]), w, h)
    cuda.cuda.synchronize()
    assert np.array_equal(color.view(cuda.int16).cpu().numpy().view(np.uint16), r["color"])
    assert np.array_equal(dep.view(cuda.int16).cpu().numpy().view(np.uint16), r["depth"])
    assert rend.counters()["total_assignments"] == r["total_assignments"]
    for buf in (gsm.BufferId.RENDER_DATA, gsm.BufferId.SORTED_KEYS, gsm.BufferId.SORTED_VALUES):
        with pytest.raises(gsm.RendererError) as e:
            rend.copy_buffer(buf)
        assert e.value.status == gsm.Status.MISSING_REQUIRED_BUFFER
    g2 = gpu_render(gsm, cuda, case, renderer=rend, keep=False)
    assert_frame_equal(g2, r)
    rend.close()


def test_tile_row_slabs_compose_to_full_frame(gsm, cuda, oracle):
    """Multi-GPU slab partition: rows [b, e) rendered alone equal the full frame there."""
    case = _synth(30_000, 640, 360, 16, 1, 31)
    r = oracle_render(oracle, case)
    tiles_y = r["tiles_y"]
    cfg = gsm.RendererConfig(max_gaussians=30_000, max_width=640, max_height=360, precision=1,
                             gaussian_color_space=0)
    rend = gsm.GlobalRenderer(config=cfg)
    composed = np.zeros_like(r["color"])
    bounds = [0, 7, 15, tiles_y]
    for b, e in zip(bounds[:-1], bounds[1:]):
        rend.set_tile_rows(b, e)
        g = gpu_render(gsm, cuda, case, renderer=rend, color_fill=-7.0, keep=False)
        y0, y1 = b * 16, min(e * 16, 360)
        composed[y0:y1] = g["color"][y0:y1]
        outside = np.concatenate([g["color"][:y0].reshape(-1), g["color"][y1:].reshape(-1)])
        assert np.all(outside.view(np.float16) == -7.0), "slab wrote outside its rows"
    assert np.array_equal(composed, r["color"])
    rend.close()


@pytest.mark.parametrize("world,n,w,h,prec,adv", [(2, 40_000, 640, 360, 1, False), (3, 60_000, 1280, 720, 1, False),
                                                  (8, 50_000, 640, 360, 0, False), (4, 40_000, 1280, 720, 1, True),
                                                  (3, 30_000, 640, 360, 0, True)])
def test_partitioned_frame_matches_single_gpu(gsm, cuda, oracle, world, n, w, h, prec, adv):
    """All-to-all slab partition (include/gsm_multigpu.h) over `world` virtual
    ranks on one GPU: every rank projects its id range once, records are exchanged in
    source-rank order (gsm_amd.exchange.emulate = the order the real all_to_all delivers,
    checked with gloo in test_exchange_distributed), every slab is rendered from its
    records.  The composed frame equals the single-GPU frame and the oracle bit for bit."""
    from gsm_amd import exchange
    if adv:  # tests/adversarial.py's edge values (test_adversarial_scenes_bit_exact) through the partition
        import adversarial
        case = adversarial.scene("f16" if prec else "f32", n, w, h, 16 if prec else 4, 31 + world)
    else:
        case = _synth(n, w, h, 16 if prec else 4, prec, 77)
    mg = case["max_gaussians"]
    r = oracle_render(oracle, case)
    assert r["overflow"] == 0
    full = gpu_render(gsm, cuda, case, keep=False)
    full["renderer"].close()
    assert np.array_equal(full["color"], r["color"])
    tiles_y = r["tiles_y"]
    rows = exchange.slab_rows(tiles_y, h, world)
    cfg = gsm.RendererConfig(max_gaussians=mg, max_width=w, max_height=h, precision=prec, gaussian_color_space=0)
    ranks = [gsm.GlobalRenderer(config=cfg) for _ in range(world)]
    wt, ht = to_dev(cuda, case["world"]), to_dev(cuda, case["harm"])
    inp = gsm.GaussianInput(wt, ht, n, case["sh"])
    cam = gsm.CameraParams.from_dict(case["cam"])
    sends, counts = [], []
    for rk in range(world):
        first, cnt = exchange.id_range(n, world, rk)
        cap = max(cnt, 1) * world
        send = cuda.zeros(cap * exchange.RECORD_BYTES, dtype=cuda.uint8, device="cuda")
        sc = cuda.zeros(world, dtype=cuda.int32, device="cuda")
        ranks[rk].project_partition(inp, cam, w, h, first, cnt, rows, send, cap, sc)
        cuda.cuda.synchronize()
        counts.append([int(x) for x in sc.tolist()])
        sends.append(send)
    recv = exchange.emulate(sends, counts)
    color = cuda.full((h, w, 4), float("nan"), dtype=cuda.float16, device="cuda")
    depth = cuda.full((h, w), float("nan"), dtype=cuda.float16, device="cuda")
    for d in range(world):
        if rows[d] == rows[d + 1]:
            continue
        ranks[d].set_tile_rows(rows[d], rows[d + 1])
        nrec = recv[d].numel() // exchange.RECORD_BYTES
        buf = recv[d] if nrec else cuda.zeros(16, dtype=cuda.uint8, device="cuda")
        ranks[d].render_records(color, depth, buf, nrec, w, h)
    cuda.cuda.synchronize()
    got = color.view(cuda.int16).cpu().numpy().view(np.uint16)
    gd = depth.view(cuda.int16).cpu().numpy().view(np.uint16)
    assert np.array_equal(got, r["color"]), "color: " + first_diff(got, r["color"])
    assert np.array_equal(gd, r["depth"]), "depth: " + first_diff(gd, r["depth"])
    # a gaussian with tiles in the frame travels to 1..world slabs, one with none stays home
    with_tiles = int(np.count_nonzero(r["tile_counts"]))
    assert with_tiles <= sum(map(sum, counts)) <= with_tiles * world
    for rend in ranks:
        rend.close()


def test_crowded_tiles_take_the_long_run_sort(gsm, cuda, oracle):
    """Tiles whose list exceeds the per-tile LDS sort (2048 entries per wave) go through the
    wave's two global LSD passes; the frame must still match the oracle bit for bit."""
    case = _synth(40_000, 320, 180, 4, 1, 5, spread=0.002, scale_px=0.8)
    r = oracle_render(oracle, case)
    hdr = r["headers"].reshape(-1, 2)
    assert hdr[:, 1].max() > 8192, "scene must crowd a tile past the LDS capacity"
    g = gpu_render(gsm, cuda, case)
    assert_frame_equal(g, r)
    g["renderer"].close()


def test_stereo_side_by_side_halves_equal_mono_frames(gsm, cuda, oracle):
    """Config 5 shape (SH2, two eyes side by side, +-32 mm): each half of the
    gsm_global_render_stereo_sbs target equals the oracle frame of that eye, bit for bit."""
    from gsm_amd import scenes
    n, w, h = 30_000, 360, 400
    world, harm, _ = scenes.gen_scene(n, w, h, 9, 1, seed=11)
    cams = [scenes.make_camera(w, h, -0.032), scenes.make_camera(w, h, 0.032)]
    refs = [oracle_render(oracle, dict(world=world, harm=harm, sh=9, cam=c, width=w, height=h,
                                      max_gaussians=n)) for c in cams]
    rend = gsm.GlobalRenderer(config=gsm.RendererConfig(max_gaussians=n, max_width=w, max_height=h, precision=1,
                                                        gaussian_color_space=0))
    color = cuda.full((h, 2 * w, 4), float("nan"), dtype=cuda.float16, device="cuda")
    depth = cuda.full((h, 2 * w), float("nan"), dtype=cuda.float16, device="cuda")
    inp = gsm.GaussianInput(to_dev(cuda, world), to_dev(cuda, harm), n, 9)
    rend.render_stereo_sbs(color, depth, inp, gsm.CameraParams.from_dict(cams[0]),
                           gsm.CameraParams.from_dict(cams[1]), w, h)
    cuda.cuda.synchronize()
    c = color.view(cuda.int16).cpu().numpy().view(np.uint16)
    d = depth.view(cuda.int16).cpu().numpy().view(np.uint16)
    for eye, r in enumerate(refs):
        assert np.array_equal(c[:, eye * w:(eye + 1) * w], r["color"]), f"eye {eye}"
        assert np.array_equal(d[:, eye * w:(eye + 1) * w], r["depth"]), f"eye {eye} depth"
    assert not np.array_equal(refs[0]["color"], refs[1]["color"])  # the eyes do differ
    rend.close()


def test_stereo_is_unsupported_like_the_reference(gsm, cuda):
    rend = gsm.GlobalRenderer(config=gsm.RendererConfig(max_gaussians=16, max_width=64, max_height=32))
    x = cuda.zeros(16, dtype=cuda.uint8, device="cuda")
    cam = gsm.CameraParams(np.eye(4, dtype=np.float32).reshape(-1), np.eye(4, dtype=np.float32).reshape(-1))
    with pytest.raises(gsm.RendererError) as e:
        rend.render_stereo(x, None, gsm.GaussianInput(x, x, 0, 0), cam, cam, 32, 32)
    assert e.value.status == gsm.Status.UNSUPPORTED
    with pytest.raises(gsm.RendererError) as e:
        rend.render(x, None, gsm.GaussianInput(x, x, 17, 0), cam, 32, 32)
    assert e.value.status == gsm.Status.INVALID_GAUSSIAN_COUNT
    with pytest.raises(gsm.RendererError) as e:
        rend.render(x, None, gsm.GaussianInput(x, x, 1, 0), cam, 65, 32)
    assert e.value.status == gsm.Status.INVALID_DIMENSIONS
    rend.close()


@pytest.mark.parametrize("env", [{"GSM_SORT_RANK": "ballot"}, {"GSM_BLEND_SCHED": "0"},
                                 {"GSM_SORT": "radix4"}, {"GSM_BLEND_CLAIM": "early"},
                                 {"GSM_BLEND_CLAIM": "auto"}, {"GSM_SORT_WIDE": "0"},
                                 {"GSM_SORT_WIDE": "0", "GSM_SORT_RANK": "ballot"}])
def test_create_time_switches_frames_match(gsm, cuda, oracle, monkeypatch, env):
    """The A/B switches read once at create (Tuning, gsm_internal.h) -- ballot sort ranks, index-order
    blend schedule, the 4 x 8-bit full-key sort, the blend queue's claim point, narrow tile passes
    instead of the one wide pass of this frame's 1800 tiles -- render the same
    frames bit for bit, first and later frames (later ones take last frame's cost order when the
    schedule is on)."""
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    case = _synth(200_000, 1280, 720, 16, 1, 33)
    r = oracle_render(oracle, case)
    g = gpu_render(gsm, cuda, case, keep=False)
    for k in env:  # read at create: the live renderer keeps its setting
        monkeypatch.delenv(k)
    assert_frame_equal(g, r)
    for _ in range(3):
        g2 = gpu_render(gsm, cuda, case, renderer=g["renderer"], keep=False)
        assert np.array_equal(g["color"], g2["color"])
        assert np.array_equal(g["depth"], g2["depth"])
    g["renderer"].close()


@pytest.mark.parametrize("fused", ["1", "0"])
def test_scan_modes_frame_sequence(gsm, cuda, oracle, monkeypatch, fused):
    """The block-count scan (GSM_SCAN_FUSED, read at create): the scatter adding up every earlier block
    count (default up to 8192 blocks) or the k_scan_blocks launch.  One renderer renders a sequence of
    different frames -- several sizes, an empty frame in between (no projection blocks: the scan kernel
    writes its header) -- each bit for bit against the oracle."""
    monkeypatch.setenv("GSM_SCAN_FUSED", fused)
    cases = [_synth(200_000, 1280, 720, 16, 1, 51), _synth(40_000, 1280, 720, 4, 1, 52),
             _synth(200_000, 1280, 720, 16, 1, 53), _synth(9_000, 1280, 720, 9, 1, 54)]
    for c in cases:
        c["max_gaussians"] = 300_000
    empty = dict(cases[1])
    empty["count"] = 0
    seq = [cases[0], cases[1], empty, cases[2], cases[3], empty, cases[0]]
    renderer = None
    for c in seq:
        r = oracle_render(oracle, c)
        g = gpu_render(gsm, cuda, c, renderer=renderer, keep=False)
        renderer = g["renderer"]
        monkeypatch.delenv("GSM_SCAN_FUSED", raising=False)
        assert_frame_equal(g, r)
    renderer.close()


@pytest.mark.parametrize("env", [{"GSM_BLEND_WAVES": "16"}, {"GSM_BLEND_WAVES": "16", "GSM_BLEND_PAIR_SPLIT": "1"},
                                 {"GSM_BLEND_WAVES": "16", "GSM_BLEND_PAIR_SPLIT": "256"},
                                 {"GSM_BLEND_WAVES": "16", "GSM_BLEND_PAIR_SPLIT": "200"},
                                 {"GSM_BLEND_WAVES": "16", "GSM_BLEND_SCHED": "0"},
                                 {"GSM_BLEND_WAVES": "16", "GSM_BLEND_PAIRS": "0"}])
def test_pair_walk_blend_frames_match(gsm, cuda, oracle, monkeypatch, env):
    """The pair-walk blend (k_blend_pw, r05): a 1080p frame of half-tile units at 16 waves per workgroup
    -- two units per wave in the 8- / 4- / 2-pixels-per-lane layouts, single units beside them (the
    schedule's split: 1 = almost all units paired, 256 = none, 200 = most alone), with and without the
    schedule, and one unit per wave (GSM_BLEND_PAIRS=0) -- renders the oracle's frame bit for bit, first
    and later frames (later ones are paired by last frame's walks)."""
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    case = _synth(300_000, 1920, 1080, 4, 1, 35)
    r = oracle_render(oracle, case)
    g = gpu_render(gsm, cuda, case, keep=False)
    for k in env:
        monkeypatch.delenv(k)
    assert_frame_equal(g, r)
    for _ in range(3):
        g2 = gpu_render(gsm, cuda, case, renderer=g["renderer"], keep=False)
        assert np.array_equal(g["color"], g2["color"])
        assert np.array_equal(g["depth"], g2["depth"])
    g["renderer"].close()


@pytest.mark.parametrize("cfg_name,precision", [
    ("cfg2_1m_sh3_1080p_f16", None),
    # the same 1M / SH3 / 1080p frame from PackedWorldGaussian (48 B) + fp32 SH
    # (globalProjectCullKernel, GlobalShaders.metal:127-131)
    ("cfg2_1m_sh3_1080p_f16", 0),
    # BASELINE configs[2]: 5M, SH3, 3840x2160 -- ~13M assignments, 2 x 7-bit tile passes, near the
    # reference's 16.78M radix cap (GlobalShaders.metal:866-911), which this sort does not have
    ("cfg3_5m_sh3_4k_f16", None),
])
def test_full_size_config_bit_exact(gsm, cuda, oracle, cfg_name, precision):
    """BASELINE configs[1] and [2] end to end against the oracle, every intermediate bit for bit."""
    from gsm_amd import scenes
    c = scenes.CONFIGS[cfg_name]
    prec = c["precision"] if precision is None else precision
    case = _synth(c["count"], c["width"], c["height"], c["sh"], prec, 42)
    r = oracle_render(oracle, case)
    g = gpu_render(gsm, cuda, case, keep=False)
    assert r["overflow"] == 0
    if cfg_name.startswith("cfg3"):
        assert 10_000_000 < r["total_assignments"] < 16_777_216
    assert_frame_equal(g, r)
    g["renderer"].close()


@pytest.mark.parametrize("rank", ["atomic", "ballot"])
def test_1080p_tile_field_two_narrow_passes(gsm, cuda, oracle, monkeypatch, rank):
    """A 1080p frame's 4080 tiles (a 12-bit tile field): two narrow 6-bit passes writing the tile starts
    (lane-ordered atomic or ballot ranks; the one-pass 12-bit variant measured slower and lives in
    tools/exp/rejected_variants.patch) -- the same frame as the oracle's, every intermediate bit for bit,
    first and second frame."""
    monkeypatch.setenv("GSM_SORT_RANK", rank)
    case = _synth(200_000, 1920, 1080, 4, 1, 61)
    r = oracle_render(oracle, case)
    g = gpu_render(gsm, cuda, case)
    monkeypatch.delenv("GSM_SORT_RANK")
    assert r["tiles_y"] * ((1920 + 31) // 32) == 4080
    assert_frame_equal(g, r)
    g2 = gpu_render(gsm, cuda, case, renderer=g["renderer"])
    assert_frame_equal(g2, r)
    g["renderer"].close()


@pytest.mark.parametrize("fmt,pairs", [(1, False), (2, False), (3, False), (4, False), (5, False),
                                      (1, True), (3, True), (5, True)])
def test_color_formats(gsm, cuda, oracle, monkeypatch, fmt, pairs):
    """The colour target in every gsm_color_format equals the oracle's rgba16f frame converted by
    the declared rules (include/gsm_renderer.h; oracle.convert_color); depth stays r16f.  pairs: the
    pair-walk blend's own pixel writes (k_blend_pw: a 1080p frame of half-tile units at 16 waves per
    workgroup)."""
    if pairs:
        monkeypatch.setenv("GSM_BLEND_WAVES", "16")
    case = _synth(60000, 1920, 1080, 4, 1, 21) if pairs else _synth(20000, 320, 180, 9, 1, 21)
    w, h = case["width"], case["height"]
    ref = oracle_render(oracle, case)
    want = oracle.convert_color(ref["color"], fmt)
    r = gsm.GlobalRenderer(config=gsm.RendererConfig(max_gaussians=case["max_gaussians"], max_width=w,
                                                      max_height=h, precision=1, color_format=fmt,
                                                      gaussian_color_space=0))
    dt = cuda.float32 if fmt == 1 else cuda.uint8
    color = cuda.full((h, w, 4), 7, dtype=dt, device="cuda")
    dep = cuda.full((h, w), float("nan"), dtype=cuda.float16, device="cuda")
    inp = gsm.GaussianInput(to_dev(cuda, case["world"]), to_dev(cuda, case["harm"]), len(case["world"]), case["sh"])
    r.render(color, dep, inp, gsm.CameraParams.from_dict(case["cam"]), w, h)
    cuda.cuda.synchronize()
    got = color.cpu().numpy()
    if fmt == 1:
        np.testing.assert_array_equal(got.view(np.uint32), want.view(np.uint32))
    else:
        np.testing.assert_array_equal(got, want)
    np.testing.assert_array_equal(dep.view(cuda.int16).cpu().numpy().view(np.uint16), ref["depth"])
    # an unaligned pitch is rejected, not written
    with pytest.raises(gsm.RendererError):
        r.render(color, dep, inp, gsm.CameraParams.from_dict(case["cam"]), w, h,
                 color_pitch=w * gsm.ColorFormat(fmt).bytes_per_pixel + 2)
    r.close()


def test_assignment_total_past_2_32_clamps_with_overflow(gsm, cuda):
    """A frame whose assignment total passes 2^32 by less than its capacity (265 126 screen-covering
    gaussians x 16 200 tiles of 3840x2160 = 2^32 + 73 904): a 32-bit scan of the block sums would wrap
    the total to 73 904 < 4N and sort a garbage frame without the overflow flag.  The exact scan
    (k_scan_blocks) clamps it to 4N with overflow = 1, as the reference's clamp does
    (GlobalShaders.metal:696-701).  No oracle: 4.3G tile tests are out of reach on the CPU."""
    from gsm_amd.types import WORLD32
    n, w, h = 265_126, 3840, 2160
    assert n * 120 * 135 - 2 ** 32 == 73_904
    world = np.zeros(n, WORLD32)
    world["pz"], world["opacity"] = 5.0, 0.99
    world["sx"] = world["sy"] = world["sz"] = 50.0  # sigma clamped to 2 * 3840 / 3 px: every tile
    world["rot"][:, 3] = 1.0
    harm = np.tile(np.array([0.3, 0.2, 0.1], np.float32), n)
    from gsm_amd import scenes
    cam = scenes.make_camera(w, h)
    rend = gsm.GlobalRenderer(config=gsm.RendererConfig(max_gaussians=n, max_width=w, max_height=h, precision=0,
                                                        gaussian_color_space=0))
    color = cuda.empty((h, w, 4), dtype=cuda.float16, device="cuda")
    rend.render(color, None, gsm.GaussianInput(to_dev(cuda, world), to_dev(cuda, harm), n, 1),
                gsm.CameraParams.from_dict(cam), w, h)
    cuda.cuda.synchronize()
    c = rend.counters()
    assert c["overflow"] == 1
    assert c["total_assignments"] == 4 * n
    rend.close()
