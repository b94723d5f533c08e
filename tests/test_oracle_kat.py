"""The oracle against the reference's own known-answer tests and the numeric contract.

Reference KATs: Tests/RendererTests/GlobalUnitTests.swift:23-105 (seed 42, 1024 keys,
10 tiles: GPU-sorted keys == CPU-sorted keys) and :107-178 (seed 123, 50000 keys, 100
tiles: non-decreasing).  The keys are regenerated from glibc drand48 exactly as the
Swift test builds them; SURVEY.md section 4 lists the expected first keys and extremes.
"""
import json
import os

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = os.path.join(HERE, "golden")


def kat_keys(oracle, seed, count, tiles):
    L = oracle.lib()
    L.og_srand48(seed)
    keys = np.zeros(count, np.uint32)
    for i in range(count):
        tile = int(L.og_drand48() * tiles)
        depth = np.float32(L.og_drand48() * 100.0)  # Float(drand48() * 100.0)
        keys[i] = L.og_sort_key(tile, L.og_f2h(float(depth)))  # Float16(depth).bits ^ 0x8000
    return keys


def test_radix_kat_seed42_matches_reference_values(oracle):
    keys = kat_keys(oracle, 42, 1024, 10)
    assert [hex(k) for k in keys[:8]] == ["0x7d049", "0x1d147", "0xd55a", "0x4d1fc", "0x6d537",
                                          "0x4d338", "0x5c12e", "0x7d384"]
    np.testing.assert_array_equal(keys, np.load(os.path.join(GOLD, "radix_kat_seed42.npz"))["keys"])
    vals = np.arange(1024, dtype=np.int32)
    sk, sv = oracle.radix_sort_pairs(keys, vals)
    # GlobalUnitTests.swift:96-104: non-decreasing and equal to the CPU sort
    assert np.all(sk[:-1] <= sk[1:])
    np.testing.assert_array_equal(sk, np.sort(keys))
    assert hex(sk[0]) == "0xbd07" and hex(sk[-1]) == "0x9d62f"
    # stability (payload order) -- stronger than the reference test, which skips it
    np.testing.assert_array_equal(sv, np.argsort(keys, kind="stable"))


def test_radix_kat_seed123_large(oracle):
    keys = kat_keys(oracle, 123, 50_000, 100)
    np.testing.assert_array_equal(keys, np.load(os.path.join(GOLD, "radix_kat_seed123.npz"))["keys"])
    assert len(np.unique(keys)) == 45_859  # duplicates make stability matter
    sk, sv = oracle.radix_sort_pairs(keys, np.arange(keys.size, dtype=np.int32))
    assert np.all(sk[:-1] <= sk[1:])
    np.testing.assert_array_equal(sv, np.argsort(keys, kind="stable"))


def test_f2h_matches_ieee_rne(oracle):
    L = oracle.lib()
    rng = np.random.default_rng(0)
    xs = np.concatenate([
        rng.normal(0, 1, 3000), rng.normal(0, 1e-5, 2000), rng.normal(0, 3e4, 2000),
        np.array([0.0, -0.0, 65504.0, 65519.99, 65520.0, 1e-8, 2.98e-8, 5.97e-8, 6.1e-5, -6.1e-5,
                  np.inf, -np.inf]),
    ]).astype(np.float32)
    got = np.array([L.og_f2h(float(x)) for x in xs], np.uint16)
    want = xs.astype(np.float16).view(np.uint16)
    np.testing.assert_array_equal(got, want)
    assert all(L.og_h2f(int(b)) == np.uint16(b).view(np.float16).astype(np.float32)
               for b in range(0, 0x7C00, 97))


def test_exp_table_is_correctly_rounded(oracle):
    """The contract's fp16 exp equals the decimal-exact nearest-even e^x for all 65536 x."""
    gold = np.load(os.path.join(GOLD, "exp_h_table.npy"))
    L = oracle.lib()
    got = np.array([L.og_exp_h(i) for i in range(65536)], np.uint16)
    np.testing.assert_array_equal(got, gold)


def test_deterministic_math_accuracy(oracle):
    L = oracle.lib()
    rng = np.random.default_rng(1)
    y = rng.normal(size=2000).astype(np.float32)
    x = rng.normal(size=2000).astype(np.float32)
    got = np.array([L.og_atan2f(float(a), float(b)) for a, b in zip(y, x)])
    np.testing.assert_allclose(got, np.arctan2(y.astype(np.float64), x), atol=4e-7)
    v = rng.uniform(1e-3, 10.0, 2000).astype(np.float32)
    np.testing.assert_allclose([L.og_log2f(float(a)) for a in v], np.log2(v.astype(np.float64)),
                               atol=4e-7, rtol=2e-7)
    e = rng.uniform(-20, 20, 2000).astype(np.float32)
    np.testing.assert_allclose([L.og_exp2f(float(a)) for a in e], np.exp2(e.astype(np.float64)),
                               rtol=4e-7)


@pytest.fixture(scope="module")
def golden_digests():
    with open(os.path.join(GOLD, "oracle_digests.json")) as f:
        return json.load(f)


@pytest.mark.parametrize("name", ["ref_grid_4096_640x360_sh0_f32", "synth_20k_640x360_sh3_f16",
                                  "synth_20k_640x360_sh2_f16_srgb", "synth_20k_640x360_sh1_f32",
                                  "ref_visible_50k_640x360_sh0_f32"])
def test_oracle_frame_matches_golden_digests(oracle, golden_digests, name):
    from golden import make_golden as MG
    r = MG.render(name)
    assert r["status"] == 0
    assert MG.frame_digests(r) == golden_digests[name]


def test_oracle_frame_invariants(oracle):
    """Structural properties of the reference's pipeline (SURVEY.md 8a determinism contract)."""
    from golden import make_golden as MG
    r = MG.render("synth_20k_640x360_sh3_f16")
    tot = r["total_assignments"]
    # sort == stable sort by (tile, fp16 depth) with ties in gid order
    order = np.lexsort((r["values"], r["keys"]))
    np.testing.assert_array_equal(r["sorted_keys"], r["keys"][order])
    np.testing.assert_array_equal(r["sorted_values"], r["values"][order])
    # headers: offset = lower bound, count = run length; empty tiles too
    tiles = r["sorted_keys"] >> 16
    hdr = r["headers"]
    exp_off = np.searchsorted(tiles, np.arange(r["tile_count"]), side="left")
    exp_end = np.searchsorted(tiles, np.arange(r["tile_count"]), side="right")
    np.testing.assert_array_equal(hdr[:, 0], exp_off)
    np.testing.assert_array_equal(hdr[:, 1], exp_end - exp_off)
    assert hdr[:, 1].sum() == tot
    # each gaussian appears tile_counts times
    np.testing.assert_array_equal(np.bincount(r["values"], minlength=r["count"]), r["tile_counts"])
    # inactive tiles keep the clear colour (0,0,0,1)
    col = r["color"].view(np.float16)
    tx, ty = r["tiles_x"], r["tiles_y"]
    for t in np.nonzero(hdr[:, 1] == 0)[0][:20]:
        y0, x0 = (t // tx) * 16, (t % tx) * 32
        blk = col[y0:y0 + 16, x0:x0 + 32]
        if blk.size:
            assert np.all(blk[..., :3] == 0) and np.all(blk[..., 3] == 1)
