"""The N > 1 product path of include/gsm_multigpu.h with real processes, on one MI355X.

Two to four rank processes share GPU 0 (tests/mg_worker.py): each owns a fine-grained exchange
allocation, the handles go over torch.distributed (gloo) and every rank opens its peers' allocations
with hipIpcOpenMemHandle -- the set-up the 8-GPU node runs, where the mappings cross xGMI.  Per frame
every record is stored by k_part_copy straight into another process's receive buffer, the count
matrix rows and the barrier flags cross the processes, the slab blends write their pixels into rank
0's gathered frame, and rank 0's stream waits for every slab.  The frames must equal the oracle's bit
for bit, with no barrier timeout.  (RCCL cannot run two ranks on one GPU -- "Duplicate GPU detected",
DESIGN.md 7 -- which is one reason the frame uses no collective library.)

The same kernels run for W virtual ranks in one process (phases issued rank by rank on one stream,
include/gsm_multigpu.h gsm_multigpu_render_phase) up to config 4, 5M / SH3 / 4K over 8 ranks."""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _run_ranks(tmp_path, world, extra=(), timeout=150):
    port = _free_port()
    env = dict(os.environ)
    procs = [subprocess.Popen([sys.executable, "-u", os.path.join(ROOT, "tests", "mg_worker.py"), "--rank", str(r),
                               "--world", str(world), "--port", str(port), "--out", str(tmp_path), *extra],
                              stdout=subprocess.PIPE, stderr=subprocess.STDOUT, env=env) for r in range(world)]
    outs = []
    try:
        for p in procs:
            out, _ = p.communicate(timeout=timeout)
            outs.append(out.decode(errors="replace"))
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    for r, (p, o) in enumerate(zip(procs, outs)):
        assert p.returncode == 0, f"rank {r} exited {p.returncode}:\n{o[-3000:]}"
    return [json.load(open(os.path.join(tmp_path, f"status_{r}.json"))) for r in range(world)]


@pytest.mark.parametrize("world,n,w,h,sh,prec,rows", [(2, 40_000, 640, 360, 16, 1, "contiguous"),
                                                      (3, 30_000, 1280, 720, 4, 0, "interleaved"),
                                                      (4, 30_000, 640, 360, 9, 1, "contiguous")])
def test_processes_on_one_gpu_render_the_oracle_frame(oracle, tmp_path, monkeypatch, world, n, w, h, sh, prec, rows):
    from gsm_amd import scenes
    monkeypatch.setenv("GSM_MG_ROWS", rows)  # (the rank processes inherit it)
    st = _run_ranks(tmp_path, world, ["--n", str(n), "--width", str(w), "--height", str(h), "--sh", str(sh),
                                      "--precision", str(prec)])
    assert all(s["timeouts"] == 0 for s in st)
    world_np, harm_np, cam_d = scenes.gen_scene(n, w, h, sh, prec, seed=11)
    ref = oracle.render(world_np, harm_np, sh, cam_d, w, h, max_gaussians=n)
    # A: gathered into the library frames (colour and depth) across the processes
    assert np.array_equal(np.load(tmp_path / "frame_a.npy"), ref["color"])
    assert np.array_equal(np.load(tmp_path / "depth_a.npy"), ref["depth"])
    # B: next camera, the library's copies into the caller's tensors
    ref_b = oracle.render(world_np, harm_np, sh, scenes.orbit_camera(w, h, 3.0), w, h, max_gaussians=n)
    assert np.array_equal(np.load(tmp_path / "frame_b.npy"), ref_b["color"])
    assert np.array_equal(np.load(tmp_path / "depth_b.npy"), ref_b["depth"])
    # D / E: rank 1 alone refused frame D (INVALID_DIMENSIONS) but kept every barrier step; the others
    # finished it without timing out and counted its failed arrivals; frame E is bit-exact again
    assert st[1]["d_status"] == 7 and all(s["d_status"] == 0 for r, s in enumerate(st) if r != 1)
    assert all(s["timeouts_de"] == 0 for s in st)
    assert st[0]["failed_peer_arrivals"] >= 1
    assert np.array_equal(np.load(tmp_path / "frame_e.npy"), ref["color"])
    assert np.array_equal(np.load(tmp_path / "depth_e.npy"), ref["depth"])
    # C: each rank's tile rows (a contiguous block, or r, r + W, ... interleaved) in its own targets
    from gsm_amd import exchange
    tiles_y = (h + 15) // 16
    for r in range(world):
        own = np.zeros(h, bool)
        for t in exchange.rank_tile_rows(tiles_y, world, r, interleave=rows == "interleaved"):
            own[16 * t:min(16 * t + 16, h)] = True
        col = np.load(tmp_path / f"band_c_color_{r}.npy")
        dep = np.load(tmp_path / f"band_c_depth_{r}.npy")
        assert np.array_equal(col[own], ref["color"][own])
        assert np.array_equal(dep[own], ref["depth"][own])
        assert np.all((col[~own].reshape(-1) & 0x7C00) == 0x7C00)  # rows of other ranks untouched (NaN)
    # every rank holds the same count matrix; its column sums are the slabs' receive counts
    cm = np.array(st[0]["counts"], np.int64)
    assert all(np.array_equal(np.array(s["counts"]), cm) for s in st)
    with_tiles = int(np.count_nonzero(ref["tile_counts"]))
    assert with_tiles <= cm.sum() <= with_tiles * world


@pytest.mark.parametrize("world,rows", [(2, "contiguous"), (3, "interleaved")])
def test_processes_pipelined(oracle, tmp_path, monkeypatch, world, rows):
    """GSM_MG_PIPELINE=1 across rank processes (IPC-mapped exchange memory): four frames over three
    views issued back to back, each rank's projection and push of frame f + 1 on its own stream beside
    its slab render of frame f -- every gathered frame (colour and depth) bit-exact with the oracle;
    then a frame that rank 1 alone refuses and the next one, back to back: the ranks stay in step and
    the next frame is bit-exact (pipelined)."""
    from gsm_amd import scenes
    monkeypatch.setenv("GSM_MG_ROWS", rows)
    n, w, h, sh, prec = 40_000, 640, 360, 16, 1
    st = _run_ranks(tmp_path, world, ["--n", str(n), "--pipelined", "1"])
    assert all(s["timeouts"] == 0 for s in st)
    world_np, harm_np, cam_d = scenes.gen_scene(n, w, h, sh, prec, seed=11)
    cams = [cam_d, scenes.orbit_camera(w, h, 3.0), scenes.orbit_camera(w, h, 6.0), cam_d]
    for i, cam in enumerate(cams):
        ref = oracle.render(world_np, harm_np, sh, cam, w, h, max_gaussians=n)
        assert np.array_equal(np.load(os.path.join(tmp_path, f"frame_p{i}.npy")), ref["color"]), f"frame {i}"
        assert np.array_equal(np.load(os.path.join(tmp_path, f"depth_p{i}.npy")), ref["depth"]), f"depth {i}"
    # then D (rank 1 alone refuses) and E (the first view), pipelined back to back: E bit-exact
    assert st[1]["pd0_status"] == 7 and all(s["pd0_status"] == 0 for k, s in enumerate(st) if k != 1)
    assert all(s["pd1_status"] == 0 and s["timeouts_de"] == 0 for s in st)
    assert st[0]["failed_peer_arrivals"] >= 1
    ref = oracle.render(world_np, harm_np, sh, cams[0], w, h, max_gaussians=n)
    assert np.array_equal(np.load(os.path.join(tmp_path, "frame_pe.npy")), ref["color"])
    assert np.array_equal(np.load(os.path.join(tmp_path, "depth_pe.npy")), ref["depth"])


def test_processes_refuse_a_frame_over_the_smallest_capacity(tmp_path):
    """A rank sized for less than the frame: every rank returns INVALID_GAUSSIAN_COUNT before it
    enqueues any work of the frame (its barrier steps still run, marked failed: no rank waits for a
    peer that stopped, no peer's receive buffer is overrun)."""
    st = _run_ranks(tmp_path, 2, ["--n", "20000", "--cap", "15000"])
    assert all(s["refused"] for s in st)


def _virtual_frame(gsm, cuda, world, n, w, h, sh, prec, seed, cams, options=None):
    from gsm_amd import scenes
    world_np, harm_np, cam_d = scenes.gen_scene(n, w, h, sh, prec, seed=seed)
    wt = cuda.from_numpy(world_np.view(np.uint8).reshape(-1).copy()).cuda()
    ht = cuda.from_numpy(harm_np.view(np.uint8).reshape(-1).copy()).cuda()
    del world_np, harm_np
    inp = gsm.GaussianInput(wt, ht, n, sh)
    cfg = gsm.RendererConfig(max_gaussians=n, max_width=w, max_height=h, precision=prec, gaussian_color_space=0)
    rends = [gsm.GlobalRenderer(device=0, config=cfg) for _ in range(world)]
    pre = [gsm.MultiGpuRenderer.prepare(r, k, world, options) for k, r in enumerate(rends)]
    handles = [hd for _, hd in pre]
    mgs = [m.connect_handles(handles) for m, _ in pre]
    frame_ptr, _ = mgs[0].frame()
    stream = cuda.cuda.current_stream()
    frames, depths = [], []
    for cam in cams:
        cp = gsm.CameraParams.from_dict(cam)
        for ph in range(4):  # phase p of every rank before phase p + 1 of any (one stream)
            for k, m in enumerate(mgs):
                m.render_phases([ph], None, None, inp, cp, w, h, gather=True, stream=stream,
                                gather_target=frame_ptr if k == 0 else None, gather_depth=True)
        cuda.cuda.synchronize()
        frames.append(mgs[0].copy_frame(w, h))
        depths.append(mgs[0].copy_depth(w, h))
    counts = mgs[0].counts()
    timeouts = [m.status() for m in mgs]
    for m in mgs:
        m.close()
    for r in rends:
        r.close()
    return frames, counts, timeouts, depths


@pytest.mark.parametrize("world,n,w,h,prec,rows", [(2, 40_000, 640, 360, 1, "contiguous"),
                                                   (3, 60_000, 1280, 720, 1, "contiguous"),
                                                   (8, 50_000, 640, 360, 0, "contiguous"),
                                                   (16, 30_000, 640, 360, 1, "contiguous"),
                                                   (3, 60_000, 1280, 720, 1, "interleaved"),
                                                   (8, 50_000, 640, 360, 0, "interleaved"),
                                                   (16, 30_000, 640, 360, 1, "interleaved")])
def test_virtual_ranks_product_path(gsm, cuda, oracle, world, n, w, h, prec, rows):
    """W ranks of one process through the product kernels (barriers, pushes, gather into rank 0's
    frame), two cameras: the second frame reuses the parity-double-buffered count matrix.  Rows in
    contiguous blocks (the default) or interleaved over the ranks, chosen through the C ABI's
    gsm_multigpu_options (r06; the environment's GSM_MG_ROWS is only a test override)."""
    from gsm_amd import scenes
    sh = 16 if prec else 4
    cams = [scenes.make_camera(w, h), scenes.orbit_camera(w, h, 5.0)]
    opts = gsm.MultiGpuOptions(rows=rows, timeout_ms=20000)
    frames, counts, timeouts, depths = _virtual_frame(gsm, cuda, world, n, w, h, sh, prec, 78, cams, opts)
    assert timeouts == [0] * world
    world_np, harm_np, _ = scenes.gen_scene(n, w, h, sh, prec, seed=78)
    for i, (got, gd, cam) in enumerate(zip(frames, depths, cams)):
        ref = oracle.render(world_np, harm_np, sh, cam, w, h, max_gaussians=n)
        bad = np.nonzero(np.any(got != ref["color"], axis=(1, 2)))[0]
        assert len(bad) == 0, f"frame {i}: {len(bad)} rows differ, first {bad[:16].tolist()}"
        assert np.array_equal(gd, ref["depth"]), f"frame {i}: gathered depth differs"
    assert counts.shape == (world, world)


def test_config4_virtual_ranks_full_size(gsm, cuda, oracle):
    """BASELINE config 4: 5M gaussians, SH3, 3840x2160, fp16, partitioned over 8 ranks (virtual ranks
    on one GPU, the product kernels and fine-grained exchange memory) -- colour and gathered depth
    bit-exact with the oracle."""
    from gsm_amd import scenes
    c = scenes.CONFIGS["cfg3_5m_sh3_4k_f16"]
    n, w, h, sh, prec = c["count"], c["width"], c["height"], c["sh"], c["precision"]
    world_np, harm_np, cam_d = scenes.gen_scene(n, w, h, sh, prec, seed=42)
    frames, counts, timeouts, depths = _virtual_frame(gsm, cuda, 8, n, w, h, sh, prec, 42, [cam_d])
    assert timeouts == [0] * 8
    ref = oracle.render(world_np, harm_np, sh, cam_d, w, h, max_gaussians=n, nthreads=min(16, os.cpu_count() or 1))
    assert np.array_equal(frames[0], ref["color"])
    assert np.array_equal(depths[0], ref["depth"])
    assert counts.sum() >= int(np.count_nonzero(ref["tile_counts"]))


def test_virtual_ranks_over_poisoned_exchange_memory(gsm, cuda, oracle, monkeypatch):
    """GSM_MG_POISON (the diagnosis switch of tools/exp/mg_uncached_diag.py): the exchange memory is filled
    with 0xAB bytes at prepare, before the write-through zeroing of its control words.  Nothing of a frame may
    read a word it did not write first: three virtual ranks, two views, bit-exact, no timeout."""
    from gsm_amd import scenes
    monkeypatch.setenv("GSM_MG_POISON", "1")
    n, w, h, prec, sh = 30_000, 640, 360, 1, 16
    cams = [scenes.make_camera(w, h), scenes.orbit_camera(w, h, 5.0)]
    frames, _, timeouts, depths = _virtual_frame(gsm, cuda, 3, n, w, h, sh, prec, 91, cams,
                                                 gsm.MultiGpuOptions(timeout_ms=5000))
    assert timeouts == [0] * 3
    world_np, harm_np, _ = scenes.gen_scene(n, w, h, sh, prec, seed=91)
    for got, gd, cam in zip(frames, depths, cams):
        ref = oracle.render(world_np, harm_np, sh, cam, w, h, max_gaussians=n)
        assert np.array_equal(got, ref["color"]) and np.array_equal(gd, ref["depth"])


def test_uncached_exchange_memory_is_refused(gsm, cuda, monkeypatch):
    """GSM_MG_MEM=uncached: refused at gsm_multigpu_prepare (GSM_ERR_UNSUPPORTED) -- uncached memory
    renders wrong virtual-rank slabs on MI355X even with write-through stores and system-coherent
    loads (profiles/r04_mg_memkind_uncached.log)."""
    monkeypatch.setenv("GSM_MG_MEM", "uncached")
    r = gsm.GlobalRenderer(device=0, config=gsm.RendererConfig(max_gaussians=1024, max_width=64, max_height=32))
    with pytest.raises(gsm.RendererError) as e:
        gsm.MultiGpuRenderer.prepare(r, 0, 2)
    assert e.value.status == gsm.Status.UNSUPPORTED
    r.close()


@pytest.mark.parametrize("world,n,w,h,prec", [(3, 60_000, 1280, 720, 1), (8, 50_000, 640, 360, 0)])
def test_virtual_ranks_pipelined(gsm, cuda, oracle, world, n, w, h, prec):
    """options.pipelined (gsm_multigpu_options, r06): every rank runs phases 0-1 on the library's own stream and phases 2-3 on
    the caller's, so frame f + 1's projection and push overlap frame f's slab render; four frames
    (three views) are issued back to back with no host synchronisation, each gathered into its own
    caller tensors, and every frame's colour and depth are bit-exact with the oracle (the receive
    buffers, receive counts, blend schedules and rank 0's gathered frames alternate by frame parity)."""
    from gsm_amd import scenes
    sh = 16 if prec else 4
    world_np, harm_np, cam0 = scenes.gen_scene(n, w, h, sh, prec, seed=91)
    cams = [cam0, scenes.orbit_camera(w, h, 5.0), scenes.orbit_camera(w, h, 10.0), cam0]
    wt = cuda.from_numpy(world_np.view(np.uint8).reshape(-1).copy()).cuda()
    ht = cuda.from_numpy(harm_np.view(np.uint8).reshape(-1).copy()).cuda()
    inp = gsm.GaussianInput(wt, ht, n, sh)
    cfg = gsm.RendererConfig(max_gaussians=n, max_width=w, max_height=h, precision=prec, gaussian_color_space=0)
    rends = [gsm.GlobalRenderer(device=0, config=cfg) for _ in range(world)]
    opts = gsm.MultiGpuOptions(pipelined=True)
    pre = [gsm.MultiGpuRenderer.prepare(r, k, world, opts) for k, r in enumerate(rends)]
    mgs = [m.connect_handles([hd for _, hd in pre]) for m, _ in pre]
    stream = cuda.cuda.current_stream()
    colors = [cuda.full((h, w, 4), float("nan"), dtype=cuda.float16, device="cuda") for _ in cams]
    depths = [cuda.full((h, w), float("nan"), dtype=cuda.float16, device="cuda") for _ in cams]
    for f, cam in enumerate(cams):
        cp = gsm.CameraParams.from_dict(cam)
        for ph in range(4):
            for k, m in enumerate(mgs):
                m.render_phases([ph], colors[f] if k == 0 else None, depths[f] if k == 0 else None, inp, cp, w, h,
                                gather=True, stream=stream, gather_depth=True)
    cuda.cuda.synchronize()
    assert [m.status() for m in mgs] == [0] * world
    for f, cam in enumerate(cams):
        ref = oracle.render(world_np, harm_np, sh, cam, w, h, max_gaussians=n)
        got = colors[f].view(cuda.int16).cpu().numpy().view(np.uint16)
        bad = np.nonzero(np.any(got != ref["color"], axis=(1, 2)))[0]
        assert len(bad) == 0, f"frame {f}: {len(bad)} rows differ, first {bad[:16].tolist()}"
        assert np.array_equal(depths[f].view(cuda.int16).cpu().numpy().view(np.uint16), ref["depth"]), f"frame {f} depth"
    for m in mgs:
        m.close()
    for r in rends:
        r.close()


def test_virtual_ranks_pipelined_inputs_written_between_frames(gsm, cuda, oracle, monkeypatch):
    """pipelined phases 0-1 run on the library's own stream, so a frame's projection is not
    ordered after the caller's stream by itself.  The caller rewrites the one input buffer on its own
    stream between frames (scenes A, B, A, B), records an event after each write and hands it to every
    rank with gsm_multigpu_wait_event; every frame is bit-exact with the oracle of the scene written
    for it."""
    from gsm_amd import scenes
    monkeypatch.setenv("GSM_MG_PIPELINE", "1")
    world, n, w, h, sh, prec = 3, 40_000, 1280, 720, 16, 1
    sc = [scenes.gen_scene(n, w, h, sh, prec, seed=s) for s in (91, 92)]
    srcw = [cuda.from_numpy(x[0].view(np.uint8).reshape(-1).copy()).cuda() for x in sc]
    srch = [cuda.from_numpy(x[1].view(np.uint8).reshape(-1).copy()).cuda() for x in sc]
    wt, ht = cuda.empty_like(srcw[0]), cuda.empty_like(srch[0])
    inp = gsm.GaussianInput(wt, ht, n, sh)
    cfg = gsm.RendererConfig(max_gaussians=n, max_width=w, max_height=h, precision=prec, gaussian_color_space=0)
    rends = [gsm.GlobalRenderer(device=0, config=cfg) for _ in range(world)]
    pre = [gsm.MultiGpuRenderer.prepare(r, k, world) for k, r in enumerate(rends)]
    mgs = [m.connect_handles([hd for _, hd in pre]) for m, _ in pre]
    stream = cuda.cuda.current_stream()
    order = [0, 1, 0, 1]
    cam = sc[0][2]
    cp = gsm.CameraParams.from_dict(cam)
    colors = [cuda.full((h, w, 4), float("nan"), dtype=cuda.float16, device="cuda") for _ in order]
    evs = []
    for f, s in enumerate(order):
        wt.copy_(srcw[s])  # on the caller's stream, after frame f - 1's phases were issued
        ht.copy_(srch[s])
        ev = cuda.cuda.Event()
        ev.record(stream)
        evs.append(ev)
        for m in mgs:
            m.wait_event(ev)
        for ph in range(4):
            for k, m in enumerate(mgs):
                m.render_phases([ph], colors[f] if k == 0 else None, None, inp, cp, w, h, gather=True, stream=stream,
                                gather_depth=False)
    cuda.cuda.synchronize()
    assert [m.status() for m in mgs] == [0] * world
    refs = [oracle.render(sc[s][0], sc[s][1], sh, cam, w, h, max_gaussians=n) for s in (0, 1)]
    for f, s in enumerate(order):
        got = colors[f].view(cuda.int16).cpu().numpy().view(np.uint16)
        bad = np.nonzero(np.any(got != refs[s]["color"], axis=(1, 2)))[0]
        assert len(bad) == 0, f"frame {f} (scene {s}): {len(bad)} rows differ, first {bad[:16].tolist()}"
    for m in mgs:
        m.close()
    for r in rends:
        r.close()


def test_virtual_ranks_phase_order_and_finish_frame(gsm, cuda, oracle):
    """a phase out of order returns GSM_ERR_PHASE_ORDER (nothing enqueued); a caller that
    stopped after phase 1 calls gsm_multigpu_finish_frame (barrier steps, the slabs abandoned with
    failed arrivals at the gather barrier), and the next frame renders bit-exact with no timeout."""
    from gsm_amd import scenes
    world, n, w, h, sh, prec = 2, 30_000, 640, 360, 16, 1
    world_np, harm_np, cam = scenes.gen_scene(n, w, h, sh, prec, seed=17)
    wt = cuda.from_numpy(world_np.view(np.uint8).reshape(-1).copy()).cuda()
    ht = cuda.from_numpy(harm_np.view(np.uint8).reshape(-1).copy()).cuda()
    inp = gsm.GaussianInput(wt, ht, n, sh)
    cfg = gsm.RendererConfig(max_gaussians=n, max_width=w, max_height=h, precision=prec, gaussian_color_space=0)
    rends = [gsm.GlobalRenderer(device=0, config=cfg) for _ in range(world)]
    pre = [gsm.MultiGpuRenderer.prepare(r, k, world) for k, r in enumerate(rends)]
    mgs = [m.connect_handles([hd for _, hd in pre]) for m, _ in pre]
    frame_ptr, _ = mgs[0].frame()
    stream = cuda.cuda.current_stream()
    cp = gsm.CameraParams.from_dict(cam)

    def phases(phs, k):
        mgs[k].render_phases(phs, None, None, inp, cp, w, h, gather=True, stream=stream,
                             gather_target=frame_ptr if k == 0 else None, gather_depth=False)

    for ph in (0, 1):
        for k in range(world):
            phases([ph], k)
    with pytest.raises(gsm.RendererError) as e:  # phase 0 while phase 2 is pending
        phases([0], 0)
    assert e.value.status == gsm.Status.PHASE_ORDER
    # one stream for both ranks: rank 1's remaining steps (its failed gather arrival) before rank 0's
    # gather wait
    mgs[1].finish_frame(stream)
    mgs[0].finish_frame(stream)
    mgs[0].finish_frame(stream)  # nothing pending: a no-op
    for ph in range(4):
        for k in range(world):
            phases([ph], k)
    cuda.cuda.synchronize()
    ref = oracle.render(world_np, harm_np, sh, cam, w, h, max_gaussians=n)
    assert np.array_equal(mgs[0].copy_frame(w, h), ref["color"])
    errs = [m.errors() for m in mgs]
    assert all(t == 0 for t, _ in errs), errs
    assert errs[0][1] >= 1  # rank 1's abandoned slab arrived failed at rank 0's gather barrier
    for m in mgs:
        m.close()
    for r in rends:
        r.close()


@pytest.mark.parametrize("pipelined", ["0", "1"])
def test_virtual_ranks_epoch_wrap(gsm, cuda, oracle, monkeypatch, pipelined):
    """the barrier epochs are frame numbers masked to 31 bits (0 skipped); the flags are compared
    modulo 2^31 and the frame parity (count matrix, receive buffers, schedules, pipelined gathered frames)
    alternates in a counter of its own.  Three ranks start at epoch 2^31 - 4 and render six frames across
    the wrap 2^31 - 1 -> 1 -> 2, serial and pipelined: every frame bit-exact, no barrier timeout."""
    from gsm_amd import scenes
    monkeypatch.setenv("GSM_MG_PIPELINE", pipelined)
    world, n, w, h, sh, prec = 3, 30_000, 640, 360, 16, 1
    world_np, harm_np, cam0 = scenes.gen_scene(n, w, h, sh, prec, seed=23)
    wt = cuda.from_numpy(world_np.view(np.uint8).reshape(-1).copy()).cuda()
    ht = cuda.from_numpy(harm_np.view(np.uint8).reshape(-1).copy()).cuda()
    inp = gsm.GaussianInput(wt, ht, n, sh)
    cfg = gsm.RendererConfig(max_gaussians=n, max_width=w, max_height=h, precision=prec, gaussian_color_space=0)
    rends = [gsm.GlobalRenderer(device=0, config=cfg) for _ in range(world)]
    pre = [gsm.MultiGpuRenderer.prepare(r, k, world) for k, r in enumerate(rends)]
    mgs = [m.connect_handles([hd for _, hd in pre]) for m, _ in pre]
    for m in mgs:
        m.debug_set_epoch(2**31 - 4)
    stream = cuda.cuda.current_stream()
    cams = [cam0, scenes.orbit_camera(w, h, 5.0)] * 3
    colors = [cuda.full((h, w, 4), float("nan"), dtype=cuda.float16, device="cuda") for _ in cams]
    for f, cam in enumerate(cams):
        cp = gsm.CameraParams.from_dict(cam)
        for ph in range(4):
            for k, m in enumerate(mgs):
                m.render_phases([ph], colors[f] if k == 0 else None, None, inp, cp, w, h, gather=True, stream=stream,
                                gather_depth=False)
    cuda.cuda.synchronize()
    assert [m.errors() for m in mgs] == [(0, 0)] * world
    refs = [oracle.render(world_np, harm_np, sh, c, w, h, max_gaussians=n)["color"] for c in cams[:2]]
    for f in range(len(cams)):
        got = colors[f].view(cuda.int16).cpu().numpy().view(np.uint16)
        bad = np.nonzero(np.any(got != refs[f % 2], axis=(1, 2)))[0]
        assert len(bad) == 0, f"frame {f}: {len(bad)} rows differ, first {bad[:16].tolist()}"
    for m in mgs:
        m.close()
    for r in rends:
        r.close()


def test_options_must_agree_across_ranks(gsm, cuda):
    """gsm_multigpu_options are checked at connect like the old environment switches: ranks prepared
    with another row layout, pipelining or transport refuse the connect (GSM_ERR_INVALID_ARGUMENT); a
    malformed options struct (unknown row layout) is refused at prepare; the RCCL transport without a
    communicator is refused at prepare, and pipelined RCCL is unsupported."""
    cfg = gsm.RendererConfig(max_gaussians=4096, max_width=256, max_height=128)
    rends = [gsm.GlobalRenderer(device=0, config=cfg) for _ in range(2)]
    for other in (gsm.MultiGpuOptions(rows="interleaved"), gsm.MultiGpuOptions(pipelined=True)):
        a, ha = gsm.MultiGpuRenderer.prepare(rends[0], 0, 2, gsm.MultiGpuOptions())
        b, hb = gsm.MultiGpuRenderer.prepare(rends[1], 1, 2, other)
        for m in (a, b):
            with pytest.raises(gsm.RendererError) as e:
                m.connect_handles([ha, hb])
            assert e.value.status == gsm.Status.INVALID_ARGUMENT
            m.close()
    bad = gsm.MultiGpuOptions()
    bad.rows = "interleaved"
    o = bad._c()
    o.rows = 7
    import ctypes as C
    h = C.c_void_p()
    buf = C.create_string_buffer(gsm.MULTIGPU_HANDLE_BYTES)
    st = gsm._lib().gsm_multigpu_prepare_with_options(rends[0]._h, 0, 2, C.byref(o), C.byref(h), buf)
    assert st == gsm.Status.INVALID_ARGUMENT
    with pytest.raises(gsm.RendererError) as e:
        gsm.MultiGpuRenderer.prepare(rends[0], 0, 1, gsm.MultiGpuOptions(transport="rccl"))
    assert e.value.status == gsm.Status.INVALID_ARGUMENT
    with pytest.raises(gsm.RendererError) as e:
        gsm.MultiGpuRenderer.prepare(rends[0], 0, 1, gsm.MultiGpuOptions(transport="rccl", pipelined=True, nccl_comm=1))
    assert e.value.status == gsm.Status.UNSUPPORTED
    for r in rends:
        r.close()


def test_fine_exchange_after_freed_uncached_allocations(tmp_path):
    """r05's barrier timeouts came from the first frame of a fine-grained exchange whose
    allocations reused the address ranges of freed *uncached* ones.  A child process (tests/mg_uc_reuse.py)
    replays that sequence twice -- virtual-rank frames over uncached exchange memory (the A/B kind) plus raw
    uncached allocations of the same sizes, all freed, then a fine-grained exchange of the same shape -- and
    the fine-grained exchange must either render both frames bit-exact with zero barrier timeouts, or refuse
    (the mapping check, GSM_ERR_DEVICE_NOT_AVAILABLE, with its evidence on stderr).  r06: gsm_multigpu_prepare
    checks each rank's own allocation and replaces one that fails (held back until destroy), so the
    virtual-rank exchange renders instead of refusing.  The barrier timeout is 2 s, so a lost flag costs
    seconds, not a hang."""
    out = tmp_path / "uc.json"
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    env.pop("GSM_MG_MEM", None)
    r = subprocess.run([sys.executable, os.path.join(os.path.dirname(__file__), "mg_uc_reuse.py"), str(out)], env=env,
                       capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    res = json.loads(out.read_text())
    assert res["cases"], res
    refusals = r.stderr.count("mapping check failed (")
    for c in res["cases"]:
        assert c["refused"] or (c["timeouts"] == 0 and c["bad_rows"] == [0, 0]), c
    # a refusal is the mapping check's, with its evidence on stderr -- not an error left by another call
    # (r06: an error of the child's own raw allocations once read as one)
    assert refusals >= sum(1 for c in res["cases"] if c["refused"]), (res, r.stderr[-3000:])
    assert "mapping check failed to run" not in r.stderr, r.stderr[-3000:]
    print(json.dumps(res["cases"]), "held back:", r.stderr.count("held back"))
