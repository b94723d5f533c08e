"""Multi-GPU screen-slab partition on CPU: partition algebra + a world_size-2 gloo run of
the gather/compose step bench.py uses (every rank contributes its band of the frame;
rank 0 reassembles it).  The bands come from the oracle here; on the GPU the HIP
renderer writes them (test_gpu_parity.test_tile_row_slabs_compose_to_full_frame)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from gsm_amd import slabs


@pytest.mark.parametrize("tiles_y,height,n", [(23, 360, 1), (23, 360, 2), (68, 1080, 8), (135, 2160, 8),
                                              (100, 1600, 3), (5, 70, 8)])
def test_partition_covers_rows_once(tiles_y, height, n):
    ss = slabs.all_slabs(tiles_y, height, n)
    rows = np.zeros(tiles_y, int)
    pix = np.zeros(height, int)
    for s in ss:
        rows[s.row_begin:s.row_end] += 1
        pix[s.y0:s.y1] += 1
        assert s.y1 - s.y0 <= s.rows_padded
    assert np.all(rows == 1) and np.all(pix == 1)


@pytest.mark.parametrize("tiles_y,n", [(23, 2), (68, 8), (135, 8), (5, 8), (5, 16), (68, 3)])
@pytest.mark.parametrize("interleave", [False, True])
def test_native_rank_rows_cover_rows_once(tiles_y, n, interleave):
    """The native multi-GPU frame's row ownership (gsm_amd.exchange.rank_tile_rows, the rule of
    csrc/gsm_multigpu.hip): contiguous blocks or interleaved rows, every tile row owned once."""
    from gsm_amd import exchange
    owned = np.zeros(tiles_y, int)
    for r in range(n):
        rows = exchange.rank_tile_rows(tiles_y, n, r, interleave=interleave)
        assert rows == sorted(rows)
        if interleave:
            assert all(t % n == r for t in rows)
        elif rows:
            assert rows == list(range(rows[0], rows[-1] + 1))
        owned[rows] += 1
    assert np.all(owned == 1)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, frame, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    H = frame.shape[0]
    s = slabs.partition((H + 15) // 16, H, world, rank)
    band = torch.zeros((s.rows_padded,) + frame.shape[1:] + (2,), dtype=torch.uint8)  # fp16 bits as bytes
    band[: s.y1 - s.y0] = torch.from_numpy(np.ascontiguousarray(frame[s.y0:s.y1]).view(np.uint8).reshape(
        (s.y1 - s.y0,) + frame.shape[1:] + (2,)))
    gl = [torch.zeros_like(band) for _ in range(world)] if rank == 0 else None
    dist.gather(band, gather_list=gl, dst=0)
    if rank == 0:
        full = slabs.compose(gl, slabs.all_slabs((H + 15) // 16, H, world), H)
        q.put(bool(np.array_equal(np.ascontiguousarray(full.numpy()).view(np.uint16).reshape(frame.shape), frame)))
    dist.destroy_process_group()


def test_gloo_gather_composes_full_frame(oracle):
    from golden import make_golden as MG
    r = MG.render("synth_20k_640x360_sh3_f16")
    frame = r["color"]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(i, 2, port, frame, q)) for i in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
    assert all(p.exitcode == 0 for p in procs)
    assert q.get(timeout=5) is True
