"""All-to-all partition exchange on CPU (gsm_amd.exchange): world_size 2 and 3 with gloo.
Each rank sends slab-major byte records; every rank must receive exactly its slab's
records from all ranks, concatenated in source-rank order (the order the GPU renderer's
stable sort relies on), and the single-process emulation used by the GPU parity test must
agree with the real collective.  The device side (project_partition / render_records) is
covered bit-exactly by tests/test_gpu_parity.py::test_partitioned_frame_matches_single_gpu."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from gsm_amd import exchange

R = exchange.RECORD_BYTES


def _records(rank, world, n_per):
    """Deterministic records: rank r sends n_per[r][d] records to slab d; byte pattern encodes
    (source rank, destination, index) so the receiver can check provenance and order."""
    chunks = []
    for d in range(world):
        for i in range(n_per[rank][d]):
            rec = torch.zeros(R, dtype=torch.uint8)
            rec[0], rec[1], rec[2], rec[3] = rank, d, i & 0xFF, i >> 8
            chunks.append(rec)
    return torch.cat(chunks) if chunks else torch.zeros(0, dtype=torch.uint8)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, n_per, q, short_rank=-1):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    send = _records(rank, world, n_per)
    counts = torch.tensor(n_per[rank], dtype=torch.int32)
    need = sum(n_per[r][rank] for r in range(world)) * R
    recv = torch.zeros(need - R if rank == short_rank else need + 64, dtype=torch.uint8)
    if short_rank >= 0:  # every rank must raise, none may block in the records collective
        try:
            exchange.exchange(send, counts, recv)
            q.put((rank, -1, False))
        except ValueError:
            q.put((rank, 0, True))
        dist.destroy_process_group()
        return
    got = exchange.exchange(send, counts, recv)
    sends = [_records(r, world, n_per) for r in range(world)]
    want = exchange.emulate(sends, n_per)[rank]
    q.put((rank, got, bool(torch.equal(recv[: got * R], want))))
    dist.destroy_process_group()


@pytest.mark.parametrize("n_per", [
    [[3, 5], [0, 7]],                       # world 2, an empty segment
    [[2, 0, 4], [1, 1, 1], [0, 300, 2]],    # world 3, a large segment
])
def test_gloo_all_to_all_delivers_slab_records_in_rank_order(n_per):
    world = len(n_per)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n_per, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
    assert all(p.exitcode == 0 for p in procs)
    res = sorted(q.get(timeout=5) for _ in range(world))
    for rank, got, ok in res:
        assert got == sum(n_per[r][rank] for r in range(world))
        assert ok


def test_too_small_receive_buffer_raises_on_every_rank():
    n_per = [[2, 0, 4], [1, 1, 1], [0, 3, 2]]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 3, port, n_per, q, 1)) for r in range(3)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
    assert all(p.exitcode == 0 for p in procs)
    assert all(ok for _, _, ok in (q.get(timeout=5) for _ in range(3)))


def test_id_ranges_and_slab_rows_cover_everything():
    for n, world in [(1_000_000, 8), (7, 3), (0, 2), (5, 8)]:
        rs = [exchange.id_range(n, world, r) for r in range(world)]
        assert sum(c for _, c in rs) == n
        assert all(rs[i][0] + rs[i][1] <= rs[i + 1][0] or rs[i + 1][1] == 0 for i in range(world - 1))
    rows = exchange.slab_rows(68, 1080, 8)
    assert rows[0] == 0 and rows[-1] == 68 and rows == sorted(rows) and len(rows) == 9
