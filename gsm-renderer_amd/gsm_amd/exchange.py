"""All-to-all screen-slab partition of one frame across GPUs (the north-star
variant; include/gsm_multigpu.h for the device side).

One process per GPU.  Rank r owns the gaussian ids [first_r, first_r + count_r) and the tile
rows of slab r (gsm_amd.slabs).  Per frame:

  1. project_partition: rank r projects its ids once and packs, per slab, the 48-byte
     records of its gaussians that meet that slab (ascending id order);
  2. all_to_all of the per-slab counts, then all_to_all(v) of the records (RCCL over xGMI
     on MI355X; gloo in the CPU tests): rank d receives slab d's records from every rank,
     concatenated in source-rank order -- ascending id order, so the stable sort's ties
     break exactly as on one GPU;
  3. render_records: rank d renders its slab's rows from the records.

Only the gaussians a slab needs cross the fabric, once per (gaussian, slab), instead of
every rank projecting every gaussian ("replicas", gsm_amd.slabs).
"""
from __future__ import annotations

from typing import List, Sequence, Tuple

from . import slabs as _slabs

RECORD_BYTES = 48


def id_range(n: int, world_size: int, rank: int) -> Tuple[int, int]:
    """Contiguous, balanced id ranges: (first, count) of rank."""
    per = -(-n // world_size) if n else 0
    first = min(rank * per, n)
    return first, min(per, n - first)


def slab_rows(tiles_y: int, height: int, world_size: int) -> List[int]:
    """num_slabs + 1 tile-row boundaries of the ranks' slabs (gsm_global_project_partition)."""
    ss = _slabs.all_slabs(tiles_y, height, world_size)
    return [s.row_begin for s in ss] + [ss[-1].row_end]


def rank_tile_rows(tiles_y: int, world_size: int, rank: int, interleave: bool = False) -> List[int]:
    """Tile rows rank owns in the native multi-GPU frame (gsm_multigpu_render): its contiguous
    block of ceil(tiles_y / W) rows (the default), or rows rank, rank + W, rank + 2W, ... when the
    ranks were prepared with GSM_MG_ROWS=interleaved."""
    if interleave:
        return list(range(rank, tiles_y, world_size))
    per = -(-tiles_y // world_size)
    return list(range(min(rank * per, tiles_y), min((rank + 1) * per, tiles_y)))


def exchange(send, send_counts, recv, group=None, staged: bool = False) -> int:
    """all_to_all of per-slab record counts, then of the records themselves.

    send: byte tensor holding the slab-major records of this rank; send_counts: int32
    tensor, one count per destination rank; recv: byte tensor large enough for every
    record this rank receives.  Returns the number of records received (they sit at the
    front of `recv` in source-rank order).  Works for any torch.distributed backend that
    implements all_to_all_single (nccl = RCCL on ROCm, gloo).  staged=True moves device
    tensors through host memory (gloo rehearsal of a multi-GPU run)."""
    import torch
    import torch.distributed as dist

    if staged and send.is_cuda:
        hr = torch.empty(recv.numel(), dtype=torch.uint8)
        got = exchange(send.cpu(), send_counts.cpu(), hr, group=group)
        recv[: got * RECORD_BYTES].copy_(hr[: got * RECORD_BYTES])
        return got
    recv_counts = torch.empty_like(send_counts)
    dist.all_to_all_single(recv_counts, send_counts, group=group)
    sc = [int(x) for x in send_counts.tolist()]
    rc = [int(x) for x in recv_counts.tolist()]
    out_bytes = sum(rc) * RECORD_BYTES
    in_bytes = sum(sc) * RECORD_BYTES
    # a too-small receive buffer on any rank must stop every rank before the records collective
    # (one rank raising alone would leave the others blocked in it)
    short = torch.tensor([1 if recv.numel() < out_bytes else 0], dtype=torch.int32, device=send_counts.device)
    dist.all_reduce(short, op=dist.ReduceOp.MAX, group=group)
    if int(short.item()):
        raise ValueError(f"a receive buffer is too small (this rank: {recv.numel()} B for {out_bytes} B arriving)")
    dist.all_to_all_single(recv[:out_bytes], send[:in_bytes],
                           output_split_sizes=[c * RECORD_BYTES for c in rc],
                           input_split_sizes=[c * RECORD_BYTES for c in sc], group=group)
    return sum(rc)


def emulate(sends: Sequence, counts: Sequence[Sequence[int]]):
    """Single-process stand-in for `exchange` over R virtual ranks (tests): sends[r] holds
    rank r's slab-major records, counts[r][d] how many go to slab d.  Returns, per slab d,
    the concatenation in source-rank order that rank d would receive."""
    import torch

    world = len(sends)
    out = []
    for d in range(world):
        parts = []
        for r in range(world):
            off = sum(counts[r][:d]) * RECORD_BYTES
            parts.append(sends[r][off: off + counts[r][d] * RECORD_BYTES])
        out.append(torch.cat(parts) if parts else sends[0][:0])
    return out
