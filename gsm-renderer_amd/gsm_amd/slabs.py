"""Screen-slab partition of a frame across GPUs.

One process per GPU.  Rank r owns a contiguous band of 32x16 tile rows; every rank
projects all gaussians ("replicas + slab culling", the 8e baseline: no all-to-all),
keeps only the assignments of its rows (gsm_global_set_tile_rows), sorts and blends
them, and the bands are gathered on rank 0 with one collective (RCCL over xGMI on
MI355X, gloo in the CPU tests).
"""
from __future__ import annotations

from dataclasses import dataclass

TILE_H = 16


@dataclass(frozen=True)
class Slab:
    rank: int
    row_begin: int  # tile rows [row_begin, row_end)
    row_end: int
    y0: int         # pixel rows [y0, y1) of the frame
    y1: int
    rows_padded: int  # pixel rows of the (equal-sized) gather buffer


def partition(tiles_y: int, height: int, world_size: int, rank: int) -> Slab:
    """Contiguous, balanced tile-row bands; every rank gets ceil(tiles_y / N) rows except the tail."""
    per = -(-tiles_y // world_size)
    b = min(rank * per, tiles_y)
    e = min(b + per, tiles_y)
    y0 = min(b * TILE_H, height)
    y1 = min(e * TILE_H, height)
    return Slab(rank, b, e, y0, y1, per * TILE_H)


def all_slabs(tiles_y: int, height: int, world_size: int):
    return [partition(tiles_y, height, world_size, r) for r in range(world_size)]


def compose(gathered, slabs, height: int):
    """Stack gathered band buffers (each rows_padded tall) into a full frame (torch or numpy)."""
    parts = [g[: s.y1 - s.y0] for g, s in zip(gathered, slabs) if s.y1 > s.y0]
    try:
        import torch
        if parts and isinstance(parts[0], torch.Tensor):
            return torch.cat(parts, 0)[:height]
    except ImportError:  # pragma: no cover
        pass
    import numpy as np
    return np.concatenate(parts, 0)[:height]
