"""Row-slab sharding of one frame across ranks + the single gather step.

One process per GPU (torch.distributed; backend "nccl" is RCCL on ROCm).
Every pixel is independent and the scene is read-only, so a frame partitions
into contiguous row slabs with no exchange until the very end, where ONE
all-gather over xGMI assembles the RGBA8 frame.  Slabs are
equal-height (the last one padded) so the gather is a single
``all_gather_into_tensor`` whose output is the frame in row order — no
permutation pass.
"""
from __future__ import annotations

from typing import Tuple


def slab_rows(height: int, world: int, rank: int) -> Tuple[int, int, int]:
    """(row_begin, row_end, padded_rows) of `rank`'s slab; row 0 = bottom."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError("bad world/rank")
    rows = -(-height // world)
    r0 = min(height, rank * rows)
    r1 = min(height, (rank + 1) * rows)
    return r0, r1, rows


def gather_frame(slab, full, dist, group=None):
    """Assemble equal-height slabs into `full` ([world*rows, W, 4]) on every
    rank.  RCCL: one all-gather; gloo (CPU tests): the list form."""
    world = dist.get_world_size(group)
    if world == 1:
        if full.data_ptr() != slab.data_ptr():
            full.copy_(slab)
        return full
    if dist.get_backend(group) == "gloo":
        parts = list(full.chunk(world, 0))
        dist.all_gather(parts, slab.contiguous(), group=group)
        return full
    dist.all_gather_into_tensor(full, slab, group=group)
    return full
