"""Row-slab sharding of one frame across ranks + the single gather step.

One process per GPU (torch.distributed; backend "nccl" is RCCL on ROCm).
Every pixel is independent and the scene is read-only, so a frame partitions
into contiguous row slabs with no exchange until the very end, where the
slabs meet in ONE gather over xGMI:

* ``RootGather`` — the frame is assembled on rank 0 (the display / writer):
  rank 0 renders its slab straight into the frame buffer and receives every
  other slab in one ``dist.gather`` per frame (RCCL has no ncclGather;
  torch's NCCL backend issues it as one group of point-to-point sends and
  receives, so each peer uses its own direct xGMI link to the root).  Frames
  are double-buffered, so the gather of frame k runs on RCCL's stream while
  frame k+1 renders on the compute stream.
* ``gather_frame`` — the all-gather form (every rank gets the frame).

Slabs are equal-height (the last one padded) so a frame is one contiguous
buffer of ``world * rows`` rows in row order — no permutation pass.

With the gloo backend (CPU collectives: tests, and several ranks sharing one
GPU, which RCCL refuses) the same gather is staged through host tensors:
each rank copies its slab to the host, gloo gathers the host slabs to rank 0,
and rank 0 copies the frame back into HBM.  RCCL is the default and the only
backend the benchmark's numbers are quoted on.
"""
from __future__ import annotations

from typing import List, Optional, Tuple


def slab_rows(height: int, world: int, rank: int) -> Tuple[int, int, int]:
    """(row_begin, row_end, padded_rows) of `rank`'s slab; row 0 = bottom.
    Slab heights are multiples of 8 rows (the last slab takes the rest)."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError("bad world/rank")
    # heights in whole 8-row tiles, so every wave covers one tile row of the
    # frame (the camera buffer's unit)
    rows = -(-(-(-height // world)) // 8) * 8
    r0 = min(height, rank * rows)
    r1 = min(height, (rank + 1) * rows)
    return r0, r1, rows


def band_layout(height: int, world: int, band_rows: int = 16) -> Tuple[int, int]:
    """Cyclic row bands (rt_frame.band_rows): (bands per rank Q, rows per
    rank Q * band_rows).  Every rank gets an equal buffer; rank r's band k is
    the frame's band k * world + r (rows past the frame are left unwritten)."""
    if world <= 0 or band_rows <= 0 or band_rows % 16:
        raise ValueError("bad band layout")
    q = -(-(-(-height // band_rows)) // world)
    return q, q * band_rows


def gather_frame(slab, full, dist, group=None):
    """All-gather equal-height slabs into `full` ([world*rows, W, 4]) on every
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


class RootGather:
    """Double-buffered gather of row slabs to rank 0.

    Per frame k: ``out = g.target(k)`` is where this rank renders its slab
    (on rank 0 a view into frame buffer k % depth); ``g.submit(k)`` posts the
    sends/receives asynchronously; ``g.frame(k)`` (rank 0) is the assembled
    frame once ``g.wait(k)`` (or ``g.finish()``) has run.
    """

    def __init__(self, dist, height: int, width: int, device, depth: int = 2, dtype=None, channels: int = 4,
                 band_rows: int = 0):
        import torch

        self.dist = dist
        self.world = dist.get_world_size()
        self.rank = dist.get_rank()
        self.H, self.W, self.C = height, width, channels
        # band_rows > 0: each rank renders cyclic row bands (rt_frame.band_rows)
        # for load balance; rank 0 gathers the band sets into a staging buffer
        # and un-permutes them into the frame with one strided copy.
        self.band_rows = band_rows
        if band_rows:
            self.q, self.rows = band_layout(height, self.world, band_rows)
        else:
            _, _, self.rows = slab_rows(height, self.world, self.rank)
        self.depth = depth
        dtype = dtype or torch.uint8
        shape_full = (self.world * self.rows, width, channels)
        shape_slab = (self.rows, width, channels)
        # gloo moves host tensors only: stage the device slabs through them
        self.host = str(device) != "cpu" and dist.get_backend() == "gloo"
        if self.host:
            self.h_slabs = [torch.zeros(shape_slab, dtype=dtype) for _ in range(depth)]
            self.h_full = ([torch.zeros(shape_full, dtype=dtype) for _ in range(depth)] if self.rank == 0 else [])
            self.h_views = ([[f[r * self.rows:(r + 1) * self.rows] for r in range(self.world)] for f in self.h_full]
                            if self.rank == 0 else [])
        self.staging = []
        if self.rank == 0:
            self.frames = [torch.zeros(shape_full, dtype=dtype, device=device) for _ in range(depth)]
            if band_rows:
                self.staging = [torch.zeros(shape_full, dtype=dtype, device=device) for _ in range(depth)]
            src = self.staging if band_rows else self.frames
            self.slabs = [f[: self.rows] for f in src]
            # the gather's targets: row blocks in rank order (contiguous views)
            self.views = [[f[r * self.rows:(r + 1) * self.rows] for r in range(self.world)] for f in src]
        else:
            self.frames = []
            self.slabs = [torch.zeros(shape_slab, dtype=dtype, device=device) for _ in range(depth)]
            self.views = []
        self.pending: List[Optional[list]] = [None] * depth

    def target(self, k: int):
        """Buffer to render frame k's slab into (waits until it is free)."""
        self.wait(k)
        return self.slabs[k % self.depth]

    def submit(self, k: int):
        """Post frame k's gather: ONE collective call per frame (RCCL runs it
        as a group of point-to-point receives on rank 0 and one send per
        peer, each over its own direct xGMI link), so the host cost per frame
        does not grow with the number of ranks."""
        if self.world == 1:
            return
        d, b = self.dist, k % self.depth
        if self.host:
            import torch

            self.h_slabs[b].copy_(self.slabs[b])  # waits for the render on the current stream
            views = self.h_views[b] if self.rank == 0 else None
            self.pending[b] = [d.gather(self.h_slabs[b], gather_list=views, dst=0, async_op=True)]
            return
        views = self.views[b] if self.rank == 0 else None
        self.pending[b] = [d.gather(self.slabs[b], gather_list=views, dst=0, async_op=True)]

    def wait(self, k: int):
        b = k % self.depth
        if self.pending[b] is not None:
            for w in self.pending[b]:
                w.wait()
            self.pending[b] = None
            if self.host and self.rank == 0:
                (self.staging if self.band_rows else self.frames)[b].copy_(self.h_full[b])
            if self.band_rows and self.rank == 0:
                # staging[rank][local band][row] -> frame[global band = local * world + rank][row]
                br, W, C = self.band_rows, self.W, self.C
                self.frames[b].view(self.q, self.world, br, W, C).copy_(
                    self.staging[b].view(self.world, self.q, br, W, C).transpose(0, 1))

    def finish(self):
        for b in range(self.depth):
            self.wait(b)

    def frame(self, k: int):
        """Rank 0: the assembled frame k (H rows, bottom-up)."""
        return self.frames[k % self.depth][: self.H]
