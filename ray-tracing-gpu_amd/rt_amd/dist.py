"""Row-slab sharding of one frame across ranks + the single gather step.

One process per GPU (torch.distributed; backend "nccl" is RCCL on ROCm).
Every pixel is independent and the scene is read-only, so a frame partitions
into contiguous row slabs with no exchange until the very end, where the
slabs meet in ONE gather over xGMI:

* ``RootGather`` — the frame is assembled on rank 0 (the display / writer):
  rank 0 renders its slab straight into the receive buffer and receives
  every other slab in one ``dist.gather`` per batch of frames (RCCL has no
  ncclGather; torch's NCCL backend issues it as one group of point-to-point
  sends and receives, so each peer uses its own direct xGMI link to the
  root).  Batches are double-buffered, so the gather of batch j runs on
  RCCL's stream while batch j+1 renders on the compute stream.
* ``gather_frame`` — the all-gather form (every rank gets the frame).

Slabs are equal-height (the last one padded) so with one frame per gather
the receive buffer is the frame (``world * rows`` rows in row order, no
permutation pass); a batch of K frames, or cyclic bands, costs rank 0 one
strided device copy per batch.

With the gloo backend (CPU collectives: tests, and several ranks sharing one
GPU, which RCCL refuses) the same gather is staged through host tensors:
each rank copies its slab to the host, gloo gathers the host slabs to rank 0,
and rank 0 copies the frame back into HBM.  RCCL is the default and the only
backend the benchmark's numbers are quoted on.
"""
from __future__ import annotations

import contextlib
import os
import sys
from typing import List, Optional, Tuple

# Collective deadline of the benchmark's process group: a rank that dies or
# hangs makes every other rank's pending rendezvous or collective fail after
# this long (gloo raises; RCCL's watchdog aborts the communicator), instead
# of holding the node until an outer kill.
RANK_TIMEOUT_S = 180.0


def init_ranks(dist, backend: str, device=None, timeout_s: float = RANK_TIMEOUT_S):
    """init_process_group with a deadline (env:// rendezvous from the
    launcher).  backend "nccl" (RCCL) binds the rank's device."""
    import datetime

    kw = {"timeout": datetime.timedelta(seconds=timeout_s)}
    if backend == "nccl":
        kw["device_id"] = device
    dist.init_process_group(backend, **kw)


@contextlib.contextmanager
def rank_guard(rank: int, what: str = "bench.py"):
    """Any exception on a rank ends that process at once with status 1 and a
    one-line message naming the rank (no interpreter teardown, which could
    block in a collective's destructor): the launcher then stops the other
    ranks and exits non-zero, and a rank still waiting on this one fails at
    its collective deadline."""
    try:
        yield
    except SystemExit:
        raise
    except BaseException as e:  # noqa: BLE001 — report any failure, then end the rank
        print(f"{what}: rank {rank} failed: {type(e).__name__}: {e}", file=sys.stderr, flush=True)
        sys.stdout.flush()
        os._exit(1)


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
    """Double-buffered gather of row slabs to rank 0, `batch` frames per
    collective.

    Per frame k: ``out = g.target(k)`` is where this rank renders its slab
    (on rank 0 a view into the gather's own receive buffer; with
    ``send_channels=3`` a staging batch packed to RGB before the gather);
    ``g.submit(k)`` posts the gather once a batch of `batch` frames is
    rendered (one collective for all of them: RCCL's fixed cost per call is
    comparable to a 1/n slab of a 1080p frame, so batching amortises it —
    ``batch=1`` is one gather per frame); ``g.finish()`` posts a partial
    last batch and waits for everything; ``g.frame(k)`` (rank 0) is the
    assembled frame k of the last ``depth * batch`` frames.
    """

    def __init__(self, dist, height: int, width: int, device, depth: int = 2, dtype=None, channels: int = 4,
                 band_rows: int = 0, batch: int = 1, send_channels: int = 0, fill: int = 255):
        import torch

        if batch < 1:
            raise ValueError("batch >= 1")
        self.dist = dist
        self.world = dist.get_world_size()
        self.rank = dist.get_rank()
        self.H, self.W, self.C = height, width, channels
        self.batch = batch
        # send_channels < channels: only the first send_channels of every
        # pixel travel (the RGBA8 frame's alpha is 0xFF for every pixel, so
        # RGB carries it all — 3/4 of the bytes over the links); each rank
        # renders into a staging batch and packs it with one strided copy
        # per batch, rank 0 unpacks into frames whose other channels hold
        # `fill`.
        Ct = send_channels or channels
        if not 0 < Ct <= channels:
            raise ValueError("0 < send_channels <= channels")
        self.Ct = Ct
        self.packed = Ct < channels
        # band_rows > 0: each rank renders cyclic row bands (rt_frame.band_rows)
        # for load balance; rank 0 un-permutes the gathered band sets into
        # frames with one strided copy per batch.
        self.band_rows = band_rows
        if band_rows:
            self.q, self.rows = band_layout(height, self.world, band_rows)
        else:
            _, _, self.rows = slab_rows(height, self.world, self.rank)
        self.depth = depth
        dtype = dtype or torch.uint8
        K, R, n = batch, self.rows, self.world
        # gloo moves host tensors only: stage the device slabs through them
        self.host = str(device) != "cpu" and dist.get_backend() == "gloo"
        if self.rank == 0:
            # receive buffers [rank][frame in batch][row], rank 0's own part
            # rendered (or packed) in place; frames [frame in batch][frame row]
            self.recv = [torch.zeros((n, K, R, width, Ct), dtype=dtype, device=device) for _ in range(depth)]
            # one frame of row slabs per gather: the receive buffer IS the frame
            self.alias = K == 1 and not band_rows and not self.packed
            self.frames = [r.view(K, n * R, width, channels) if self.alias else
                           torch.full((K, n * R, width, channels), fill, dtype=dtype, device=device)
                           for r in self.recv]
            self.slabs = [r[0] for r in self.recv]
            self.views = [[r[i] for i in range(n)] for r in self.recv]
        else:
            self.recv, self.frames, self.views = [], [], []
            self.slabs = [torch.zeros((K, R, width, Ct), dtype=dtype, device=device) for _ in range(depth)]
        # render targets: the slabs themselves, or full-pixel staging batches
        self.stage = ([torch.zeros((K, R, width, channels), dtype=dtype, device=device) for _ in range(depth)]
                      if self.packed else self.slabs)
        if self.host:
            self.h_slabs = [torch.zeros((K, R, width, Ct), dtype=dtype) for _ in range(depth)]
            self.h_recv = ([torch.zeros((n, K, R, width, Ct), dtype=dtype) for _ in range(depth)]
                           if self.rank == 0 else [])
            self.h_views = [[r[i] for i in range(n)] for r in self.h_recv]
        self.pending: List[Optional[list]] = [None] * depth
        self.posted = -1   # last batch whose gather was posted
        self.last = -1     # last frame rendered

    def _slot(self, batch_index: int) -> int:
        return batch_index % self.depth

    def target(self, k: int):
        """Buffer to render frame k's slab into (waits until it is free)."""
        if k % self.batch == 0:
            self._wait_slot(self._slot(k // self.batch))
        self.last = max(self.last, k)
        return self.stage[self._slot(k // self.batch)][k % self.batch]

    def submit(self, k: int):
        """Post the gather of frame k's batch once its last frame is
        rendered: ONE collective call per batch (RCCL runs it as a group of
        point-to-point receives on rank 0 and one send per peer, each over
        its own direct xGMI link), so the host cost per batch does not grow
        with the number of ranks.  With one rank the same collective runs (a
        local copy inside the backend), so packing, bands and the batch
        unpack are the same code at every world size."""
        if k % self.batch != self.batch - 1:
            return
        self._post(k // self.batch)

    def _post(self, bi: int):
        d, b = self.dist, self._slot(bi)
        if self.packed:  # the batch's first Ct channels, one strided copy
            self.slabs[b].copy_(self.stage[b][..., : self.Ct])
        if self.host:
            self.h_slabs[b].copy_(self.slabs[b])  # waits for the renders on the current stream
            views = self.h_views[b] if self.rank == 0 else None
            self.pending[b] = [d.gather(self.h_slabs[b], gather_list=views, dst=0, async_op=True)]
        else:
            views = self.views[b] if self.rank == 0 else None
            self.pending[b] = [d.gather(self.slabs[b], gather_list=views, dst=0, async_op=True)]
        self.posted = bi

    def _wait_slot(self, b: int):
        if self.pending[b] is None:
            return
        for w in self.pending[b]:
            w.wait()
        self.pending[b] = None
        if self.rank != 0:
            return
        if self.host:
            self.recv[b].copy_(self.h_recv[b])
        K, n, R, W, C, Ct = self.batch, self.world, self.rows, self.W, self.C, self.Ct
        if self.alias:
            return
        if self.band_rows:
            # recv[rank][frame][local band][row] -> frames[frame][global band = local * n + rank][row]
            br, q = self.band_rows, self.q
            self.frames[b].view(K, q, n, br, W, C)[..., :Ct].copy_(
                self.recv[b].view(n, K, q, br, W, Ct).permute(1, 2, 0, 3, 4, 5))
        else:
            self.frames[b].view(K, n, R, W, C)[..., :Ct].copy_(self.recv[b].transpose(0, 1))

    def wait(self, k: int):
        """Wait for the gather of frame k's batch (posted by submit/finish)."""
        self._wait_slot(self._slot(k // self.batch))

    def finish(self):
        """Post a partial last batch, then wait for every pending gather."""
        if self.last >= 0 and self.last // self.batch > self.posted:
            self._post(self.last // self.batch)
        for b in range(self.depth):
            self._wait_slot(b)

    def frame(self, k: int):
        """Rank 0: the assembled frame k (H rows, bottom-up)."""
        return self.frames[self._slot(k // self.batch)][k % self.batch][: self.H]
