"""The N>1 path on CPU: world_size-2 (and 3) gloo process groups run the
product's slab partition + gather (rt_amd.dist) with the oracle standing in
for the per-rank renderer (no GPU here), and the assembled frame must equal
the single-process frame byte for byte."""
from __future__ import annotations

import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import SCENES, rgba8

from rt_amd.dist import slab_rows


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, path, w, h, depth, out_q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from conftest import Oracle
    from rt_amd.dist import gather_frame

    r0, r1, rows = slab_rows(h, world, rank)
    slab = torch.zeros((rows, w, 4), dtype=torch.uint8)
    if r1 > r0:
        img = Oracle().render(path, w, h, depth, (r0, r1, 0, w), threads=1)
        slab[: r1 - r0] = torch.from_numpy(rgba8(img))
    full = torch.zeros((world * rows, w, 4), dtype=torch.uint8)
    gather_frame(slab, full, dist)
    if rank == 0:
        out_q.put(full[:h].numpy().copy())
    dist.barrier()
    dist.destroy_process_group()


def _worker_root(rank, world, port, path, w, h, depth, out_q, band_rows=0, batch=1, nframes=3, send_channels=0):
    """RootGather: `nframes` frames through the double-buffered gather,
    `batch` frames per collective (row slabs, or cyclic bands of
    `band_rows` rows un-permuted on rank 0; send_channels 3: RGB on the
    wire, rank 0 restoring the constant alpha).  Frame k = the scene at depth
    k % 3 (different images per frame)."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from conftest import Oracle
    from rt_amd.dist import RootGather

    g = RootGather(dist, h, w, "cpu", depth=2, band_rows=band_rows, batch=batch, send_channels=send_channels)
    r0, r1, rows = slab_rows(h, world, rank)
    frames = []
    for k in range(nframes):
        buf = g.target(k)
        buf.zero_()
        if band_rows:
            # this rank's bands, packed in order
            for q in range(g.q):
                a = (q * world + rank) * band_rows
                if a < h:
                    e = min(h, a + band_rows)
                    img = Oracle().render(path, w, h, k % 3, (a, e, 0, w), threads=1)
                    buf[q * band_rows: q * band_rows + (e - a)] = torch.from_numpy(rgba8(img))
        elif r1 > r0:
            img = Oracle().render(path, w, h, k % 3, (r0, r1, 0, w), threads=1)
            buf[: r1 - r0] = torch.from_numpy(rgba8(img))
        g.submit(k)
        if rank == 0 and batch == 1 and k >= 1:  # frame by frame, as the frames arrive
            g.wait(k - 1)
            frames.append(g.frame(k - 1).numpy().copy())
    g.finish()
    if rank == 0:
        if batch == 1:
            frames.append(g.frame(nframes - 1).numpy().copy())
        else:  # the last depth * batch frames are held after finish()
            frames = [g.frame(k).numpy().copy() for k in range(nframes)]
        out_q.put(frames)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,h,band_rows,batch,nframes,send_channels", [
    (2, 30, 0, 1, 3, 0), (3, 31, 0, 1, 3, 0), (2, 70, 16, 1, 3, 0), (3, 71, 16, 1, 3, 0), (3, 50, 32, 1, 3, 0),
    (2, 30, 0, 2, 4, 0), (3, 31, 0, 3, 5, 0), (2, 70, 16, 2, 3, 0), (3, 71, 16, 4, 7, 0),
    (2, 30, 0, 1, 3, 3), (3, 31, 0, 3, 5, 3), (3, 71, 16, 4, 7, 3),
    # one rank: the same collective path (frames must not stay the fill)
    (1, 30, 0, 1, 3, 0), (1, 31, 0, 4, 6, 3), (1, 70, 16, 2, 3, 3), (1, 50, 16, 3, 5, 4)])
def test_root_gather_pipelined(oracle, world, h, band_rows, batch, nframes, send_channels):
    w = 36
    path = os.path.join(SCENES, "scene7.dat")
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_root,
                         args=(r, world, port, path, w, h, 0, q, band_rows, batch, nframes, send_channels))
             for r in range(world)]
    for p in procs:
        p.start()
    got = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert len(got) == nframes
    for k in range(nframes):
        assert np.array_equal(got[k], rgba8(oracle.render(path, w, h, k % 3))), k


@pytest.mark.parametrize("world,h", [(2, 30), (3, 31)])
def test_gather_matches_single_frame(oracle, world, h):
    w, depth = 40, 3
    path = os.path.join(SCENES, "scene7.dat")
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, path, w, h, depth, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    want = rgba8(oracle.render(path, w, h, depth))
    assert np.array_equal(got, want)


def test_slab_rows_cover_frame():
    for h in (1, 7, 1080, 4320, 2161):
        for world in (1, 2, 3, 4, 8):
            spans = [slab_rows(h, world, r) for r in range(world)]
            rows = [r1 - r0 for r0, r1, _ in spans]
            assert sum(rows) == h
            assert all(s[2] == spans[0][2] for s in spans)
            assert spans[0][0] == 0 and spans[-1][1] == h
            for a, b in zip(spans, spans[1:]):
                assert a[1] == b[0]


def test_band_layout_covers_frame():
    from rt_amd import band_rows
    from rt_amd.dist import band_layout

    for h in (1, 17, 1080, 4320, 2161):
        for world in (1, 2, 3, 8):
            for br in (16, 32):
                q, rows = band_layout(h, world, br)
                assert rows == q * br
                # every rank's packed band set fits its equal buffer, and the
                # band sets tile the frame's bands exactly once
                assert all(band_rows(h, br, world, r) <= rows for r in range(world))
                assert sum(band_rows(h, br, world, r) for r in range(world)) == -(-h // br) * br


# ---- bench.py's --gpus contract, before any GPU call
def _bench_rc(args, extra_env):
    import subprocess
    import sys

    from conftest import REPO

    env = dict(os.environ, **extra_env)
    return subprocess.run([sys.executable, "bench.py"] + args, cwd=REPO, capture_output=True, text=True,
                          timeout=120, env=env)


def test_bench_refuses_world_size_other_than_gpus():
    r = _bench_rc(["--gpus", "1", "--steps", "1"], {"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode == 2
    assert "WORLD_SIZE=2" in r.stderr and '{"metric"' not in r.stdout
    r = _bench_rc(["--gpus", "8", "--steps", "1"], {"WORLD_SIZE": "4", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode == 2


def test_bench_refuses_zero_gpus():
    r = _bench_rc(["--gpus", "0"], {})
    assert r.returncode == 2


# ---- the N>1 failure bound: bench.py's own dist_setup
# under rank_guard, two gloo ranks, rank 1 misbehaving
@pytest.mark.parametrize("mode", ["before_init", "after_init", "raise"])
def test_rank_failure_ends_the_run(mode):
    import subprocess
    import sys
    import time

    from conftest import REPO

    deadline = 10.0
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(REPO, "tests", "dist_fail_worker.py"), "--mode", mode, "--timeout", str(deadline)]
    env = dict(os.environ, OMP_NUM_THREADS="1")
    t0 = time.perf_counter()
    r = subprocess.run(cmd, cwd=REPO, capture_output=True, text=True, timeout=120, env=env)
    took = time.perf_counter() - t0
    assert r.returncode != 0, (r.stdout, r.stderr[-2000:])
    assert "ok" not in r.stdout.split()
    # rank 0 itself failed with a message naming it (or was stopped by the
    # launcher after rank 1's failure), well inside the deadline + start-up
    assert "rank 0 failed" in r.stderr or "rank 1 failed" in r.stderr, r.stderr[-2000:]
    assert took < deadline + 60, took
