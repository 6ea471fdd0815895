"""The N>1 product path on one GPU: bench.py itself, launched by
torch.distributed.run with 2 and 3 ranks, each rank rendering its share with
librt_amd.so (row slabs, cyclic 16-row bands, or the measured choice) and
rt_amd.dist.RootGather assembling the frame on rank 0 — over gloo, staged
through host memory, since RCCL refuses two ranks on one device.  The
assembled RGBA8 frame must be byte-identical to the 1-rank frame, and for
scene2 to the reference's digest ("validate by running n
virtual ranks on one GPU and requiring byte-equality with the 1-rank
image")."""
from __future__ import annotations

import json
import os
import socket
import subprocess
import sys

import pytest

from conftest import REPO

pytestmark = pytest.mark.gpu


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _bench(n, config, partition="auto", gather_batch=4, gather_channels=3):
    args = ["bench.py", "--gpus", str(n), "--steps", "3", "--warmup", "1", "--config", config, "--frame-sha",
            "--no-cpu-baseline", "--no-host-boundary"]
    if n > 1:
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", str(n),
               "--master-addr", "127.0.0.1", "--master-port", str(_port())] + args + [
                   "--dist-backend", "gloo", "--partition", partition,
                   "--gather-batch", str(gather_batch), "--gather-channels", str(gather_channels)]
    else:
        cmd = [sys.executable] + args
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0", OMP_NUM_THREADS="2")
    r = subprocess.run(cmd, cwd=REPO, capture_output=True, text=True, timeout=240, env=env)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith('{"metric"')]
    assert len(lines) == 1, r.stdout[-2000:]
    return json.loads(lines[0])


@pytest.fixture(scope="module")
def one_rank():
    return {c: _bench(1, c) for c in ("c2", "c3")}


# 4 frames per run (1 warmup + 3 timed): gather batches of 4 (one collective),
# 1 (one per frame) and 3 (a full batch, then a partial one posted by finish);
# RGB on the wire (the default) and the RGBA8 pixels as rendered
@pytest.mark.parametrize("n,partition,gather_batch,gather_channels", [
    (2, "slabs", 4, 3), (2, "bands", 4, 3), (3, "auto", 4, 3), (3, "slabs", 1, 3), (2, "bands", 3, 3),
    (3, "slabs", 3, 4), (2, "slabs", 1, 4)])
def test_scene2_ranks_match_reference_digest(one_rank, digests, n, partition, gather_batch, gather_channels):
    out = _bench(n, "c2", partition, gather_batch, gather_channels)
    assert out["n_gpus"] == out["ranks_seen"] == n
    assert out["frame_rgba8_sha256"] == one_rank["c2"]["frame_rgba8_sha256"]
    # the N>1 model's terms
    rk = out["ranks"]
    assert 0 < rk["render_ms_fastest"] <= rk["render_ms_slowest"]
    assert rk["gather_ms_per_batch"] > 0 and rk["gather_batch"] == gather_batch
    assert rk["bytes_per_link_per_frame"] > 0
    # scene2 has no reflective/refractive surface: depth 3 renders the depth-0 image
    assert out["frame_rgba8_sha256"] == digests["scene2_1920x1080_d0_rgba8_sha256"]
    assert out["rays_per_frame"]["primary"] == 1920 * 1080
    want = "row-band16" if partition == "bands" else ("row-slab" if partition == "slabs" else None)
    if want:
        assert out["config"]["parallelism"].startswith(want)


def _bare(args, timeout=240):
    """bench.py started the way the driver may start it — no launcher."""
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0", OMP_NUM_THREADS="2")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    return subprocess.run([sys.executable, "bench.py"] + args, cwd=REPO, capture_output=True, text=True,
                          timeout=timeout, env=env)


def test_bare_bench_gpus_n_runs_n_ranks(one_rank, digests):
    """`bench.py --gpus 2` without a launcher starts the
    two ranks itself (torch.distributed.run as a child) — here sharing the
    one GPU over gloo — and the line proves both joined the collective."""
    r = _bare(["--gpus", "2", "--dist-backend", "gloo", "--frame-sha", "--steps", "3", "--warmup", "1",
               "--config", "c2", "--no-cpu-baseline", "--no-host-boundary"])
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith('{"metric"')]
    assert len(lines) == 1, r.stdout[-2000:]
    out = json.loads(lines[0])
    assert out["n_gpus"] == out["ranks_seen"] == 2
    assert out["gpus_used"] == 1  # both gloo ranks on the box's one GPU
    assert out["frame_rgba8_sha256"] == digests["scene2_1920x1080_d0_rgba8_sha256"]
    assert out["frame_rgba8_sha256"] == one_rank["c2"]["frame_rgba8_sha256"]


def test_bare_bench_refuses_more_rccl_ranks_than_gpus():
    """Two RCCL ranks on a one-GPU box: refused with a message, non-zero."""
    import torch

    if torch.cuda.device_count() >= 2:
        pytest.skip("more than one GPU visible")
    r = _bare(["--gpus", "2", "--steps", "2", "--warmup", "1", "--no-cpu-baseline", "--no-host-boundary"])
    assert r.returncode != 0
    assert "visible GPU" in r.stderr
    assert '{"metric"' not in r.stdout


@pytest.mark.parametrize("n", [2, 3])
def test_heightfield_ranks_match_one_rank(one_rank, n):
    """C3: the mesh fills the middle rows, so the measured choice is bands."""
    out = _bench(n, "c3", "auto")
    assert out["frame_rgba8_sha256"] == one_rank["c3"]["frame_rgba8_sha256"]
    assert out["config"]["slab_imbalance"] is not None


# ---- RCCL itself on the 1-GPU box: an "nccl" process
# group of one rank runs the code the driver's 8-GPU run depends on — the
# process-group init with device_id, the CUDA-tensor all-reduce, and
# RootGather's dist.gather of device tensors with async_op on RCCL's stream.
def _rccl_worker(port, cfgs, q):
    import numpy as np
    import torch
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0", WORLD_SIZE="1")
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
    try:
        assert dist.get_backend() == "nccl"
        t = torch.tensor([2.5], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        assert float(t.item()) == 2.5
        import rt_amd
        from rt_amd.dist import RootGather, band_layout

        s = rt_amd.Scene(os.path.join(REPO, "tests", "golden", "scenes", "scene7.dat"), 96, 70, 3)
        ctx = rt_amd.Context(0)
        ctx.upload(s)
        stream = torch.cuda.current_stream().cuda_stream
        fails = []
        for band, batch, ch, nframes in cfgs:
            g = RootGather(dist, 70, 96, "cuda", band_rows=band, batch=batch, send_channels=ch)
            want = []
            for k in range(nframes):
                f = s.frame.copy()
                f.cam_pos[0] += 0.5 * k  # a different image per frame
                if band:
                    f.band_rows, f.band_count, f.band_index = band, 1, 0
                out = g.target(k)
                ctx.render_async(f, out.data_ptr(), 0, stream)
                g.submit(k)
                full = s.frame.copy()
                full.cam_pos[0] += 0.5 * k
                want.append(ctx.render(full))
            g.finish()
            for k in range(max(0, nframes - 2 * batch), nframes):
                got = g.frame(k).cpu().numpy()
                if not np.array_equal(got, want[k]):
                    fails.append((band, batch, ch, k))
        ctx.close()
        q.put(("ok", fails))
    except Exception as e:  # report, then tear down
        q.put(("error", repr(e)))
    finally:
        dist.destroy_process_group()


def test_rccl_one_rank_root_gather():
    import torch.multiprocessing as mp

    cfgs = [(0, 1, 0, 3), (0, 4, 0, 6), (0, 1, 3, 3), (0, 4, 3, 7), (16, 1, 3, 3), (16, 4, 4, 6), (16, 3, 3, 5)]
    ctxm = mp.get_context("spawn")
    q = ctxm.Queue()
    p = ctxm.Process(target=_rccl_worker, args=(_port(), cfgs, q))
    p.start()
    status, res = q.get(timeout=180)
    p.join(timeout=60)
    assert status == "ok", res
    assert res == [], res
    assert p.exitcode == 0


def test_bench_nccl_one_rank_runs_the_rccl_path(one_rank):
    """bench.py under torch.distributed.run with one rank and --force-dist:
    init_process_group("nccl", device_id=...), the CUDA-tensor all-reduces and
    the RootGather path, with the frame byte-identical to the plain run."""
    args = ["bench.py", "--gpus", "1", "--steps", "3", "--warmup", "1", "--config", "c2", "--frame-sha",
            "--no-cpu-baseline", "--no-host-boundary", "--force-dist", "--dist-backend", "nccl"]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", "1",
           "--master-addr", "127.0.0.1", "--master-port", str(_port())] + args
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0", OMP_NUM_THREADS="2")
    r = subprocess.run(cmd, cwd=REPO, capture_output=True, text=True, timeout=240, env=env)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith('{"metric"')]
    assert len(lines) == 1, r.stdout[-2000:]
    out = json.loads(lines[0])
    assert "RCCL gather" in out["config"]["parallelism"]
    assert out["ranks"]["bytes_per_link_per_frame"] == 1920 * 1080 * 3
    assert out["frame_rgba8_sha256"] == one_rank["c2"]["frame_rgba8_sha256"]
