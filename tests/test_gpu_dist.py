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
    assert out["n_gpus"] == n
    assert out["frame_rgba8_sha256"] == one_rank["c2"]["frame_rgba8_sha256"]
    # scene2 has no reflective/refractive surface: depth 3 renders the depth-0 image
    assert out["frame_rgba8_sha256"] == digests["scene2_1920x1080_d0_rgba8_sha256"]
    assert out["rays_per_frame"]["primary"] == 1920 * 1080
    want = "row-band16" if partition == "bands" else ("row-slab" if partition == "slabs" else None)
    if want:
        assert out["config"]["parallelism"].startswith(want)


@pytest.mark.parametrize("n", [2, 3])
def test_heightfield_ranks_match_one_rank(one_rank, n):
    """C3: the mesh fills the middle rows, so the measured choice is bands."""
    out = _bench(n, "c3", "auto")
    assert out["frame_rgba8_sha256"] == one_rank["c3"]["frame_rgba8_sha256"]
    assert out["config"]["slab_imbalance"] is not None
