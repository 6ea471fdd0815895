"""The headless entry surface (ray-tracing-gpu_amd/lib/rt_render, Main.cpp:
51-199): the same command line renders the reference's image.  The PPM it
writes (top row first, RGB) is turned back into the GL texture's layout
(bottom row first, RGBA8) and hashed against the digest of the reference
build's frame (tests/golden/digests.json)."""
from __future__ import annotations

import hashlib
import os
import subprocess

import numpy as np
import pytest

from conftest import REPO, rgba8, scene

pytestmark = pytest.mark.gpu
EXE = os.path.join(REPO, "ray-tracing-gpu_amd", "lib", "rt_render")


def read_ppm(path):
    with open(path, "rb") as f:
        data = f.read()
    head = data.split(b"\n", 3)
    assert head[0] == b"P6" and head[2] == b"255"
    w, h = map(int, head[1].split())
    img = np.frombuffer(head[3], np.uint8).reshape(h, w, 3)
    return img


def as_texture(img):
    """PPM (top row first, RGB) -> GL texture memory (bottom row first, RGBA8)."""
    flipped = img[::-1]
    return np.concatenate([flipped, np.full(flipped.shape[:2] + (1,), 255, np.uint8)], -1)


@pytest.mark.parametrize("extra", [["-d", "0"], ["-d", "3"], ["-d", "0", "-g", "3"], ["-d", "3", "-g", "2", "--bands"],
                                   ["-d", "0", "-g", "4", "--bands", "-n", "2"]])
def test_scene2_1080p_matches_reference_digest(tmp_path, digests, extra):
    out = tmp_path / "scene2.ppm"
    r = subprocess.run([EXE, scene(2), "-x", "1920", "-y", "1080", "-o", str(out)] + extra, capture_output=True,
                       text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert "[ETAT]: Termine!" in r.stdout
    tex = as_texture(read_ppm(out))
    assert tex.shape == (1080, 1920, 4)
    assert hashlib.sha256(tex.tobytes()).hexdigest() == digests["scene2_1920x1080_d0_rgba8_sha256"]


@pytest.mark.parametrize("extra", [["-g", "1", "--gather", "rccl"], ["-g", "1", "--gather", "rccl", "-n", "3"],
                                   ["-g", "1", "--gather", "rccl", "-n", "8", "--bands"]])
def test_rccl_gather_matches_reference_digest(tmp_path, digests, extra):
    """rt_render's native RCCL path (librt_gather.so): the rank renders into
    device memory and ONE RCCL group (ncclSend / ncclRecv, here the root to
    itself) gathers the slab into the root GPU's frame; the PPM is the
    reference's frame bit for bit.  On the 8-GPU node -g 8 takes this path
    by default (one rank per GPU, each peer on its own xGMI link)."""
    out = tmp_path / "scene2.ppm"
    r = subprocess.run([EXE, scene(2), "-x", "1920", "-y", "1080", "-o", str(out)] + extra, capture_output=True,
                       text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert "[ETAT]: gather: RCCL" in r.stdout and "send/recv pair(s)" in r.stdout, r.stdout
    # pipelined: frame k + 1 renders while frame k's group runs; per-frame render and gather times
    assert "pipelined (2 slabs)" in r.stdout and "per frame: render" in r.stdout, r.stdout
    tex = as_texture(read_ppm(out))
    assert hashlib.sha256(tex.tobytes()).hexdigest() == digests["scene2_1920x1080_d0_rgba8_sha256"]


def test_rccl_gather_refuses_shared_gpus():
    """RCCL needs one rank per GPU: more contexts than GPUs with --gather rccl
    is an argument error; without it they share GPUs and assemble on the host."""
    import torch

    n = torch.cuda.device_count() + 1
    r = subprocess.run([EXE, scene(2), "-x", "64", "-y", "32", "-g", str(n), "--gather", "rccl"], capture_output=True,
                       text=True, timeout=60)
    assert r.returncode == 1 and "--gather rccl needs one GPU per context" in r.stderr
    r = subprocess.run([EXE, scene(2), "-x", "64", "-y", "32", "-g", str(n)], capture_output=True, text=True,
                       timeout=60)
    assert r.returncode == 0 and "gather: host" in r.stdout, r.stderr


def test_bounce_scene_matches_oracle(tmp_path, oracle):
    out = tmp_path / "scene7.ppm"
    r = subprocess.run([EXE, scene(7), "-x", "96", "-y", "64", "-d", "3", "-s", "-o", str(out)], capture_output=True,
                       text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert "[STATS]: primary=6144" in r.stdout
    want = rgba8(oracle.render(scene(7), 96, 64, 3))
    assert np.array_equal(as_texture(read_ppm(out)), want)


def test_errors_are_reported_not_fatal(tmp_path):
    r = subprocess.run([EXE, str(tmp_path / "missing.dat")], capture_output=True, text=True, timeout=60)
    assert r.returncode == 1 and "[ERREUR]" in r.stderr
    r = subprocess.run([EXE, scene(2), "-g", "0"], capture_output=True, text=True, timeout=60)
    assert r.returncode == 1 and "[ERREUR]" in r.stderr
