"""Moved cameras against the reference on the CPU box (tests/golden/
cameras.json, made by oracle/_ref with each frame's explicit camera words —
ref_set_camera, the state Scene.cpp:1538-1561 reads per pixel).

* the oracle's C restatement (oracle_set_camera) and the product's CPU
  backend (rt_cpu_render_float / rt_cpu_render) render every turned /
  moved / widened camera and camera-path frame of tests/cameras.py bit for
  bit like the reference, on scene2 (depth 0), scene7 (depth 3) and scene9
  (depth 5); the 50k-triangle heightfield frames are checked on the GPU only
  (a brute-force CPU frame of it takes minutes);
* the fixtures' camera words are the ones tests/cameras.py builds (a drift
  fails here first, before any pixel comparison on the GPU)."""
from __future__ import annotations

import ctypes
import os

import numpy as np
import pytest

import cameras
import rt_amd
from conftest import CamRef, cam_golden

THREADS = min(8, os.cpu_count() or 1)
CPU_SETS = ["scene2", "scene7", "scene9"]


def test_fixture_keys_and_words(heightfield_path):
    for which, *_ in cameras.SETS:
        CamRef(which, heightfield_path)  # asserts every frame's camera words
    keys = {cameras.key(w, k, i) for w, *_ in cameras.SETS for k in cameras.KINDS for i in range(6)}
    keys |= {"scene7_3840x2160_d5_full", "scene9_3840x2160_d5_full"}
    name, w, h, d, idx = cameras.MOVING_FULL
    keys |= {f"{name}_{w}x{h}_d{d}_moving{i}" for i in idx}
    assert keys == set(cam_golden())


@pytest.mark.parametrize("which", CPU_SETS)
@pytest.mark.parametrize("kind", ["cams", "path", "moving"])
def test_oracle_explicit_camera(oracle, heightfield_path, which, kind):
    r = CamRef(which, heightfield_path)
    L = oracle.L
    L.oracle_set_camera.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p] + [ctypes.c_float] * 4 + \
                                   [ctypes.c_int, ctypes.c_int]
    rc, p = oracle.load(r.path, r.w, r.h, r.depth)
    assert rc == 0
    try:
        for i, f in enumerate(r.frames[kind]):
            w = cameras.words(f)
            pos, orient = np.asarray(w[:3], np.float32), np.asarray(w[3:19], np.float32)
            assert L.oracle_set_camera(p, pos.ctypes.data, orient.ctypes.data, *w[19:23], r.w, r.h) == 0
            out = np.zeros((r.h, r.w, 3), np.float32)
            L.oracle_render_window(p, 0, r.h, 0, r.w, out.ctypes.data, THREADS)
            assert r.matches(out, kind, i), (which, kind, i)
    finally:
        L.oracle_free(p)


@pytest.mark.parametrize("which", CPU_SETS)
def test_cpu_backend_moved_cameras(heightfield_path, which):
    r = CamRef(which, heightfield_path)
    ctx = rt_amd.CpuContext(THREADS)
    ctx.upload(r.scene)
    for kind, frames in r.frames.items():
        for i, f in enumerate(frames):
            assert r.matches(ctx.render_float(f), kind, i), (which, kind, i)
            assert r.matches(ctx.render(f), kind, i), (which, kind, i, "rgba8")
    ctx.close()
