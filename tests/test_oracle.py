"""The oracle (oracle/rt_oracle.c) pinned against the golden fixtures, which
were produced by oracle/_ref — the reference's own Triangle/Plan/Quadrique/
Matrice4/Vecteur3/Couleur sources (tests/golden/make_golden.py).  Everything
here is bit-exact: float32 images, prepared geometry and per-primitive hits."""
from __future__ import annotations

import hashlib
import os

import numpy as np
import pytest

from conftest import bits_equal, rgba8, scene


@pytest.mark.parametrize("i", range(1, 10))
@pytest.mark.parametrize("depth", [0, 1, 3, 5])
def test_oracle_images_match_reference(oracle, golden_images, i, depth):
    got = oracle.render(scene(i), 64, 48, depth)
    assert bits_equal(got, golden_images[f"scene{i}_64x48_d{depth}"])


@pytest.mark.parametrize("wh", [(1, 1), (13, 7), (67, 33)])
def test_oracle_ragged_sizes(oracle, golden_images, wh):
    w, h = wh
    assert bits_equal(oracle.render(scene(5), w, h, 3), golden_images[f"scene5_{w}x{h}_d3"])


@pytest.mark.parametrize("i", range(1, 10))
def test_oracle_prepared_state(oracle, golden_prepared, i):
    s, c, l = oracle.dump(scene(i), 64, 48)
    assert bits_equal(s, golden_prepared[f"scene{i}_surf"])
    assert bits_equal(c, golden_prepared[f"scene{i}_cam"])
    assert bits_equal(l, golden_prepared[f"scene{i}_lights"])
    _, c2, _ = oracle.dump(scene(i), 1920, 1080)
    assert bits_equal(c2, golden_prepared[f"scene{i}_1080p_cam"])


def test_oracle_heightfield_prepared(oracle, golden_prepared, digests, heightfield_path):
    s, c, l = oracle.dump(heightfield_path, 1920, 1080, 1)
    assert s.shape[0] == digests["hf_n_surfaces"] == 50001
    assert hashlib.sha256(s.tobytes()).hexdigest() == digests["hf_surf_sha256"]
    assert bits_equal(c, golden_prepared["hf_cam"]) and bits_equal(l, golden_prepared["hf_lights"])


def test_oracle_kat(oracle, golden_kat):
    keys = sorted({k.rsplit("_", 1)[0] for k in golden_kat.files})
    n = 0
    t = np.zeros(1, np.float32)
    nv = np.zeros(3, np.float32)
    for k in keys:
        typ = int(golden_kat[k + "_type"])
        g, o, d = golden_kat[k + "_geom"], golden_kat[k + "_o"], golden_kat[k + "_d"]
        for j in range(o.shape[0]):
            oj, dj = np.ascontiguousarray(o[j]), np.ascontiguousarray(d[j])
            hit = oracle.L.oracle_intersect(typ, g.ctypes.data, oj.ctypes.data, dj.ctypes.data, t.ctypes.data, nv.ctypes.data)
            assert hit == golden_kat[k + "_hit"][j], (k, j)
            assert bits_equal(t, golden_kat[k + "_t"][j : j + 1]), (k, j)
            assert bits_equal(nv, golden_kat[k + "_n"][j]), (k, j)
            n += 1
    assert n >= 4000


@pytest.mark.parametrize("name,path,w,h,depth", [
    ("scene2_1080p_d0", 2, 1920, 1080, 0),
    ("scene2_1080p_d3", 2, 1920, 1080, 3),
    ("scene7_2160p_d5", 7, 3840, 2160, 5),
    ("scene9_2160p_d5", 9, 3840, 2160, 5),
])
def test_oracle_big_frame_windows(oracle, golden_images, name, path, w, h, depth):
    keys = [k for k in golden_images.files if k.startswith(name + "_win_")]
    assert keys
    for k in keys:
        r0, r1, c0, c1 = map(int, k.rsplit("_win_", 1)[1].split("_"))
        assert bits_equal(oracle.render(scene(path), w, h, depth, (r0, r1, c0, c1)), golden_images[k]), k


def test_oracle_heightfield_windows(oracle, golden_images, heightfield_path):
    keys = [k for k in golden_images.files if k.startswith("hf_1080p_d1_win_")]
    for k in keys:
        r0, r1, c0, c1 = map(int, k.rsplit("_win_", 1)[1].split("_"))
        assert bits_equal(oracle.render(heightfield_path, 1920, 1080, 1, (r0, r1, c0, c1)), golden_images[k]), k


def test_oracle_heightfield_column_windows(oracle, heightfield_path):
    """The restatement against _ref down the C3 frame (make_c3_column_golden.py):
    mesh, shadowed ground, far plane — a third of the windows, for time."""
    with np.load(os.path.join(os.path.dirname(__file__), "golden", "c3_column.npz")) as z:
        keys = sorted(z.files)[::3]
        assert len(keys) >= 15
        for k in keys:
            r0, r1, c0, c1 = map(int, k.rsplit("_win_", 1)[1].split("_"))
            assert bits_equal(oracle.render(heightfield_path, 1920, 1080, 1, (r0, r1, c0, c1), threads=8), z[k]), k


def test_oracle_scene2_1080p_digest(oracle, digests):
    full = oracle.render(scene(2), 1920, 1080, 0, threads=8)
    assert hashlib.sha256(full.tobytes()).hexdigest() == digests["scene2_1920x1080_d0_rgb_f32_sha256"]
    assert hashlib.sha256(rgba8(full).tobytes()).hexdigest() == digests["scene2_1920x1080_d0_rgba8_sha256"]


def test_oracle_depth_semantics(oracle):
    """depth 0 == the shipped executable; bounces only change scenes with Kr/Kt."""
    for i in (1, 2, 3, 4):  # no reflect/refract surfaces
        assert bits_equal(oracle.render(scene(i), 32, 24, 0), oracle.render(scene(i), 32, 24, 5))
    for i in (5, 6, 7, 8, 9):
        assert not bits_equal(oracle.render(scene(i), 32, 24, 0), oracle.render(scene(i), 32, 24, 5))
