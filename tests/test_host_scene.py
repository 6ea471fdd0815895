"""The product's host CScene mirror (rt_scene_* in librt_amd.so, reached
through the C ABI): loader, camera, Pretraitement and flattening, pinned
bit-for-bit against the golden fixtures made from the reference's own sources,
and the loader's quirks pinned against the oracle on crafted files.
No GPU needed: these entry points never touch HIP."""
from __future__ import annotations

import hashlib
import os

import numpy as np
import pytest

import rt_amd
from conftest import GOLDEN, bits_equal, scene
from loader_quirks import QUIRK_RES, QUIRKS


def product_dump(path, w, h, depth=0):
    """Product state in the canonical 24/27/7-word layout of oracle_dump."""
    s = rt_amd.Scene(path, w, h, depth)
    t, g, m, l = s.arrays()
    n = t.shape[0]
    out = np.zeros((n, 24), np.float32)
    out[:, 0] = t
    out[:, 1:11] = m
    for i in range(n):
        if t[i] == rt_amd.TRIANGLE:
            out[i, 11:23] = g[i, :12]
        elif t[i] == rt_amd.PLANE:
            out[i, 11:15] = g[i, :4]
        else:
            out[i, 11:21] = g[i, :10]
    f = s.frame
    cam = np.zeros(27, np.float32)
    cam[0:3] = f.cam_pos[:]
    cam[3:19] = f.orient[:]
    cam[20], cam[21], cam[22], cam[23] = f.half_w, f.half_h, f.inv_w, f.inv_h
    cam[24:27] = f.background[:]
    return out, cam, l, s


def cam_eq(a, b):
    # word 19 (camera angle) is not part of rt_frame: the kernel only needs halfW/halfH
    return bits_equal(np.delete(a, 19), np.delete(b, 19))


@pytest.mark.parametrize("i", range(1, 10))
def test_prepared_state_matches_reference(golden_prepared, i):
    s, c, l, _ = product_dump(scene(i), 64, 48)
    assert bits_equal(s, golden_prepared[f"scene{i}_surf"])
    assert cam_eq(c, golden_prepared[f"scene{i}_cam"])
    assert bits_equal(l, golden_prepared[f"scene{i}_lights"])
    _, c2, _, _ = product_dump(scene(i), 1920, 1080)
    assert cam_eq(c2, golden_prepared[f"scene{i}_1080p_cam"])


def test_heightfield_prepared(golden_prepared, digests, heightfield_path):
    s, c, l, _ = product_dump(heightfield_path, 1920, 1080, 1)
    assert s.shape[0] == 50001
    assert hashlib.sha256(s.tobytes()).hexdigest() == digests["hf_surf_sha256"]
    assert cam_eq(c, golden_prepared["hf_cam"])


def test_frame_defaults():
    _, _, _, s = product_dump(scene(2), 320, 200, 3)
    f = s.frame
    assert (f.width, f.height, f.row_begin, f.row_end) == (320, 200, 0, 200)
    assert f.max_bounces == 3 and np.float32(f.min_energy) == np.float32(0.01) and f.scene_ior == 1.0


@pytest.fixture(scope="module")
def quirk_golden():
    with np.load(os.path.join(GOLDEN, "loader_quirks.npz")) as z:
        return {k: z[k] for k in z.files}


@pytest.mark.parametrize("name", sorted(QUIRKS))
def test_loader_quirks_match_reference(quirk_golden, oracle, tmp_path, name):
    """TraiterFichierDeScene's quirks (Scene.cpp:231-501) on crafted files:
    the product's loader + Pretraitement against the reference build's
    (tests/golden/loader_quirks.npz, made by make_loader_golden.py with the
    reference's own CMatrice4 rotate/translate/scale, CCouleur and
    Pretraitement), and the oracle restatement against the same fixture."""
    p = tmp_path / f"{name}.dat"
    p.write_bytes(QUIRKS[name].encode())
    s, c, l, _ = product_dump(str(p), *QUIRK_RES)
    gs, gc, gl = (quirk_golden[f"{name}_{k}"] for k in ("surf", "cam", "lights"))
    assert bits_equal(s, gs) and cam_eq(c, gc) and bits_equal(l, gl)
    so, co, lo = oracle.dump(str(p), *QUIRK_RES)
    assert bits_equal(so, gs) and cam_eq(co, gc) and bits_equal(lo, gl)


def test_stale_rgb_semantics(tmp_path):
    p = tmp_path / "s.dat"
    p.write_text(QUIRKS["stale_rgb"])
    s, c, l, _ = product_dump(str(p), 8, 8)
    # the quadric got the plane's colour through the indented "comment"
    assert bits_equal(s[1, 1:4], s[0, 1:4])
    assert np.allclose(s[0, 1:4], np.array([100, 150, 200]) / 255.0)


def test_long_line_is_an_error_not_a_hang(tmp_path):
    p = tmp_path / "long.dat"
    p.write_text("background: 0 0 0\n" + "*" + "x" * 85 + "\n")
    with pytest.raises(rt_amd.RtError) as e:
        rt_amd.Scene(str(p), 8, 8)
    assert e.value.code == -3
    # 79 characters is still fine
    p.write_text("background: 0 0 0\n" + "*" + "x" * 78 + "\n")
    rt_amd.Scene(str(p), 8, 8)


def test_bad_point_index(tmp_path):
    p = tmp_path / "bad.dat"
    p.write_text("Poly: t\n  point: 3 0 0 0\n")
    with pytest.raises(rt_amd.RtError) as e:
        rt_amd.Scene(str(p), 8, 8)
    assert e.value.code == -3


def test_missing_file():
    with pytest.raises(rt_amd.RtError) as e:
        rt_amd.Scene("/nonexistent/scene.dat", 8, 8)
    assert e.value.code == -2


def test_empty_scene(tmp_path):
    p = tmp_path / "empty.dat"
    p.write_text("")
    s, c, l, sc = product_dump(str(p), 8, 8)
    assert s.shape == (0, 24) and l.shape == (0, 7)
    so, co, lo = rt_amd_oracle_dump(str(p))
    assert cam_eq(c, co)


def rt_amd_oracle_dump(path):
    from conftest import Oracle

    return Oracle().dump(path, 8, 8)


def test_bad_resolution():
    with pytest.raises(rt_amd.RtError):
        rt_amd.Scene(scene(1), 0, 8)
