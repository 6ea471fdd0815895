"""CPU side of the bounce-ray BVH (rt_bvh.h): the margin bound its box test
relies on, checked on adversarial ray-triangle pairs evaluated with the
reference's float32 operation order (tools/bvh_bound_probe.py), and the
oracle restatement pinned to the reference build on the reflective
heightfield the BVH kernels render (tests/golden/hf_reflect.npz)."""
from __future__ import annotations

import os
import sys

import numpy as np
import pytest

from conftest import GOLDEN, REPO, bits_equal

sys.path.insert(0, os.path.join(REPO, "tools"))
import bvh_bound_probe  # noqa: E402


def test_margin_bound_holds_on_adversarial_pairs():
    worst, hits, total = bvh_bound_probe.run(n_batches=2, batch=500_000, seed=3)
    assert hits > 20_000  # the sample reports hits, grazing ones included
    assert worst < 1.0, worst  # every reported hit lies within mu of its triangle
    assert worst < 0.25  # (slack: the analysis is a worst case)


def test_margin_bound_on_grazing_pairs_only():
    rng = np.random.default_rng(99)
    O, D, p0, e1, e2 = bvh_bound_probe.sample(rng, 400_000)
    nrm = np.cross(e1.astype(np.float64), e2.astype(np.float64))
    nrm /= np.linalg.norm(nrm, axis=1, keepdims=True)
    a = np.abs(np.einsum("ij,ij->i", D.astype(np.float64), nrm))
    g = a < 1e-2
    ok, t = bvh_bound_probe.ref_test(O[g], D[g], p0[g], e1[g], e2[g])
    ok &= np.isfinite(t)
    assert ok.sum() > 100
    Og, Dg, pg, e1g, e2g, tg = O[g][ok], D[g][ok], p0[g][ok], e1[g][ok], e2[g][ok], t[ok]
    X = Og.astype(np.float64) + tg.astype(np.float64)[:, None] * Dg.astype(np.float64)
    base = pg.astype(np.float64)
    d = bvh_bound_probe.point_tri_dist(X, base, base + e1g.astype(np.float64), base + e2g.astype(np.float64))
    mu = bvh_bound_probe.margin(Og, Dg, pg, e1g, e2g)
    assert np.all(d <= mu)


def test_oracle_matches_reference_reflective_heightfield(oracle, heightfield_r05_path):
    with np.load(os.path.join(GOLDEN, "hf_reflect.npz")) as z:
        for k in ("hfr_1920x1080_d3_win_400_408_944_976", "hfr_1920x1080_d6_win_480_488_1500_1532"):
            w, h = map(int, k.split("_")[1].split("x"))
            d = int(k.split("_")[2][1:])
            r0, r1, c0, c1 = map(int, k.rsplit("_win_", 1)[1].split("_"))
            got = oracle.render(heightfield_r05_path, w, h, d, window=(r0, r1, c0, c1), threads=8)
            assert bits_equal(got, z[k]), k
        # the mirrors change the picture: the same window of the plain mesh differs
        with np.load(os.path.join(GOLDEN, "c3_column.npz")) as p:
            assert not np.array_equal(p["hf_1080p_d1_win_400_408_944_976"], z["hfr_1920x1080_d1_win_400_408_944_976"])


# ---- the host build's depth bound: every tree fits the walk's
# 24-entry stack, whatever the triangle distribution
def _build(tri):
    import ctypes

    import rt_amd

    L = rt_amd.lib()
    L.rt_debug_bvh_build.argtypes = [ctypes.c_void_p, ctypes.c_longlong, ctypes.c_void_p]
    tri = np.ascontiguousarray(tri, np.float32)
    out = np.zeros(3, np.int32)
    rc = L.rt_debug_bvh_build(tri.ctypes.data, tri.shape[0], out.ctypes.data)
    return rc, out


def _tris(p0, size):
    n = p0.shape[0]
    t = np.zeros((n, 12), np.float32)
    t[:, 0:3] = p0
    t[:, 3] = size
    t[:, 7] = size
    t[:, 11] = 1.0
    return t


@pytest.mark.parametrize("kind", ["grid", "geometric", "clustered"])
def test_bvh_depth_fits_the_stack_on_big_meshes(kind):
    n = 1_200_000
    rng = np.random.default_rng(5)
    if kind == "grid":
        k = np.arange(n)
        p0 = np.stack([(k % 1000).astype(np.float32), np.zeros(n, np.float32), (k // 1000).astype(np.float32)], 1)
        size = np.ones(n, np.float32)
    elif kind == "geometric":
        # centroids spread over ~34 decades: SAH's 16 bins over the widest
        # extent split off a few triangles per level (the round-5 build
        # reached depth 20 with ~1M triangles left, then 38 levels)
        x = np.power(np.float64(1.00006), np.arange(n)).astype(np.float32)
        p0 = np.stack([x, np.zeros(n, np.float32), np.zeros(n, np.float32)], 1)
        size = np.maximum(x * np.float32(1e-3), np.float32(1e-3))
    else:
        c = rng.integers(0, 8, n)
        p0 = (rng.normal(size=(n, 3)) * np.power(10.0, c)[:, None]).astype(np.float32)
        size = np.power(10.0, c - 3).astype(np.float32)
    rc, (depth, inner, leaves) = _build(_tris(p0, size))
    assert rc == 0
    assert 1 <= depth <= 24, depth
    assert leaves == inner + 1
    assert leaves >= n // 4


def test_bvh_build_refuses_what_the_leaf_encoding_cannot_hold():
    import ctypes

    import rt_amd

    L = rt_amd.lib()
    L.rt_debug_bvh_build.argtypes = [ctypes.c_void_p, ctypes.c_longlong, ctypes.c_void_p]
    out = np.zeros(3, np.int32)
    dummy = np.zeros(12, np.float32)
    # (the size check comes before any read of the triangles)
    assert L.rt_debug_bvh_build(dummy.ctypes.data, (4 << 24) + 1, out.ctypes.data) == -6
    assert L.rt_debug_bvh_build(dummy.ctypes.data, 4, out.ctypes.data) == -1
