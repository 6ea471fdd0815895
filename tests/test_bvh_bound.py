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
