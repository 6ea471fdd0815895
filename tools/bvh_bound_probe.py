"""Empirical check of the bounce-ray BVH's margin bound (DESIGN.md §3
"Bounce rays: BVH").

The reference's f32 Moller-Trumbore test (Triangle.cpp:127-172) can report a
hit whose exact point O + t~ D lies off the triangle: for a reported hit
(|det~| >= 0.01, u~ in [0, 1], v~ >= 0, fl(u~ + v~) <= 1),

    dist(O + t~ D, T) <= mu = eps (40 K + 4) |S| + 16 eps L,
    K = 1.01 |e1||e2| / (0.01 - 6.1 eps 1.01 |e1||e2|),  S = O - p0,
    L = max(|e1|, |e2|), eps = 2^-24

(first-order forward error analysis, rt_bvh.h: the relative error of det~
is common to u~, v~ and t~ and moves the point by r |S| since
t D - u e1 - v e2 = -S exactly; the numerators' errors give 20.5 eps K |S|;
the products' roundings 2 eps (|S| + 4 L); in all 26.3 eps K |S| + 2 eps |S|
+ 9 eps L, with a 1.5x safety factor).  This script samples
adversarial ray-triangle pairs — near-grazing rays (|cos| down to 1e-6),
slivers, long edges, far origins — evaluates the reference test in float32
with the reference's operation order, and reports the largest ratio
dist / mu over the reported hits.  tests/test_bvh_bound.py runs a smaller
sample of the same generator.
"""
from __future__ import annotations

import numpy as np

EPS = 2.0 ** -24


def ref_test(O, D, p0, e1, e2):
    """Triangle.cpp:127-172 in float32, the reference's operation order
    (numpy float32 ops round each result; no FMA)."""
    f = np.float32
    O, D, p0, e1, e2 = (np.asarray(a, f) for a in (O, D, p0, e1, e2))
    Px = D[:, 1] * e2[:, 2] - D[:, 2] * e2[:, 1]
    Py = D[:, 2] * e2[:, 0] - D[:, 0] * e2[:, 2]
    Pz = D[:, 0] * e2[:, 1] - D[:, 1] * e2[:, 0]
    det = e1[:, 0] * Px + e1[:, 1] * Py + e1[:, 2] * Pz
    with np.errstate(all="ignore"):
        inv = f(1.0) / det
        S = O - p0
        u = (S[:, 0] * Px + S[:, 1] * Py + S[:, 2] * Pz) * inv
        Qx = S[:, 1] * e1[:, 2] - S[:, 2] * e1[:, 1]
        Qy = S[:, 2] * e1[:, 0] - S[:, 0] * e1[:, 2]
        Qz = S[:, 0] * e1[:, 1] - S[:, 1] * e1[:, 0]
        v = (D[:, 0] * Qx + D[:, 1] * Qy + D[:, 2] * Qz) * inv
        t = (e2[:, 0] * Qx + e2[:, 1] * Qy + e2[:, 2] * Qz) * inv
        ok = ~(np.abs(det) < f(0.01)) & ~((u < 0) | (u > 1)) & ~((v < 0) | ((u + v) > 1))
    return ok, t


def point_tri_dist(X, a, b, c):
    """Distance from points X to triangles (a, b, c), float64, vectorised
    (Ericson's closest-point by Voronoi regions)."""
    ab, ac, ap = b - a, c - a, X - a
    d1 = np.einsum("ij,ij->i", ab, ap)
    d2 = np.einsum("ij,ij->i", ac, ap)
    bp = X - b
    d3 = np.einsum("ij,ij->i", ab, bp)
    d4 = np.einsum("ij,ij->i", ac, bp)
    cp = X - c
    d5 = np.einsum("ij,ij->i", ab, cp)
    d6 = np.einsum("ij,ij->i", ac, cp)
    va = d3 * d6 - d5 * d4
    vb = d5 * d2 - d1 * d6
    vc = d1 * d4 - d3 * d2
    with np.errstate(all="ignore"):
        den = 1.0 / (va + vb + vc)
        s_in, t_in = vb * den, vc * den
        cl = a + s_in[:, None] * ab + t_in[:, None] * ac
        r1 = (d1 <= 0) & (d2 <= 0)
        r2 = (d3 >= 0) & (d4 <= d3)
        r3 = (vc <= 0) & (d1 >= 0) & (d3 <= 0)
        r4 = (d6 >= 0) & (d5 <= d6)
        r5 = (vb <= 0) & (d2 >= 0) & (d6 <= 0)
        r6 = (va <= 0) & ((d4 - d3) >= 0) & ((d5 - d6) >= 0)
        w3 = d1 / (d1 - d3)
        w5 = d2 / (d2 - d6)
        w6 = (d4 - d3) / ((d4 - d3) + (d5 - d6))
    cl = np.where(r6[:, None], b + w6[:, None] * (c - b), cl)
    cl = np.where(r5[:, None], a + w5[:, None] * ac, cl)
    cl = np.where(r4[:, None], c, cl)
    cl = np.where(r3[:, None], a + w3[:, None] * ab, cl)
    cl = np.where(r2[:, None], b, cl)
    cl = np.where(r1[:, None], a, cl)
    return np.linalg.norm(X - cl, axis=1)


def margin(O, D, p0, e1, e2):
    n1 = np.linalg.norm(e1.astype(np.float64), axis=1)
    n2 = np.linalg.norm(e2.astype(np.float64), axis=1)
    prod = n1 * n2
    den = 0.01 - 6.1 * EPS * 1.01 * prod
    K = np.where(den > 0.001, 1.01 * prod / np.maximum(den, 1e-30), np.inf)
    S = np.linalg.norm(O.astype(np.float64) - p0.astype(np.float64), axis=1)
    L = np.maximum(n1, n2)
    return EPS * (40.0 * K + 4.0) * S + 16.0 * EPS * L


def sample(rng, n):
    """Adversarial pairs: the ray aimed at a point near the triangle from a
    random distance, at angles down to 1e-6 rad above the plane."""
    f = np.float32
    p0 = rng.uniform(-200, 200, (n, 3))
    scale = np.exp(rng.uniform(np.log(0.02), np.log(60.0), (n, 1)))
    e1 = rng.normal(size=(n, 3)) * scale
    # slivers and near-degenerate shapes for a third of the pairs
    sl = rng.random(n) < 0.33
    e2 = rng.normal(size=(n, 3)) * scale
    e2[sl] = e1[sl] * rng.uniform(0.2, 1.2, (sl.sum(), 1)) + rng.normal(size=(sl.sum(), 3)) * scale[sl] * 1e-2
    p0, e1, e2 = p0.astype(f), e1.astype(f), e2.astype(f)
    nrm = np.cross(e1.astype(np.float64), e2.astype(np.float64))
    nn = np.linalg.norm(nrm, axis=1, keepdims=True)
    nrm = nrm / np.maximum(nn, 1e-30)
    bu = rng.uniform(-0.3, 1.3, n)
    bv = rng.uniform(-0.3, 1.3, n)
    X = p0 + bu[:, None] * e1 + bv[:, None] * e2
    # in-plane direction and elevation angle
    w = rng.normal(size=(n, 3))
    w -= np.einsum("ij,ij->i", w, nrm)[:, None] * nrm
    w /= np.maximum(np.linalg.norm(w, axis=1, keepdims=True), 1e-30)
    elev = np.exp(rng.uniform(np.log(1e-6), np.log(1.5), n))
    side = np.where(rng.random(n) < 0.5, 1.0, -1.0)
    dirn = np.cos(elev)[:, None] * w + (side * np.sin(elev))[:, None] * nrm
    dist = np.exp(rng.uniform(np.log(0.5), np.log(1500.0), n))
    O = (X + dist[:, None] * dirn).astype(f)
    # D = Normaliser(X - O) in float32 (v * (1 / len))
    v = (X.astype(f) - O).astype(f)
    ln = np.sqrt((v[:, 0] * v[:, 0] + v[:, 1] * v[:, 1] + v[:, 2] * v[:, 2]).astype(f)).astype(f)
    with np.errstate(all="ignore"):
        D = (v * (f(1.0) / ln)[:, None]).astype(f)
    keep = np.isfinite(D).all(axis=1) & (ln > 0.01)
    return O[keep], D[keep], p0[keep], e1[keep], e2[keep]


def run(n_batches=10, batch=1_000_000, seed=7):
    rng = np.random.default_rng(seed)
    worst, hits, total = 0.0, 0, 0
    for _ in range(n_batches):
        O, D, p0, e1, e2 = sample(rng, batch)
        ok, t = ref_test(O, D, p0, e1, e2)
        ok &= np.isfinite(t)
        total += len(O)
        if not ok.any():
            continue
        O, D, p0, e1, e2, t = O[ok], D[ok], p0[ok], e1[ok], e2[ok], t[ok]
        X = O.astype(np.float64) + t.astype(np.float64)[:, None] * D.astype(np.float64)
        a = p0.astype(np.float64)
        d = point_tri_dist(X, a, a + e1.astype(np.float64), a + e2.astype(np.float64))
        mu = margin(O, D, p0, e1, e2)
        r = d / mu
        worst = max(worst, float(np.max(r)))
        hits += int(ok.sum())
    return worst, hits, total


if __name__ == "__main__":
    import sys

    nb = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    w, h, tot = run(nb)
    print(f"pairs {tot}, reported hits {h}, max dist / mu = {w:.4f}")
