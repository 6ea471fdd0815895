"""Scenes built to break bounding-cone culling (test input generator).

Every triangle family here puts an apex the kernel culls from — the camera
or a light — in or near the triangle's plane, or makes the reference's f32
triangle test badly conditioned (slivers, tiny and very large triangles,
far lights), so the GPU's culled loops must still return the reference's
exact hits (rt_cone_prepass's rounding argument).  Written in the
reference's .dat format with %.3f coordinates (lines <= 78 characters).
"""
from __future__ import annotations

import numpy as np

CAMERA = np.array([0.0, 8.0, 70.0])
LIGHTS = [(np.array([40.0, 80.0, 50.0]), 0.5), (np.array([-30.0, 5.0, 10.0]), 0.4),
          (np.array([1000.0, 3000.0, -2000.0]), 0.3)]


def _unit(v):
    return v / np.linalg.norm(v)


def cull_stress_dat(seed: int, reflect: float = 0.0, n_small: int = 40) -> str:
    rng = np.random.default_rng(seed)
    camera, lights = CAMERA, LIGHTS
    if seed >= 100:  # randomised viewpoint and lights (tests/test_cull_stress.py vs the oracle)
        camera = rng.uniform([-80, -10, 20], [80, 90, 120])
        lights = [(rng.uniform([-150, -15, -150], [150, 300, 150]), 0.5),
                  (rng.uniform([-60, -15, -60], [60, 60, 60]), 0.4),
                  (rng.normal(size=3) * 3000.0, 0.3)]
    out = ["* cull stress scene (tests/cull_scenes.py)", "        background: 0 0 150",
           "        origin: %.3f %.3f %.3f" % tuple(camera), "        eye: 0.0 0.0 0.0", "        up:  0.0 1.0 0.0"]
    for i, (p, inten) in enumerate(lights):
        out += [f"Lumiere: l{i}", "        position: %.3f %.3f %.3f" % tuple(p), f"        intens: {inten}"]
    out += ["Plane: ground", "        v_linear: 0.0 1.0 0.0", "        v_const:  20.0",
            "        color:   10 255 11", "        ambient: 0.3", "        diffus:  0.7"]
    tris = []

    def edge_on(apex, n, size):
        for _ in range(n):
            q = rng.uniform([-30, -15, -30], [30, 20, 10])
            a = _unit(apex - q)
            w = _unit(np.cross(a, rng.normal(size=3)))
            s = size * rng.uniform(0.2, 1.0)
            # vertices in the plane through the apex spanned by a and w
            pts = [q + s * (x * a + y * w) for x, y in rng.uniform(-1, 1, (3, 2))]
            tris.append(pts)

    edge_on(camera, 30, 12.0)
    for p, _ in lights[:2]:
        edge_on(p, 25, 12.0)
    for _ in range(12):  # large triangles (longest edge up to ~400: never culled past 110)
        c = rng.uniform([-60, -20, -150], [60, 40, -40])
        tris.append([c + rng.normal(size=3) * rng.uniform(30, 160) for _ in range(3)])
    for _ in range(n_small):  # small ones (> 1,024 triangles in all: the clustered culling)
        c = rng.uniform([-30, -15, -30], [30, 25, 20])
        tris.append([c + rng.normal(size=3) * rng.uniform(0.05, 4.0) for _ in range(3)])
    for _ in range(12):  # slivers
        c = rng.uniform([-30, -15, -30], [30, 25, 20])
        d = _unit(rng.normal(size=3)) * rng.uniform(5, 30)
        e = _unit(rng.normal(size=3)) * rng.uniform(0.005, 0.05)
        tris.append([c, c + d, c + d * 0.5 + e])
    for k, pts in enumerate(tris):
        out.append(f"Poly: t{k}")
        for j, p in enumerate(pts):
            out.append("        point: %d %.3f %.3f %.3f" % (j, p[0], p[1], p[2]))
        out.append("        color:  %d %d %d" % tuple(rng.integers(20, 255, 3)))
        if reflect and k % 3 == 0:
            out.append(f"        reflect: {reflect}")
    text = "\n".join(out) + "\n"
    assert max(len(l) for l in text.split("\n")) <= 78
    return text


def write(path, seed: int, reflect: float = 0.0, n_small: int = 40) -> str:
    with open(path, "w") as f:
        f.write(cull_stress_dat(seed, reflect, n_small))
    return path


# seeds >= 10: big lists (two-level culling, Morton-ordered triangles)
def n_small_for(seed: int) -> int:
    return 1500 if seed >= 10 else 40
