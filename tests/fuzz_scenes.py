"""Seeded random scenes in the reference's .dat format (test input
generator): a camera on a sphere around the origin, 0-4 lights, an optional
ground plane, triangles and quadrics (spheres, ellipsoids, cylinders, with
mixed terms) with random colours, some reflective, some refractive /
translucent (their colour filters shadow rays), some transformed (rotate /
translate / scale: the host's Pretraitement), and optionally Phong
specular.  %.3f numbers, lines <= 78 characters (Scene.cpp:231-501)."""
from __future__ import annotations

import numpy as np


def fuzz_dat(seed: int, specular: bool = False, big: bool = False) -> str:
    """big: 1,100-1,600 small triangles (above the 1,024 of the big-list
    kernel: clusters, the light-buffer ladder, the LDS-staged walks)."""
    rng = np.random.default_rng(seed)
    out = ["* fuzz scene (tests/fuzz_scenes.py)"]
    out.append("        background: %d %d %d" % tuple(rng.integers(0, 256, 3)))
    d = rng.normal(size=3)
    d[1] = abs(d[1]) + 0.2
    cam = d / np.linalg.norm(d) * rng.uniform(150, 250)
    out += ["        origin: %.3f %.3f %.3f" % tuple(cam), "        eye: 0.0 0.0 0.0", "        up:  0.0 1.0 0.0"]
    for i in range(int(rng.integers(0, 5))):
        p = rng.uniform([-200, 20, -200], [200, 300, 200])
        out += [f"Lumiere: l{i}", "        position: %.3f %.3f %.3f" % tuple(p),
                "        intens: %.3f" % rng.uniform(0.2, 0.9)]

    def material():
        m = ["        color: %d %d %d" % tuple(rng.integers(0, 256, 3))]
        if rng.random() < 0.5:
            m.append("        ambient: %.3f" % rng.uniform(0.1, 0.5))
            m.append("        diffus: %.3f" % rng.uniform(0.3, 0.9))
        if specular and rng.random() < 0.5:
            m.append("        specular: %.3f %.3f" % (rng.uniform(0.1, 0.8), rng.uniform(1.0, 40.0)))
        r = rng.random()
        if r < 0.25:
            m.append("        reflect: %.3f" % rng.uniform(0.2, 0.9))
        elif r < 0.45:
            m.append("        refract: %.3f %.3f" % (rng.uniform(0.2, 0.8), rng.uniform(1.05, 1.7)))
        return m

    def xform():
        x = []
        if rng.random() < 0.3:
            x.append("        rotate: %.3f %.3f %.3f" % tuple(rng.uniform(-90, 90, 3)))
        if rng.random() < 0.3:
            x.append("        translate: %.3f %.3f %.3f" % tuple(rng.uniform(-20, 20, 3)))
        if rng.random() < 0.2:
            x.append("        scale: %.3f %.3f %.3f" % tuple(rng.uniform(0.5, 1.5, 3)))
        return x

    if rng.random() < 0.7:
        out += ["Plane: ground", "        v_linear: 0.0 1.0 0.0", "        v_const:  %.3f" % rng.uniform(20, 60)]
        out += material()
    ntri, spread = (int(rng.integers(1100, 1600)), (1.5, 6.0)) if big else (int(rng.integers(1, 13)), (5, 30))
    for i in range(ntri):
        c = rng.uniform(-60, 60, 3)
        out.append(f"Poly: t{i}")
        for k in range(3):
            out.append("        point: %d %.3f %.3f %.3f" % ((k,) + tuple(c + rng.normal(size=3) * rng.uniform(*spread))))
        out += material() + xform()
    for i in range(int(rng.integers(0, 4))):
        c = rng.uniform(-50, 50, 3)
        kind = int(rng.integers(0, 3))
        r = rng.uniform(8, 30)
        if kind == 0:  # sphere
            q = np.array([1.0, 1.0, 1.0])
        elif kind == 1:  # ellipsoid
            q = 1.0 / rng.uniform(6, 30, 3) ** 2 * r * r
        else:  # cylinder along y
            q = np.array([1.0, 0.0, 1.0])
        lin = -2.0 * q * c
        const = float((q * c * c).sum() - r * r)
        out.append(f"Quad: q{i}")
        out.append("        v_quad: %.6f %.6f %.6f" % tuple(q))
        if rng.random() < 0.3:
            out.append("        v_mixte: %.6f %.6f %.6f" % tuple(rng.uniform(-0.05, 0.05, 3)))
        out.append("        v_linear: %.3f %.3f %.3f" % tuple(lin))
        out.append("        v_const: %.3f" % const)
        out += material() + xform()
    text = "\n".join(out) + "\n"
    assert max(len(l) for l in text.split("\n")) <= 78
    return text
