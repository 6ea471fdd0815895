"""Synthetic heightfield scene (BASELINE.json configs C3/C5).

250 x 100 cells x 2 = 50,000 triangles over x in [-150,150] (251 columns) and
z in [-200,0] (101 rows); heights y_ij = -20 + 15 * h(i,j) with
h = (splitmix64(0x5EED ^ (j*251 + i)) >> 40) / 2^24 — deterministic and
language-independent.  Colour 200 120 40, default material; the ground plane of
scene2; lights (100,400,360) I=0.7 and (-200,300,100) I=0.4; camera origin
(0,120,250), eye (0,0,-80), up (0,1,0).  Written as a reference-format .dat
with %.3f coordinates and every line <= 78 characters, so the reference's
getline(Line, 80) and our loader parse identical floats.
"""
from __future__ import annotations

import os

MASK = (1 << 64) - 1


def splitmix64(x: int) -> int:
    x = (x + 0x9E3779B97F4A7C15) & MASK
    z = x
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & MASK
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & MASK
    return z ^ (z >> 31)


def heightfield_dat(cols: int = 250, rows: int = 100, reflect: float = 0.0) -> str:
    nx, nz = cols + 1, rows + 1
    xs = [-150.0 + 300.0 * i / cols for i in range(nx)]
    zs = [-200.0 + 200.0 * j / rows for j in range(nz)]
    h = [[-20.0 + 15.0 * ((splitmix64(0x5EED ^ (j * nx + i)) >> 40) / float(1 << 24)) for i in range(nx)]
         for j in range(nz)]
    out = [
        "* synthetic heightfield (rt_amd.synth)",
        "        background: 0 0 150",
        "        origin: 0.0 120.0 250.0",
        "        eye: 0.0 0.0 -80.0",
        "        up:  0.0 1.0 0.0",
        "Lumiere: light_1",
        "        position: 100.0 400.0 360.0",
        "        intens:   0.7",
        "Lumiere: light_2",
        "        position: -200.0 300.0 100.0",
        "        intens:   0.4",
        "Plane: plane_1",
        "        v_linear: 0.0 1.0 0.0",
        "        v_const:  45.0",
        "        color:   10 255 11",
        "        ambient: 0.3",
        "        diffus:  0.7",
    ]

    def pt(k, i, j):
        return f"        point: {k} {xs[i]:.3f} {h[j][i]:.3f} {zs[j]:.3f}"

    n = 0
    for j in range(rows):
        for i in range(cols):
            # upward-facing normals: (v00, v01, v10) and (v11, v10, v01)
            for tri in (((i, j), (i, j + 1), (i + 1, j)), ((i + 1, j + 1), (i + 1, j), (i, j + 1))):
                out.append(f"Poly: t{n}")
                for k, (a, b) in enumerate(tri):
                    out.append(pt(k, a, b))
                out.append("        color:  200 120 40")
                if reflect:
                    out.append(f"        reflect: {reflect}")
                n += 1
    text = "\n".join(out) + "\n"
    assert max(len(l) for l in text.split("\n")) <= 78
    return text


def write_heightfield(path: str, cols: int = 250, rows: int = 100, reflect: float = 0.0) -> str:
    """Write the .dat once (idempotent: skipped if an identical file exists)."""
    text = heightfield_dat(cols, rows, reflect)
    if os.path.exists(path):
        with open(path) as f:
            if f.read() == text:
                return path
    tmp = path + ".tmp%d" % os.getpid()
    with open(tmp, "w") as f:
        f.write(text)
    os.replace(tmp, path)
    return path
