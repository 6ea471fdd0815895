"""Golden windows of the REFLECTIVE heightfield — the 50k-triangle mesh of
rt_amd.synth with `reflect: 0.5` on every triangle (SURVEY.md §8(d) C5's
"--reflect 0.5" variant; bench configs c3r / c5r) — from oracle/_ref, the
reference's own code with the commented reflect/refract block re-enabled
(see make_golden.py).  Every bounce ray of these frames is traced by the
reference through all 50,001 surfaces (Scene.cpp:1705-1715), which the
product replaces by the BVH walk (rt_bvh.h).  Run in the build container:

    make -C oracle ref && python tests/golden/make_hf_reflect_golden.py

Windows (8 rows x 32 columns, bottom row first like m_InfoPixel):
* 1920x1080 depth 3: every 40th row from 0 to 1072 at column 944 (mesh,
  ground plane, horizon, sky), every 120th row at both frame edges, and a
  row of 8 windows across the mesh at row 400;
* 1920x1080 depths 1 and 6 (the deepest level reflect 0.5 reaches with the
  reference's 0.01 energy floor): 6 windows on the mesh;
* 7680x4320 depth 3 (c5r): 12 windows down column 3776 and across row 1600.
Output: tests/golden/hf_reflect.npz (float32 RGB per window; data only)."""
from __future__ import annotations

import os
import sys
import time
from multiprocessing import Pool

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

import make_golden  # noqa: E402

HF = os.path.join("/tmp", "rt_amd_heightfield_r05.dat")


def jobs():
    out = []
    for r in range(0, 1073, 40):
        out.append((1920, 1080, 3, (r, r + 8, 944, 976)))
    for r in range(0, 1073, 120):
        for c in (0, 1888):
            out.append((1920, 1080, 3, (r, r + 8, c, c + 32)))
    for c in range(64, 1900, 240):
        out.append((1920, 1080, 3, (400, 408, c, c + 32)))
    for d in (1, 6):
        for r, c in ((200, 300), (400, 944), (480, 1500), (560, 100), (640, 960), (700, 1200)):
            out.append((1920, 1080, d, (r, r + 8, c, c + 32)))
    for r in range(0, 4313, 480):
        out.append((7680, 4320, 3, (r, r + 8, 3776, 3808)))
    for c in (640, 7000):
        out.append((7680, 4320, 3, (1600, 1608, c, c + 32)))
    return out


def render(job):
    w, h, d, win = job
    L = make_golden.load_ref()
    ref = make_golden.Ref(L, HF, w, h, d)
    return job, ref.window(*win)


def key(w, h, d, win):
    r0, r1, c0, c1 = win
    return f"hfr_{w}x{h}_d{d}_win_{r0}_{r1}_{c0}_{c1}"


def main():
    make_golden.synth.write_heightfield(HF, reflect=0.5)
    t0 = time.time()
    with Pool(min(8, os.cpu_count() or 1)) as p:
        res = p.map(render, jobs(), chunksize=1)
    out = {key(w, h, d, win): img for (w, h, d, win), img in res}
    np.savez_compressed(os.path.join(HERE, "hf_reflect.npz"), **out)
    print(f"wrote {len(out)} windows in {time.time() - t0:.1f} s")


if __name__ == "__main__":
    main()
