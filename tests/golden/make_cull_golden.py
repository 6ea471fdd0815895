"""Golden images of the cull-stress scenes (tests/cull_scenes.py) from
oracle/_ref — the reference's own Triangle/Plan/Lumiere/... sources, see
make_golden.py.  Run in the build container:

    make -C oracle ref && python tests/golden/make_cull_golden.py

Output: cull.npz — float32 RGB per (seed, depth) at 160x120 (seeds 0-3,
depth 0 with no reflections, depth 3 with reflect 0.3 on every third
triangle) and seed 0 at 640x480 depth 0; seeds 10 and 11 with 1,500 extra
small triangles (the two-level culling path).
"""
from __future__ import annotations

import os
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, HERE)

import cull_scenes  # noqa: E402
from make_golden import Ref, load_ref  # noqa: E402

CASES = ([(seed, 160, 120, d) for seed in range(4) for d in (0, 3)] + [(0, 640, 480, 0)] +
         [(seed, 160, 120, d) for seed in (10, 11) for d in (0, 3)])


def main():
    L = load_ref()
    out = {}
    with tempfile.TemporaryDirectory() as tmp:
        for seed, w, h, d in CASES:
            path = cull_scenes.write(os.path.join(tmp, f"cs{seed}_{d}.dat"), seed, 0.3 if d else 0.0,
                                     cull_scenes.n_small_for(seed))
            out[f"cs{seed}_{w}x{h}_d{d}"] = Ref(L, path, w, h, d).window(0, h, 0, w)
            print(seed, w, h, d, flush=True)
    np.savez_compressed(os.path.join(HERE, "cull.npz"), **out)


if __name__ == "__main__":
    main()
