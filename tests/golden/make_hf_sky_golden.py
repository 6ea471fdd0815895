"""Golden windows of the 50k-triangle heightfield WITHOUT its ground plane
(sky around the mesh) at 1920x1080, depth 1, from oracle/_ref (the
reference's own code; see make_golden.py).  Run in the build container:

    make -C oracle ref && python tests/golden/make_hf_sky_golden.py

The mesh's silhouette puts waves whose lanes partly miss everything next to
waves of shadowed mesh: the big-list kernel's light-buffer and camera-list
walks then run on partial waves.  Windows of 16 rows x 32 columns on a
9 x 8 grid over the frame, and runs of them across the silhouette.  Output: tests/golden/hf_sky.npz (float32 RGB per
window; data only)."""
from __future__ import annotations

import os
import sys
import time
from multiprocessing import Pool

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

import make_golden  # noqa: E402

W, H, DEPTH = 1920, 1080, 1
PATH = os.path.join("/tmp", "rt_amd_heightfield_sky.dat")


def sky_dat() -> str:
    """The heightfield scene text with the Plane block dropped."""
    lines = make_golden.synth.heightfield_dat().split("\n")
    i = lines.index("Plane: plane_1")
    j = i + 1
    while j < len(lines) and lines[j].startswith(" "):
        j += 1
    return "\n".join(lines[:i] + lines[j:])


def windows():
    grid = [(r, r + 16, c, c + 32) for r in range(0, 1065, 133) for c in range(0, 1889, 269)]
    # the silhouette: the mesh's near and far edges down the middle column,
    # its left and right edges across the middle rows
    edges = [(r, r + 16, 944, 976) for r in range(128, 305, 16)]
    edges += [(r, r + 16, 944, 976) for r in range(608, 817, 16)]
    edges += [(400, 416, c, c + 32) for c in list(range(0, 321, 32)) + list(range(1568, 1889, 32))]
    return grid + edges


def render(win):
    L = make_golden.load_ref()
    ref = make_golden.Ref(L, PATH, W, H, DEPTH)
    return win, ref.window(*win)


def main():
    with open(PATH, "w") as f:
        f.write(sky_dat())
    t0 = time.time()
    with Pool(min(8, os.cpu_count() or 1)) as p:
        res = p.map(render, windows(), chunksize=1)
    out = {f"hfsky_1080p_d1_win_{r0}_{r1}_{c0}_{c1}": img for (r0, r1, c0, c1), img in res}
    np.savez_compressed(os.path.join(HERE, "hf_sky.npz"), **out)
    print(f"wrote {len(out)} windows in {time.time() - t0:.1f} s")


if __name__ == "__main__":
    main()
