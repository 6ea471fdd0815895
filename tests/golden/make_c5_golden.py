"""Golden windows of C5 — the 50k-triangle heightfield (rt_amd.synth) at
7680x4320, depth 3 — from oracle/_ref (the reference's own primitive,
Pretraitement, vector and colour code; see make_golden.py).  Run in the
build container:

    make -C oracle ref && python tests/golden/make_c5_golden.py

Windows (16 rows x 32 columns, bottom row first like m_InfoPixel):
  * rows 536, 1080, 1624, 2168, 2712, 3256, 3800 (each starts 8 rows into a
    16-row band, so it straddles a cyclic-band boundary; together they
    straddle every 8-way slab boundary of the frame, 540 k for equal slabs
    and 544 k for rt_amd.dist.slab_rows' 8-row multiples), plus the bottom
    and top rows of the frame;
  * columns 0, 1912, 3832, 5752, 7648 (both frame edges).
Output: tests/golden/c5.npz (float32 RGB per window; data only)."""
from __future__ import annotations

import os
import sys
import time
from multiprocessing import Pool

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

import make_golden  # noqa: E402

W, H, DEPTH = 7680, 4320, 3
ROWS = [0, 536, 1080, 1624, 2168, 2712, 3256, 3800, 4304]
COLS = [0, 1912, 3832, 5752, 7648]
HF = os.path.join("/tmp", "rt_amd_heightfield.dat")


def windows():
    return [(r, r + 16, c, c + 32) for r in ROWS for c in COLS]


def render(win):
    L = make_golden.load_ref()
    ref = make_golden.Ref(L, HF, W, H, DEPTH)
    return win, ref.window(*win)


def main():
    make_golden.synth.write_heightfield(HF)
    t0 = time.time()
    with Pool(min(8, os.cpu_count() or 1)) as p:
        res = p.map(render, windows(), chunksize=1)
    out = {f"hf_4320p_d3_win_{r0}_{r1}_{c0}_{c1}": img for (r0, r1, c0, c1), img in res}
    np.savez_compressed(os.path.join(HERE, "c5.npz"), **out)
    print(f"wrote {len(out)} windows in {time.time() - t0:.1f} s")


if __name__ == "__main__":
    main()
