"""Golden windows of C3 — the 50k-triangle heightfield (rt_amd.synth) at
1920x1080, depth 1 — down the whole frame height, from oracle/_ref (the
reference's own code; see make_golden.py).  Run in the build container:

    make -C oracle ref && python tests/golden/make_c3_column_golden.py

Windows (8 rows x 32 columns, bottom row first like m_InfoPixel): every
40th row from 0 to 1072 at column 944 (mesh, ground plane, the horizon and
the sky: tiles whose lanes partly miss everything, which is where the
light-buffer walks run on partial waves), and every 120th row at both frame
edges.  Output: tests/golden/c3_column.npz (float32 RGB per window; data
only)."""
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
HF = os.path.join("/tmp", "rt_amd_heightfield.dat")


def windows():
    out = [(r, r + 8, 944, 976) for r in range(0, 1073, 40)]
    out += [(r, r + 8, c, c + 32) for r in range(0, 1073, 120) for c in (0, 1888)]
    return out


def render(win):
    L = make_golden.load_ref()
    ref = make_golden.Ref(L, HF, W, H, DEPTH)
    return win, ref.window(*win)


def main():
    make_golden.synth.write_heightfield(HF)
    t0 = time.time()
    with Pool(min(8, os.cpu_count() or 1)) as p:
        res = p.map(render, windows(), chunksize=1)
    out = {f"hf_1080p_d1_win_{r0}_{r1}_{c0}_{c1}": img for (r0, r1, c0, c1), img in res}
    np.savez_compressed(os.path.join(HERE, "c3_column.npz"), **out)
    print(f"wrote {len(out)} windows in {time.time() - t0:.1f} s")


if __name__ == "__main__":
    main()
