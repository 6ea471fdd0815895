"""Golden post-Pretraitement state of the crafted quirk files
(tests/loader_quirks.py) from oracle/_ref — the loader restated on the
reference's own CMatrice4 / CCouleur / CVecteur3 and its Pretraitement
(Triangle.cpp, Plan.cpp, Quadrique.cpp).  Run in the build container:

    make -C oracle ref && python tests/golden/make_loader_golden.py

Output: tests/golden/loader_quirks.npz — per file, <name>_surf (n x 24),
<name>_cam (27) and <name>_lights (n x 7) in oracle_dump's layout."""
from __future__ import annotations

import os
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.dirname(HERE))

import make_golden  # noqa: E402
from loader_quirks import QUIRK_RES, QUIRKS  # noqa: E402


def main():
    L = make_golden.load_ref()
    out = {}
    with tempfile.TemporaryDirectory() as d:
        for name, text in sorted(QUIRKS.items()):
            p = os.path.join(d, name + ".dat")
            with open(p, "wb") as f:
                f.write(text.encode())
            s, c, l = make_golden.Ref(L, p, *QUIRK_RES, 0).dump()
            out[f"{name}_surf"], out[f"{name}_cam"], out[f"{name}_lights"] = s, c, l
            print(name, s.shape[0], "surfaces", l.shape[0], "lights")
    np.savez_compressed(os.path.join(HERE, "loader_quirks.npz"), **out)


if __name__ == "__main__":
    main()
