"""Reference fixtures for two BASELINE.json configs at their full size, made
by oracle/_ref (the reference's own primitive sources + the CScene harness,
see make_golden.py).  Run in the build container:

    make -C oracle ref && python tests/golden/make_config_golden.py

Outputs (data only):
  c1.npz        C1 = Scenes/scene1 at 512x512, max bounces 1: the whole
                float32 RGB frame (m_InfoPixel, row 0 = bottom).
  configs.json  C4 = Scenes/scene2 at 3840x2160, max bounces 5: SHA-256 of
                the float32 RGB frame and of its RGBA8 quantisation, and the
                float64 sum of the RGB (the frame is 100 MB, too large to keep).
                C1's digests too.
"""
from __future__ import annotations

import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

from make_golden import SCENES, Ref, load_ref, rgba8, sha  # noqa: E402


def main():
    L = load_ref()
    out = {}
    c1 = Ref(L, f"{SCENES}/scene1.dat", 512, 512, 1).window(0, 512, 0, 512)
    np.savez_compressed(os.path.join(HERE, "c1.npz"), scene1_512x512_d1=c1)
    out["scene1_512x512_d1_rgb_f32_sha256"] = sha(c1)
    out["scene1_512x512_d1_rgba8_sha256"] = sha(rgba8(c1))
    print("C1 done", flush=True)
    c4 = Ref(L, f"{SCENES}/scene2.dat", 3840, 2160, 5).window(0, 2160, 0, 3840)
    out["scene2_3840x2160_d5_rgb_f32_sha256"] = sha(c4)
    out["scene2_3840x2160_d5_rgba8_sha256"] = sha(rgba8(c4))
    out["scene2_3840x2160_d5_rgb_sum"] = float(c4.astype(np.float64).sum())
    with open(os.path.join(HERE, "configs.json"), "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
