"""Reference fixtures for moved cameras and for the big bounce frames, made
by oracle/_ref (the reference's own primitive, Pretraitement, vector and
colour sources + the CScene harness, see make_golden.py).  Run in the build
container:

    make -C oracle ref && python tests/golden/make_camera_golden.py

* Moved cameras: every frame of tests/cameras.py's sets — the reference
  camera turned / moved / widened (`cameras`) and a 6-frame camera path
  (`path`) — on scene2 (depth 0), scene7 (depth 3: reflect + refract) and the
  50k-triangle heightfield (depth 0) at 480x270.  The harness takes the
  frame's camera words explicitly (ref_set_camera: position, orientation,
  half extents, pixel reciprocals — what rt_frame carries), then runs the
  reference pixel loop (Scene.cpp:1538-1561) over the whole frame.
* Big bounce frames: scene7 and scene9 at 3840x2160, depth 5, whole frame.
* Moved C3 frames at full size: frames 3 and 6 of tests/cameras.py
  moving() (the bench's translated camera) on the heightfield at 1920x1080.

Output: tests/golden/cameras.json — per frame the SHA-256 of its camera
words (tests/cameras.py words()), of the float32 RGB frame (row 0 = bottom)
and of its RGBA8 quantisation, and the float64 sum of the RGB.  Data only.
"""
from __future__ import annotations

import ctypes
import json
import os
import sys
import time
from multiprocessing import Pool

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.dirname(HERE))

import make_golden  # noqa: E402
from make_golden import rgba8, sha  # noqa: E402

import cameras  # noqa: E402
import rt_amd  # noqa: E402

REPO_SCENES = os.path.join(HERE, "scenes")
HF = os.path.join("/tmp", "rt_amd_heightfield.dat")
BAND = 30  # rows per task


def scene_path(name):
    return HF if name == "hf" else os.path.join(REPO_SCENES, f"{name}.dat")


def frames_of(name, w, h, depth, kind):
    s = rt_amd.Scene(scene_path(name), w, h, depth)
    return cameras.KINDS[kind](s.frame)


def render_band(task):
    name, w, h, depth, words, r0, r1 = task
    L = make_golden.load_ref()
    L.ref_set_camera.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p] + [ctypes.c_float] * 4 + \
                                [ctypes.c_int, ctypes.c_int]
    ref = make_golden.Ref(L, scene_path(name), w, h, depth)
    if words is not None:
        pos = np.asarray(words[:3], np.float32)
        orient = np.asarray(words[3:19], np.float32)
        assert L.ref_set_camera(ref.p, pos.ctypes.data, orient.ctypes.data, *words[19:23], w, h) == 0
    return ref.window(r0, r1, 0, w)


def entry(img, words_sha=None):
    e = {"rgb_f32_sha256": sha(img), "rgba8_sha256": sha(rgba8(img)), "rgb_sum": float(img.astype(np.float64).sum())}
    if words_sha:
        e["camera_words_sha256"] = words_sha
    return e


def main():
    make_golden.synth.write_heightfield(HF)
    path = os.path.join(HERE, "cameras.json")
    out = json.load(open(path)) if os.path.exists(path) else {}  # only missing frames are rendered
    jobs = []  # (key, words_sha, w, h, tasks)
    for key, name, w, h, depth in cameras.SETS:
        for kind in cameras.KINDS:
            for i, f in enumerate(frames_of(name, w, h, depth, kind)):
                if cameras.key(key, kind, i) in out:
                    assert out[cameras.key(key, kind, i)]["camera_words_sha256"] == cameras.words_sha(f)
                    continue
                words = [float(x) for x in cameras.words(f)]
                tasks = [(name, w, h, depth, words, r, min(h, r + BAND)) for r in range(0, h, BAND)]
                jobs.append((cameras.key(key, kind, i), cameras.words_sha(f), w, h, tasks))
    for name in ("scene7", "scene9"):
        w, h = 3840, 2160
        if f"{name}_{w}x{h}_d5_full" in out:
            continue
        tasks = [(name, w, h, 5, None, r, min(h, r + 120)) for r in range(0, h, 120)]
        jobs.append((f"{name}_{w}x{h}_d5_full", None, w, h, tasks))
    name, w, h, depth, idx = cameras.MOVING_FULL  # full-size moved C3 frames
    mv = cameras.moving(rt_amd.Scene(scene_path(name), w, h, depth).frame, max(idx) + 1)
    for i in idx:
        k = f"{name}_{w}x{h}_d{depth}_moving{i}"
        if k in out:
            assert out[k]["camera_words_sha256"] == cameras.words_sha(mv[i])
            continue
        words = [float(x) for x in cameras.words(mv[i])]
        tasks = [(name, w, h, depth, words, r, min(h, r + BAND)) for r in range(0, h, BAND)]
        jobs.append((k, cameras.words_sha(mv[i]), w, h, tasks))
    flat = [t for j in jobs for t in j[4]]
    t0 = time.time()
    with Pool(int(os.environ.get("GOLDEN_PROCS", min(8, os.cpu_count() or 1)))) as p:
        bands = p.map(render_band, flat, chunksize=1)
    k = 0
    for key, wsha, w, h, tasks in jobs:
        img = np.concatenate(bands[k:k + len(tasks)], 0)
        k += len(tasks)
        assert img.shape == (h, w, 3)
        out[key] = entry(img, wsha)
    with open(path, "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)
    print(f"wrote {len(out)} frames in {time.time() - t0:.1f} s")


if __name__ == "__main__":
    main()
