"""Explicit cameras shared by the GPU tests and the fixture generator
(tests/golden/make_camera_golden.py), so both build the very same rt_frame
words: the reference's own camera (InitialiserCamera, Scene.cpp:624-660)
turned about its axes, moved and widened, and camera paths (yaw + move per
frame — the per-frame camera of a display loop, Main.cpp:229-250, that
LancerRayons recomputes at Scene.cpp:674).

The fixtures store, per frame, a SHA-256 of these words; a test whose frame
drifts from the generator's fails on that before comparing pixels."""
from __future__ import annotations

import hashlib

import numpy as np

import rt_amd


def rot(axis, deg):
    a = np.deg2rad(deg)
    c, s = np.cos(a), np.sin(a)
    i, j = [(1, 2), (2, 0), (0, 1)][axis]
    R = np.eye(3)
    R[i, i], R[i, j], R[j, i], R[j, j] = c, -s, s, c
    return R


def turned(frame, R, move=(0.0, 0.0, 0.0), fov_scale=1.0):
    """The camera rotated by R about its own axes (orientation rows U V N),
    moved, and its film widened by fov_scale."""
    f = frame.copy()
    o = np.array(frame.orient[:], np.float64).reshape(4, 4)
    o[:3, :3] = R @ o[:3, :3]
    for i, v in enumerate(o.astype(np.float32).ravel()):
        f.orient[i] = float(v)
    for i in range(3):
        f.cam_pos[i] += move[i]
    f.half_w *= fov_scale
    f.half_h *= fov_scale
    return f


def cameras(frame):
    """The reference camera, then moved / yawed / pitched / rolled / wide /
    backward-looking ones."""
    return [frame,
            turned(frame, rot(1, 7.0), (3.0, 0.5, -2.0)),
            turned(frame, rot(0, -11.0) @ rot(1, 23.0), (-4.0, 1.0, 2.0)),
            turned(frame, rot(2, 35.0)),                          # roll
            turned(frame, rot(0, 20.0), (0.0, -2.0, 0.0), 2.2),  # pitched, wide angle
            turned(frame, rot(1, 170.0))]                         # looking back


def path(frame):
    """A 6-frame camera path: 1.5 degrees of yaw and a move per frame."""
    return rt_amd.camera_path(frame, 6, yaw_deg=1.5, step=(0.6, 0.0, -0.4))


def moving(frame, n=6):
    """The bench's moving camera (bench.py frame_costs): translated by
    (-0.29, 0, +0.17) more every frame, orientation and film unchanged — a
    camera sliding sideways, the per-frame move of a display loop."""
    out = []
    for k in range(n):
        f = frame.copy()
        f.cam_pos[0] -= 0.29 * (k + 1)
        f.cam_pos[2] += 0.17 * (k + 1)
        out.append(f)
    return out


# Full-size moved frames of the 50k heightfield at C3 (1920x1080, depth 0):
# frames of moving() pinned by whole-frame digests (cameras.json key
# f"hf_1920x1080_d0_moving{i}")
MOVING_FULL = ("hf", 1920, 1080, 0, (3, 6))


def words(f) -> list:
    """The camera words of a frame, as the reference's pixel loop reads them."""
    return [*f.cam_pos, *f.orient, f.half_w, f.half_h, f.inv_w, f.inv_h]


def words_sha(f) -> str:
    return hashlib.sha256(np.asarray(words(f), np.float32).tobytes()).hexdigest()


# Fixture sets: (key, scene name, W, H, depth); every set renders every KINDS
W, H = 480, 270
SETS = [("scene2", "scene2", W, H, 0), ("scene7", "scene7", W, H, 3), ("scene9", "scene9", W, H, 5),
        ("hf", "hf", W, H, 0)]


def key(which, kind, i):
    """The fixture key of frame i of a set (cameras.json)."""
    name, w, h, depth = next((n, w_, h_, d) for k, n, w_, h_, d in SETS if k == which)
    return f"{which}_{w}x{h}_d{depth}_{kind}{i}"


KINDS = {"cams": cameras, "path": path, "moving": moving}
