"""Shared test setup.

Markers: tests that need an MI355X are marked ``@pytest.mark.gpu``; everything
else runs on CPU.  The oracle (oracle/liboracle.so) and the golden fixtures
(tests/golden/) are the checkers; the product is librt_amd.so, reached only
through its C ABI (rt_amd is a ctypes binding of include/rt.h).
"""
from __future__ import annotations

import ctypes
import json
import os
import subprocess
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "ray-tracing-gpu_amd")
GOLDEN = os.path.join(REPO, "tests", "golden")
SCENES = os.path.join(GOLDEN, "scenes")
if PKG not in sys.path:
    sys.path.insert(0, PKG)
if REPO not in sys.path:
    sys.path.insert(0, REPO)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP device)")


def _ensure_built():
    lib = os.path.join(PKG, "lib", "librt_amd.so")
    orc = os.path.join(REPO, "oracle", "liboracle.so")
    if not os.path.exists(lib):
        subprocess.run(["make", "-s", "-C", PKG], check=True)
    if not os.path.exists(orc):
        subprocess.run(["make", "-s", "-C", os.path.join(REPO, "oracle")], check=True)


_ensure_built()

VP = ctypes.c_void_p


class Oracle:
    """ctypes view of oracle/liboracle.so (test infrastructure only)."""

    def __init__(self):
        L = ctypes.CDLL(os.path.join(REPO, "oracle", "liboracle.so"))
        L.oracle_load.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.POINTER(VP)]
        L.oracle_render_window.argtypes = [VP, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, VP, ctypes.c_int]
        L.oracle_counts.argtypes = [VP, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int)]
        L.oracle_dump.argtypes = [VP, VP, VP, VP]
        L.oracle_free.argtypes = [VP]
        L.oracle_error.argtypes = [VP]
        L.oracle_error.restype = ctypes.c_char_p
        L.oracle_intersect.argtypes = [ctypes.c_int, VP, VP, VP, VP, VP]
        L.oracle_set_params.argtypes = [VP, ctypes.c_int, ctypes.c_float, ctypes.c_float]
        self.L = L

    def load(self, path, w, h, depth):
        p = VP()
        rc = self.L.oracle_load(os.fsencode(path), w, h, depth, ctypes.byref(p))
        return rc, p

    def render(self, path, w, h, depth, window=None, threads=4):
        rc, p = self.load(path, w, h, depth)
        assert rc == 0, (path, rc, self.L.oracle_error(p))
        r0, r1, c0, c1 = window or (0, h, 0, w)
        out = np.zeros((r1 - r0, c1 - c0, 3), np.float32)
        self.L.oracle_render_window(p, r0, r1, c0, c1, out.ctypes.data, threads)
        self.L.oracle_free(p)
        return out

    def dump(self, path, w, h, depth=0):
        rc, p = self.load(path, w, h, depth)
        assert rc == 0, (path, rc)
        ns, nl = ctypes.c_int(), ctypes.c_int()
        self.L.oracle_counts(p, ctypes.byref(ns), ctypes.byref(nl))
        s = np.zeros((ns.value, 24), np.float32)
        c = np.zeros(27, np.float32)
        l = np.zeros((max(nl.value, 1), 7), np.float32)
        self.L.oracle_dump(p, s.ctypes.data, c.ctypes.data, l.ctypes.data)
        self.L.oracle_free(p)
        return s, c, l[: nl.value]


@pytest.fixture(scope="session")
def oracle():
    return Oracle()


@pytest.fixture(scope="session")
def golden_images():
    return np.load(os.path.join(GOLDEN, "images.npz"))


@pytest.fixture(scope="session")
def golden_prepared():
    return np.load(os.path.join(GOLDEN, "prepared.npz"))


@pytest.fixture(scope="session")
def golden_kat():
    return np.load(os.path.join(GOLDEN, "kat.npz"))


@pytest.fixture(scope="session")
def digests():
    with open(os.path.join(GOLDEN, "digests.json")) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def config_golden():
    """BASELINE.json configs at full size from oracle/_ref (make_config_golden.py):
    C1's whole float32 frame and C4-scene2's digests."""
    with open(os.path.join(GOLDEN, "configs.json")) as f:
        d = json.load(f)
    d["c1_frame"] = np.load(os.path.join(GOLDEN, "c1.npz"))["scene1_512x512_d1"]
    return d


@pytest.fixture(scope="session")
def heightfield_path(tmp_path_factory):
    from rt_amd import synth

    return synth.write_heightfield(str(tmp_path_factory.mktemp("hf") / "heightfield.dat"))


@pytest.fixture(scope="session")
def heightfield_r05_path(tmp_path_factory):
    """The heightfield with `reflect: 0.5` on every triangle (bench c3r / c5r)."""
    from rt_amd import synth

    return synth.write_heightfield(str(tmp_path_factory.mktemp("hfr") / "heightfield_r05.dat"), reflect=0.5)


def scene(i: int) -> str:
    return os.path.join(SCENES, f"scene{i}.dat")


def rgba8(rgb: np.ndarray) -> np.ndarray:
    """GL float -> GL_RGBA8: clamp to [0,1] (NaN -> 0), x255, +0.5, floor; alpha 255."""
    c = np.where(rgb > 0, np.where(rgb < 1, rgb, np.float32(1)), np.float32(0)).astype(np.float32)
    q = np.floor(c * np.float32(255) + np.float32(0.5)).astype(np.uint8)
    return np.concatenate([q, np.full(q.shape[:-1] + (1,), 255, np.uint8)], -1)


def bits_equal(a: np.ndarray, b: np.ndarray) -> bool:
    return a.shape == b.shape and np.array_equal(np.ascontiguousarray(a).view(np.uint32),
                                                 np.ascontiguousarray(b).view(np.uint32))


def ulp_diff(a: np.ndarray, b: np.ndarray) -> int:
    """Max distance in float32 ULPs (sign-magnitude ordered)."""
    def key(x):
        i = np.ascontiguousarray(x, np.float32).view(np.int32).astype(np.int64)
        return np.where(i < 0, -(i & 0x7FFFFFFF), i)
    if a.size == 0:
        return 0
    return int(np.abs(key(a) - key(b)).max())


# ---- moved cameras and big bounce frames pinned to oracle/_ref
# (tests/golden/make_camera_golden.py, cameras.json): per frame the SHA-256
# of its camera words and of the reference's float32 RGB / RGBA8 frame.
def _sha(a: np.ndarray) -> str:
    import hashlib

    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


_CAM_GOLDEN = None


def cam_golden() -> dict:
    global _CAM_GOLDEN
    if _CAM_GOLDEN is None:
        with open(os.path.join(GOLDEN, "cameras.json")) as f:
            _CAM_GOLDEN = json.load(f)
    return _CAM_GOLDEN


def cam_scene_path(which: str, hf_path: str) -> str:
    return hf_path if which == "hf" else scene(int(which[-1]))


class CamRef:
    """The reference frames of one fixture set of tests/cameras.py: its Scene,
    its frames of each kind, and the check of an image against _ref."""

    def __init__(self, which: str, hf_path: str):
        import cameras
        import rt_amd

        self.which = which
        _, name, self.w, self.h, self.depth = next(s for s in cameras.SETS if s[0] == which)
        self.path = cam_scene_path(which, hf_path)
        self.scene = rt_amd.Scene(self.path, self.w, self.h, self.depth)
        self.frames = {kind: fn(self.scene.frame) for kind, fn in cameras.KINDS.items()}
        for kind, frames in self.frames.items():  # the generator's camera words
            for i, f in enumerate(frames):
                assert cam_golden()[cameras.key(which, kind, i)]["camera_words_sha256"] == cameras.words_sha(f)

    def entry(self, kind: str, i: int) -> dict:
        import cameras

        return cam_golden()[cameras.key(self.which, kind, i)]

    def matches(self, img: np.ndarray, kind: str, i: int) -> bool:
        """float32 RGB (rows, W, 3) or RGBA8 (rows, W, 4) against the reference frame."""
        e = self.entry(kind, i)
        want = e["rgba8_sha256"] if img.dtype == np.uint8 else e["rgb_f32_sha256"]
        return _sha(img) == want
