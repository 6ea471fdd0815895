"""Generate the golden fixtures in tests/golden/ from oracle/_ref.

oracle/_ref/libref_oracle.so is compiled by oracle/Makefile (`make -C oracle
ref`) from the reference's OWN sources under /root/reference (Triangle.cpp,
Plan.cpp, Quadrique.cpp, Matrice4.cpp, Vecteur3.h, Couleur.h, ...) plus the
CScene-orchestration harness oracle/ref_harness.cpp.  Every primitive test,
Pretraitement, vector/matrix/colour operation behind these numbers is the
reference's code.  Run in the build container (the reference does not exist on
the GPU box):

    make -C oracle ref && python tests/golden/make_golden.py

Outputs (data only — inputs and expected outputs):
  images.npz      float32 RGB (m_InfoPixel) for scene1..9 x depth {0,1,3,5}
                  at 64x48, plus windows of big frames (scene2 1920x1080,
                  heightfield 1920x1080 depth 1, scene7/9 3840x2160 depth 5)
  prepared.npz    post-Pretraitement state (surfaces/camera/lights) per scene
  kat.npz         per-primitive known answers through CTriangle/CPlan/
                  CQuadrique::Intersection (ray in, t / normal / hit out)
  digests.json    SHA-256 of full frames too large to store
"""
from __future__ import annotations

import ctypes
import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
SCENES = "/root/reference/Projet-INF8702/Scenes"
sys.path.insert(0, os.path.join(REPO, "ray-tracing-gpu_amd"))

from rt_amd import synth  # noqa: E402

VP = ctypes.c_void_p


def load_ref():
    L = ctypes.CDLL(os.path.join(REPO, "oracle", "_ref", "libref_oracle.so"))
    L.ref_load.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.POINTER(VP)]
    L.ref_render_window.argtypes = [VP, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, VP]
    L.ref_counts.argtypes = [VP, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int)]
    L.ref_dump.argtypes = [VP, VP, VP, VP]
    L.ref_free.argtypes = [VP]
    L.ref_intersect.argtypes = [ctypes.c_int, VP, VP, VP, VP, VP]
    return L


class Ref:
    def __init__(self, L, path, w, h, depth):
        self.L, self.w, self.h = L, w, h
        self.p = VP()
        rc = L.ref_load(path.encode(), w, h, depth, ctypes.byref(self.p))
        assert rc == 0, (path, rc)

    def window(self, r0, r1, c0, c1):
        out = np.zeros((r1 - r0, c1 - c0, 3), np.float32)
        self.L.ref_render_window(self.p, r0, r1, c0, c1, out.ctypes.data)
        return out

    def dump(self):
        ns, nl = ctypes.c_int(), ctypes.c_int()
        self.L.ref_counts(self.p, ctypes.byref(ns), ctypes.byref(nl))
        s = np.zeros((ns.value, 24), np.float32)
        c = np.zeros(27, np.float32)
        l = np.zeros((max(nl.value, 1), 7), np.float32)
        self.L.ref_dump(self.p, s.ctypes.data, c.ctypes.data, l.ctypes.data)
        return s, c, l[: nl.value]

    def __del__(self):
        self.L.ref_free(self.p)


def sha(a: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def rgba8(rgb: np.ndarray) -> np.ndarray:
    """GL float -> GL_RGBA8 (clamp, x255, round half up), alpha 255."""
    c = np.where(rgb > 0, np.where(rgb < 1, rgb, np.float32(1)), np.float32(0)).astype(np.float32)
    q = np.floor(c * np.float32(255) + np.float32(0.5)).astype(np.uint8)
    return np.concatenate([q, np.full(q.shape[:-1] + (1,), 255, np.uint8)], -1)


# Big-frame windows: (name, scene, W, H, depth, [(r0, r1, c0, c1), ...])
def big_windows(hf_path):
    return [
        ("scene2_1080p_d0", f"{SCENES}/scene2.dat", 1920, 1080, 0,
         [(0, 16, 0, 32), (500, 516, 900, 932), (1064, 1080, 1888, 1920), (300, 316, 1200, 1232)]),
        ("scene2_1080p_d3", f"{SCENES}/scene2.dat", 1920, 1080, 3, [(500, 516, 900, 932)]),
        ("hf_1080p_d1", hf_path, 1920, 1080, 1, [(540, 556, 960, 976), (200, 208, 300, 332)]),
        ("scene7_2160p_d5", f"{SCENES}/scene7.dat", 3840, 2160, 5,
         [(1000, 1016, 1800, 1832), (1080, 1096, 2400, 2432)]),
        ("scene9_2160p_d5", f"{SCENES}/scene9.dat", 3840, 2160, 5,
         [(1000, 1016, 1800, 1832), (1500, 1516, 500, 532)]),
    ]


def kat_rays(rng, n, center, spread):
    o = (center + rng.uniform(-spread, spread, (n, 3))).astype(np.float32)
    d = rng.normal(size=(n, 3))
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    return o, d.astype(np.float32)


def main():
    L = load_ref()
    hf = synth.write_heightfield(os.path.join("/tmp", "rt_amd_heightfield.dat"))
    images, prepared, digests, kat = {}, {}, {}, {}
    for i in range(1, 10):
        path = f"{SCENES}/scene{i}.dat"
        for d in (0, 1, 3, 5):
            r = Ref(L, path, 64, 48, d)
            images[f"scene{i}_64x48_d{d}"] = r.window(0, 48, 0, 64)
        s, c, l = Ref(L, path, 64, 48, 0).dump()
        prepared[f"scene{i}_surf"], prepared[f"scene{i}_cam"], prepared[f"scene{i}_lights"] = s, c, l
        s, c, l = Ref(L, path, 1920, 1080, 0).dump()
        prepared[f"scene{i}_1080p_cam"] = c
        print("scene", i, "done", flush=True)
    # ragged / odd sizes (partial 8x8 tiles, 1-pixel frames)
    for (w, h) in ((1, 1), (13, 7), (67, 33)):
        images[f"scene5_{w}x{h}_d3"] = Ref(L, f"{SCENES}/scene5.dat", w, h, 3).window(0, h, 0, w)
    # heightfield prepared state: digest + head/tail
    s, c, l = Ref(L, hf, 1920, 1080, 1).dump()
    prepared["hf_surf_head"], prepared["hf_surf_tail"] = s[:64], s[-64:]
    prepared["hf_cam"], prepared["hf_lights"] = c, l
    digests["hf_surf_sha256"] = sha(s)
    digests["hf_n_surfaces"] = int(s.shape[0])
    # big-frame windows
    for name, path, w, h, d, wins in big_windows(hf):
        r = Ref(L, path, w, h, d)
        for (r0, r1, c0, c1) in wins:
            images[f"{name}_win_{r0}_{r1}_{c0}_{c1}"] = r.window(r0, r1, c0, c1)
        print(name, "done", flush=True)
    # scene2 full 1080p depth 0: digest of float RGB and RGBA8
    full = Ref(L, f"{SCENES}/scene2.dat", 1920, 1080, 0).window(0, 1080, 0, 1920)
    digests["scene2_1920x1080_d0_rgb_f32_sha256"] = sha(full)
    digests["scene2_1920x1080_d0_rgba8_sha256"] = sha(rgba8(full))
    digests["scene2_1920x1080_d0_rgb_sum"] = float(full.astype(np.float64).sum())
    # per-primitive KATs against the scenes' own prepared primitives
    rng = np.random.default_rng(0x5EED)
    for i in (1, 2, 4, 9):
        s = prepared[f"scene{i}_surf"]
        for k, row in enumerate(s):
            typ = int(row[0])
            if typ == 0:
                geom = np.concatenate([row[11:20], row[20:23]]).astype(np.float32)
                center = row[11:20].reshape(3, 3).mean(0)
            elif typ == 1:
                geom = np.concatenate([row[11:15], np.zeros(8, np.float32)]).astype(np.float32)
                center = -row[14] * row[11:14]
            else:
                geom = np.concatenate([row[11:21], np.zeros(2, np.float32)]).astype(np.float32)
                center = np.zeros(3, np.float32)
            o, dd = kat_rays(rng, 256, center, 120.0)
            # aim half of the rays at the primitive's centre
            aim = (center - o) / np.linalg.norm(center - o, axis=1, keepdims=True)
            dd[:128] = aim[:128].astype(np.float32)
            t = np.zeros(256, np.float32)
            n = np.zeros((256, 3), np.float32)
            hit = np.zeros(256, np.int32)
            tb, nb = np.zeros(1, np.float32), np.zeros(3, np.float32)
            for j in range(256):
                hit[j] = L.ref_intersect(typ, geom.ctypes.data, o[j].ctypes.data, dd[j].ctypes.data,
                                         tb.ctypes.data, nb.ctypes.data)
                t[j], n[j] = tb[0], nb
            kat[f"s{i}_{k}_type"] = np.int32(typ)
            kat[f"s{i}_{k}_geom"], kat[f"s{i}_{k}_o"], kat[f"s{i}_{k}_d"] = geom, o, dd
            kat[f"s{i}_{k}_t"], kat[f"s{i}_{k}_n"], kat[f"s{i}_{k}_hit"] = t, n, hit
    np.savez_compressed(os.path.join(HERE, "images.npz"), **images)
    np.savez_compressed(os.path.join(HERE, "prepared.npz"), **prepared)
    np.savez_compressed(os.path.join(HERE, "kat.npz"), **kat)
    with open(os.path.join(HERE, "digests.json"), "w") as f:
        json.dump(digests, f, indent=1, sort_keys=True)
    print("wrote", len(images), "images,", len(prepared), "prepared arrays,", len(kat) // 7, "KAT sets")


if __name__ == "__main__":
    main()
