"""The CPU backend (include/rt.h rt_create_cpu / rt_cpu_render*, csrc/
rt_cpu.cpp) — SURVEY.md 8(b)'s second backend, the reference's CPU branch of
LancerRayons (Scene.cpp:1535-1563) — against the fixtures made from the
reference's own sources, on the CPU box: the same float32 bits, scene4's
Phong highlights included (glibc powf, like the reference).  And the
backend is explicit: HIP entry points refuse a CPU context, CPU entry points
a HIP one."""
from __future__ import annotations

import hashlib
import os
import subprocess

import numpy as np
import pytest

import rt_amd
from conftest import REPO, bits_equal, rgba8, scene

THREADS = min(8, os.cpu_count() or 1)


@pytest.fixture(scope="module")
def cpu():
    return rt_amd.CpuContext(THREADS)


def render(ctx, path, w, h, depth, rows=None, bands=None):
    s = rt_amd.Scene(path, w, h, depth)
    ctx.upload(s)
    f = s.frame.copy()
    if rows:
        f.row_begin, f.row_end = rows
    if bands:
        f.band_rows, f.band_count, f.band_index = bands
    return ctx.render_float(f)


@pytest.mark.parametrize("i", range(1, 10))
@pytest.mark.parametrize("depth", [0, 1, 3, 5])
def test_scene_images_match_reference(cpu, golden_images, i, depth):
    assert bits_equal(render(cpu, scene(i), 64, 48, depth), golden_images[f"scene{i}_64x48_d{depth}"])


@pytest.mark.parametrize("wh", [(1, 1), (13, 7), (67, 33)])
def test_ragged_sizes(cpu, golden_images, wh):
    w, h = wh
    assert bits_equal(render(cpu, scene(5), w, h, 3), golden_images[f"scene5_{w}x{h}_d3"])


def test_scene2_1080p_digests(cpu, digests):
    full = render(cpu, scene(2), 1920, 1080, 0)
    assert hashlib.sha256(full.tobytes()).hexdigest() == digests["scene2_1920x1080_d0_rgb_f32_sha256"]
    s = rt_amd.Scene(scene(2), 1920, 1080, 3)
    cpu.upload(s)
    q = cpu.render(s.frame)  # depth 3 renders the depth-0 image (no Kr / Kt)
    assert hashlib.sha256(q.tobytes()).hexdigest() == digests["scene2_1920x1080_d0_rgba8_sha256"]
    assert np.array_equal(q, rgba8(full))


def test_big_frame_window_slab(cpu, golden_images):
    """A row slab of the 2160p depth-5 bounce scene (rt_frame rows)."""
    got = render(cpu, scene(7), 3840, 2160, 5, rows=(1000, 1016))
    assert bits_equal(got[:, 1800:1832], golden_images["scene7_2160p_d5_win_1000_1016_1800_1832"])


def test_bands_and_slabs_reassemble(cpu):
    w, h = 160, 120
    full = render(cpu, scene(9), w, h, 5)
    got = np.full_like(full, np.nan)
    for r in range(3):
        part = render(cpu, scene(9), w, h, 5, bands=(16, 3, r))
        for q in range(part.shape[0] // 16):
            a = (q * 3 + r) * 16
            e = min(h, a + 16)
            got[a:e] = part[q * 16: q * 16 + (e - a)]
    assert bits_equal(got, full)
    parts = [render(cpu, scene(9), w, h, 5, rows=(r * 40, (r + 1) * 40)) for r in range(3)]
    assert bits_equal(np.concatenate(parts, 0), full)


def test_cull_stress_goldens(cpu, tmp_path):
    import cull_scenes

    with np.load(os.path.join(REPO, "tests", "golden", "cull.npz")) as z:
        names = sorted(z.files)[:6]
        gold = {k: z[k] for k in names}
    for n in names:
        seed, wh, d = n[2:].split("_")
        w, h = map(int, wh.split("x"))
        depth = int(d[1:])
        p = cull_scenes.write(str(tmp_path / f"c{seed}_{depth}.dat"), int(seed), 0.3 if depth else 0.0,
                              cull_scenes.n_small_for(int(seed)))
        assert bits_equal(render(cpu, p, w, h, depth), gold[n]), n


def test_backend_is_explicit(cpu):
    import ctypes

    L = rt_amd.lib()
    s = rt_amd.Scene(scene(1), 16, 16, 0)
    cpu.upload(s)
    out = np.zeros((16, 16, 4), np.uint8)
    # HIP entry points refuse a CPU context
    assert L.rt_render(cpu._h, ctypes.byref(s.frame), out.ctypes.data) == -4
    assert L.rt_render_async(cpu._h, ctypes.byref(s.frame), None, None, None) == -4
    assert L.rt_prepare_camera(cpu._h, ctypes.byref(s.frame)) == -4
    assert b"rt_cpu_render" in L.rt_last_error(cpu._h)
    # and the CScene verbs only take the CPU path when asked to
    c = rt_amd.CScene(backend="cpu", threads=THREADS)
    c.AjusterResolution(64, 48)
    c.AjusterNbRebondsMax(3)
    c.TraiterFichierDeScene(scene(7))
    assert isinstance(c._prepared() and c._ctx, rt_amd.CpuContext)
    with pytest.raises(ValueError):
        rt_amd.CScene(backend="auto")


def test_hip_context_needs_a_gpu():
    """rt_create fails loudly without a HIP device: no silent CPU path."""
    torch = pytest.importorskip("torch")
    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    with pytest.raises(rt_amd.RtError) as e:
        rt_amd.Context(0)
    assert e.value.code == -5


def test_cli_cpu_backend_matches_reference_digest(tmp_path, digests):
    """The headless entry surface with --backend cpu (Main.cpp:51-199): the
    PPM, turned back into the GL texture's layout, hashes like the
    reference build's scene2 1920x1080 frame — on a box without a GPU."""
    exe = os.path.join(REPO, "ray-tracing-gpu_amd", "lib", "rt_render")
    out = tmp_path / "s2.ppm"
    r = subprocess.run([exe, scene(2), "-x", "1920", "-y", "1080", "-d", "0", "--backend", "cpu", "--threads",
                        str(THREADS), "-o", str(out)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    data = open(out, "rb").read()
    head = data.split(b"\n", 3)
    img = np.frombuffer(head[3], np.uint8).reshape(1080, 1920, 3)[::-1]
    tex = np.concatenate([img, np.full((1080, 1920, 1), 255, np.uint8)], -1)
    assert hashlib.sha256(tex.tobytes()).hexdigest() == digests["scene2_1920x1080_d0_rgba8_sha256"]
    bad = subprocess.run([exe, scene(2), "--backend", "vulkan"], capture_output=True, text=True, timeout=60)
    assert bad.returncode == 1 and "[ERREUR]" in bad.stderr


@pytest.mark.parametrize("seed", range(120))
def test_fuzz_scenes_match_oracle(cpu, oracle, tmp_path, seed):
    """The seeded random scenes of tests/fuzz_scenes.py (pinned against
    oracle/_ref by test_oracle_fuzz.py), all 120 at the same sizes and
    depths, Phong and the 1,100-1,600-triangle scenes included: the CPU backend equals the oracle bit for bit."""
    from fuzz_scenes import fuzz_dat

    big = seed % 10 == 7
    path = tmp_path / f"fuzz{seed}.dat"
    path.write_text(fuzz_dat(seed, seed % 3 == 2, big))
    depth = 0 if big and seed % 20 == 7 else seed % 6
    w, h = (64, 48) if big else (48, 36)
    assert bits_equal(render(cpu, str(path), w, h, depth), oracle.render(str(path), w, h, depth))
