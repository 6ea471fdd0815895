"""BASELINE.json configs C1 and C4 (scene2) at their full sizes against the
reference build (tests/golden/make_config_golden.py, oracle/_ref):

* C1 = Scenes/scene1 at 512x512, max bounces 1 (Main.cpp:51-96 defaults
  for the resolution; the reference's CPU loop Scene.cpp:1538-1561): the
  whole float32 frame, bit for bit, on the HIP path and on the CPU backend;
* C4 = Scenes/scene2 at 3840x2160, max bounces 5: the SHA-256 of the float32
  frame and of its RGBA8 quantisation (GL_RGBA8 upload, Scene.cpp:1562)."""
from __future__ import annotations

import hashlib
import os

import numpy as np
import pytest

import rt_amd
from conftest import bits_equal, rgba8, scene

THREADS = min(8, os.cpu_count() or 1)


def _sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def _render(ctx, path, w, h, depth, as_float=True):
    s = rt_amd.Scene(path, w, h, depth)
    ctx.upload(s)
    return ctx.render_float(s.frame) if as_float else ctx.render(s.frame)


def test_c1_fixture_digests(config_golden):
    c1 = config_golden["c1_frame"]
    assert c1.shape == (512, 512, 3) and c1.dtype == np.float32
    assert _sha(c1) == config_golden["scene1_512x512_d1_rgb_f32_sha256"]
    assert _sha(rgba8(c1)) == config_golden["scene1_512x512_d1_rgba8_sha256"]


def test_c1_cpu_backend_full_frame(config_golden):
    cpu = rt_amd.CpuContext(THREADS)
    got = _render(cpu, scene(1), 512, 512, 1)
    assert bits_equal(got, config_golden["c1_frame"])
    q = _render(cpu, scene(1), 512, 512, 1, as_float=False)
    assert _sha(q) == config_golden["scene1_512x512_d1_rgba8_sha256"]


def test_c1_oracle_window(config_golden, oracle):
    """The C restatement on a window straddling the frame's centre."""
    got = oracle.render(scene(1), 512, 512, 1, (240, 272, 0, 512))
    assert bits_equal(got, config_golden["c1_frame"][240:272])


@pytest.mark.gpu
def test_c1_hip_full_frame(config_golden):
    ctx = rt_amd.Context(0)
    got = _render(ctx, scene(1), 512, 512, 1)
    assert bits_equal(got, config_golden["c1_frame"])
    q = _render(ctx, scene(1), 512, 512, 1, as_float=False)
    assert _sha(q) == config_golden["scene1_512x512_d1_rgba8_sha256"]
    ctx.close()


@pytest.mark.gpu
def test_c4_scene2_hip_reference_digest(config_golden):
    ctx = rt_amd.Context(0)
    got = _render(ctx, scene(2), 3840, 2160, 5)
    assert _sha(got) == config_golden["scene2_3840x2160_d5_rgb_f32_sha256"]
    assert abs(float(got.astype(np.float64).sum()) - config_golden["scene2_3840x2160_d5_rgb_sum"]) < 1e-6
    q = _render(ctx, scene(2), 3840, 2160, 5, as_float=False)
    assert _sha(q) == config_golden["scene2_3840x2160_d5_rgba8_sha256"]
    ctx.close()


@pytest.mark.gpu
@pytest.mark.parametrize("which", ["scene7", "scene9"])
def test_c4_bounce_scenes_full_frame_reference_digest(which):
    """C4's reflect / refract stress scenes at 3840x2160,
    depth 5, whole frame: float32 RGB and RGBA8 digests of oracle/_ref's
    frame (tests/golden/make_camera_golden.py)."""
    from conftest import cam_golden

    e = cam_golden()[f"{which}_3840x2160_d5_full"]
    ctx = rt_amd.Context(0)
    got = _render(ctx, scene(int(which[-1])), 3840, 2160, 5)
    assert _sha(got) == e["rgb_f32_sha256"], abs(float(got.astype(np.float64).sum()) - e["rgb_sum"])
    q = _render(ctx, scene(int(which[-1])), 3840, 2160, 5, as_float=False)
    assert _sha(q) == e["rgba8_sha256"]
    ctx.close()
