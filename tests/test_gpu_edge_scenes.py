"""Degenerate scenes through the product on the GPU, bit-exact against the
oracle (the restatement pinned to the reference build): an empty file, lights
without surfaces, surfaces without lights, one primitive of each kind, and a
reflective/translucent pair without lights — the zero-triangle, zero-light and
zero-opaque paths of the upload (no light buffer, no camera records, no
cluster or union records) at depth 0 and 3, through the synchronous, the async
and the sequence entry points (Scene.cpp:231-501 parsing, 1705-1861
shading; SURVEY.md 8(c) edge cases)."""
from __future__ import annotations

import numpy as np
import pytest
import torch

import rt_amd
from conftest import bits_equal

pytestmark = pytest.mark.gpu

HEAD = """background: 20 40 60
origin: 0.0 10.0 200.0
eye: 0.0 0.0 0.0
up: 0.0 1.0 0.0
"""
LIGHT = """Lumiere: l1
        position: 50.0 200.0 150.0
        intens: 0.8
"""
PLANE = """Plane: p1
        v_linear: 0.0 1.0 0.0
        v_const: 30.0
        color: 10 200 30
        ambient: 0.3
        diffus: 0.7
"""
TRI = """Poly: t1
        point: 0 -40.0 -20.0 0.0
        point: 1 40.0 -20.0 0.0
        point: 2 0.0 40.0 -10.0
        color: 200 120 40
"""
SPHERE = """Quad: s1
        v_quad: 1.0 1.0 1.0
        v_linear: 0.0 0.0 0.0
        v_const: -400.0
        color: 200 10 10
"""
MIRROR_GLASS = """Poly: m1
        point: 0 -60.0 -30.0 -20.0
        point: 1 60.0 -30.0 -20.0
        point: 2 0.0 60.0 -30.0
        color: 250 250 250
        reflect: 0.8
Quad: g1
        v_quad: 1.0 1.0 1.0
        v_linear: 0.0 0.0 0.0
        v_const: -100.0
        color: 100 100 250
        refract: 0.7 1.3
"""
SCENES = {
    "empty_file": "",
    "lights_only": HEAD + LIGHT,
    "plane_no_light": HEAD + PLANE,
    "triangle_no_light": HEAD + TRI,
    "sphere_no_light": HEAD + SPHERE,
    "plane_light": HEAD + PLANE + LIGHT,
    "triangle_light": HEAD + TRI + LIGHT,
    "sphere_light": HEAD + SPHERE + LIGHT,
    "mirror_glass_no_light": HEAD + MIRROR_GLASS,
    "mirror_glass_light": HEAD + PLANE + MIRROR_GLASS + LIGHT,
}


@pytest.mark.parametrize("name", sorted(SCENES))
@pytest.mark.parametrize("depth", [0, 3])
def test_edge_scene_matches_oracle(oracle, tmp_path, name, depth):
    path = tmp_path / f"{name}.dat"
    path.write_text(SCENES[name])
    w, h = 40, 28  # ragged: neither a multiple of 8 nor of 16
    s = rt_amd.Scene(str(path), w, h, depth)
    want = oracle.render(str(path), w, h, depth)
    ctx = rt_amd.Context(0)
    ctx.upload(s)
    assert bits_equal(ctx.render_float(s.frame), want), "sync"
    out = torch.zeros((h, w, 3), dtype=torch.float32, device="cuda")
    ctx.render_async(s.frame, 0, out.data_ptr(), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    assert bits_equal(out.cpu().numpy(), want), "async"
    seq = torch.zeros((2, h, w, 3), dtype=torch.float32, device="cuda")
    ctx.render_sequence_async([s.frame, s.frame], 0, 0, seq.data_ptr(), h * w * 12,
                              torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    for i in range(2):
        assert bits_equal(seq[i].cpu().numpy(), want), f"sequence {i}"
    if name == "empty_file" or name == "lights_only":
        # nothing to hit: every pixel is the background
        assert np.unique(want.reshape(-1, 3), axis=0).shape[0] == 1
