"""Seeded random scenes (tests/fuzz_scenes.py: mixed triangles, planes and
quadric kinds, 0-4 lights, reflective and refractive/translucent materials,
transforms; every tenth one with 1,100-1,600 triangles for the big-list
kernels) at depths 0-5 through the product on the GPU, against the
oracle: bit-exact without Phong specular; with it, within the Phong
tolerance of the reference scenes (ocml powf vs glibc powf, <= 8 ulp,
RGBA8 within 1) — Scene.cpp:1705-1861."""
from __future__ import annotations

import numpy as np
import pytest

import rt_amd
from conftest import bits_equal, rgba8, ulp_diff
from fuzz_scenes import fuzz_dat

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    return rt_amd.Context(0)


@pytest.mark.parametrize("seed", range(120))
def test_fuzz_scene_matches_oracle(ctx, oracle, tmp_path, seed):
    specular = seed % 3 == 2
    big = seed % 10 == 7  # above 1,024 triangles: the big-list kernels
    path = tmp_path / f"fuzz{seed}.dat"
    path.write_text(fuzz_dat(seed, specular, big))
    depth = 0 if big and seed % 20 == 7 else seed % 6
    w, h = (64, 48) if big else (48, 36)
    s = rt_amd.Scene(str(path), w, h, depth)
    want = oracle.render(str(path), w, h, depth)
    ctx.upload(s)
    got = ctx.render_float(s.frame)
    if specular:
        assert ulp_diff(got, want) <= 8
        assert np.abs(rgba8(got).astype(int) - rgba8(want).astype(int)).max() <= 1
    else:
        assert bits_equal(got, want), f"max |d| {np.abs(got - want).max()} ulps {ulp_diff(got, want)}"
