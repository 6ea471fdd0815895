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


def _assemble(ctx, s, h, n, band_rows):
    """The frame from n shares: contiguous slabs (band_rows 0) or cyclic
    bands, each rendered on its own and put back in place."""
    from rt_amd.dist import slab_rows

    full = None
    for r in range(n):
        f = s.frame.copy()
        if band_rows:
            f.band_rows, f.band_count, f.band_index = band_rows, n, r
        else:
            r0, r1, _ = slab_rows(h, n, r)
            f.row_begin, f.row_end = r0, r1
        part = ctx.render_float(f)
        if full is None:
            full = np.full((h,) + part.shape[1:], np.nan, dtype=np.float32)
        if band_rows:
            for q in range(part.shape[0] // band_rows):
                a = (q * n + r) * band_rows
                e = min(h, a + band_rows)
                full[a:e] = part[q * band_rows: q * band_rows + (e - a)]
        elif part.shape[0]:
            full[r0:r1] = part
    return full


@pytest.mark.parametrize("seed", range(0, 120, 3))
def test_fuzz_scene_other_kernels_and_shares(oracle, tmp_path, seed):
    """The same scenes through the wave-culling kernels (no light buffer,
    no camera buffer) and as 2-5 row slabs or cyclic 16-row bands: every
    pixel equals the oracle's full frame."""
    specular = seed % 3 == 2
    big = seed % 10 == 7
    path = tmp_path / f"fuzz{seed}.dat"
    path.write_text(fuzz_dat(seed, specular, big))
    depth = 0 if big and seed % 20 == 7 else seed % 6
    w, h = (64, 48) if big else (48, 36)
    s = rt_amd.Scene(str(path), w, h, depth)
    want = oracle.render(str(path), w, h, depth)

    def same(got):
        if specular:
            return ulp_diff(got, want) <= 8
        return bits_equal(got, want)

    plain = rt_amd.Context(0, light_buffer=0, camera_buffer=0)
    plain.upload(s)
    assert same(plain.render_float(s.frame)), "wave-culling kernels"
    ctx = rt_amd.Context(0)
    ctx.upload(s)
    n = 2 + seed % 4
    assert same(_assemble(ctx, s, h, n, 0)), f"{n} slabs"
    assert same(_assemble(ctx, s, h, n, 16)), f"{n} bands"
