"""Bounding-cone culling under stress (tests/cull_scenes.py): cameras and
lights in the planes of triangles, slivers, tiny and oversized triangles, a
far light.  The culled GPU loops must return the reference's image bit for
bit (golden: tests/golden/cull.npz, made by make_cull_golden.py from the
reference's own sources); the oracle is pinned against the same images."""
from __future__ import annotations

import os

import numpy as np
import pytest

import cull_scenes
from conftest import bits_equal

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.fixture(scope="module")
def cull_golden():
    with np.load(os.path.join(HERE, "golden", "cull.npz")) as z:
        return {k: z[k] for k in z.files}


def _cases():
    with np.load(os.path.join(HERE, "golden", "cull.npz")) as z:
        names = sorted(z.files)
    out = []
    for n in names:
        seed, wh, d = n[2:].split("_")
        w, h = map(int, wh.split("x"))
        out.append((n, int(seed), w, h, int(d[1:])))
    return out


CASES = _cases()


def _path(tmp_path, seed, depth):
    return cull_scenes.write(str(tmp_path / f"cs{seed}_{depth}.dat"), seed, 0.3 if depth else 0.0,
                             cull_scenes.n_small_for(seed))


@pytest.mark.parametrize("name,seed,w,h,depth", [c for c in CASES if c[2] <= 160])
def test_oracle_matches_reference(oracle, cull_golden, tmp_path, name, seed, w, h, depth):
    got = oracle.render(_path(tmp_path, seed, depth), w, h, depth)
    assert bits_equal(got, cull_golden[name])


@pytest.mark.gpu
@pytest.mark.parametrize("name,seed,w,h,depth", CASES)
def test_gpu_matches_reference(cull_golden, tmp_path, name, seed, w, h, depth):
    import rt_amd

    ctx = rt_amd.Context(0)
    s = rt_amd.Scene(_path(tmp_path, seed, depth), w, h, depth)
    ctx.upload(s)
    got = ctx.render_float(s.frame)
    want = cull_golden[name]
    bad = np.argwhere(~(got.view(np.uint32) == want.view(np.uint32)).all(-1))
    assert bits_equal(got, want), f"{len(bad)} pixels differ, first {bad[:5].tolist()}"


# Randomised viewpoints and lights (seeds >= 100), small frames: the GPU
# against the oracle restatement (itself pinned bit-for-bit to the reference
# above and in test_oracle.py).  Seeds 106+ add 1,200 small triangles (the
# two-level culling); every third seed renders with bounces.
@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(100, 112))
def test_gpu_matches_oracle_random_views(oracle, tmp_path, seed):
    import rt_amd

    depth = 3 if seed % 3 == 0 else 0
    n_small = 1200 if seed >= 106 else 60
    path = cull_scenes.write(str(tmp_path / f"r{seed}.dat"), seed, 0.3 if depth else 0.0, n_small)
    w, h = 96, 72
    ctx = rt_amd.Context(0)
    s = rt_amd.Scene(path, w, h, depth)
    ctx.upload(s)
    got = ctx.render_float(s.frame)
    want = oracle.render(path, w, h, depth)
    bad = np.argwhere(~(got.view(np.uint32) == want.view(np.uint32)).all(-1))
    assert bits_equal(got, want), f"{len(bad)} pixels differ, first {bad[:5].tolist()}"



# The light buffer (shadow cells, rt_kernels.hip shadow_opaque_lb) at cell
# resolutions from coarse to fine (RT_OPT_LB_SCALE: R from 16 up to the
# 1,024 cap), so cell borders, face edges and the per-light list all meet
# the stress geometry.
@pytest.mark.gpu
@pytest.mark.parametrize("name,seed,w,h,depth", [c for c in CASES if c[4] == 0])
def test_gpu_lightbuf_matches_reference(cull_golden, tmp_path, name, seed, w, h, depth):
    import rt_amd

    ctx = rt_amd.Context(0, light_buffer=1)
    s = rt_amd.Scene(_path(tmp_path, seed, depth), w, h, depth)
    ctx.upload(s)
    got = ctx.render_float(s.frame)
    assert bits_equal(got, cull_golden[name])


@pytest.mark.gpu
@pytest.mark.parametrize("scale", [0.25, 1.0, 4.0, 64.0])
@pytest.mark.parametrize("seed", [100, 101, 104, 106, 107, 110, 111])
def test_gpu_lightbuf_random_views(oracle, tmp_path, seed, scale):
    import rt_amd

    n_small = 1200 if seed >= 106 else 60
    path = cull_scenes.write(str(tmp_path / f"lb{seed}.dat"), seed, 0.0, n_small)
    w, h = 96, 72
    ctx = rt_amd.Context(0, light_buffer=1, lb_scale=scale)
    s = rt_amd.Scene(path, w, h, 0)
    ctx.upload(s)
    got = ctx.render_float(s.frame)
    want = oracle.render(path, w, h, 0)
    bad = np.argwhere(~(got.view(np.uint32) == want.view(np.uint32)).all(-1))
    assert bits_equal(got, want), f"{len(bad)} pixels differ, first {bad[:5].tolist()}"


# The wave-level shadow culling (the path with the light buffer switched
# off: RT_OPT_LIGHT_BUFFER 0), which the default no longer takes for these
# scenes, against the same reference goldens.
@pytest.mark.gpu
@pytest.mark.parametrize("name,seed,w,h,depth", [c for c in CASES if c[4] == 0])
def test_gpu_wave_culling_matches_reference(cull_golden, tmp_path, name, seed, w, h, depth):
    import rt_amd

    ctx = rt_amd.Context(0, light_buffer=0)
    s = rt_amd.Scene(_path(tmp_path, seed, depth), w, h, depth)
    ctx.upload(s)
    assert bits_equal(ctx.render_float(s.frame), cull_golden[name])
