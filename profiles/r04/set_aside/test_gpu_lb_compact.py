"""Compact light-buffer cell lists (RT_OPT_LB_COMPACT, big lists): the cell
entries are {triangle, key} and the walks read the triangle's record from the
triangle array (rt_lightbuf.h lb_cell_entry), so every walk tests the same
triangles with the same operands in the same order — the images are the
default buffer's bits, pinned here to the reference-built C3 windows
(tests/golden/make_golden.py, make_c3_column_golden.py).  The shadow test
these walks replace: ObtenirFiltreDeSurface, Scene.cpp:1842-1861."""
from __future__ import annotations

import numpy as np
import pytest

import rt_amd
from conftest import bits_equal, scene
from test_gpu_parity import _hf_windows, c3_column, check, render  # noqa: F401

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")


def test_compact_heightfield_windows(golden_images, c3_column, heightfield_path):  # noqa: F811
    c = rt_amd.Context(0, lb_compact=1)
    assert c.get_option("lb_compact") == 1
    full = render(c, heightfield_path, 1920, 1080, 1)
    for k, want in _hf_windows(golden_images, c3_column):
        r0, r1, c0, c1 = map(int, k.rsplit("_win_", 1)[1].split("_"))
        check(full[r0:r1, c0:c1], want, 0)
    c.close()


@pytest.mark.parametrize("near,far", [(1.05, [1.1, 1.3, 2.0, 4.0]), (1.5, [64.0])])
def test_compact_far_ladder_and_stats_equal_default(heightfield_path, near, far):
    """Far levels walk compact lists too; the counted kernel renders the
    same bits and counts the same exact tests as the default lists."""
    a = rt_amd.Context(0, dcov_near=near, far_ladder=far)
    b = rt_amd.Context(0, dcov_near=near, far_ladder=far, lb_compact=1)
    s = rt_amd.Scene(heightfield_path, 640, 360, 1)
    a.upload(s)
    b.upload(s)
    f = s.frame.copy()
    f.flags = rt_amd.FLAG_STATS
    want = a.render_float(f)
    sa = a.stats()
    got = b.render_float(f)
    sb = b.stats()
    assert bits_equal(got, want)
    fields = [n for n, _ in type(sa)._fields_ if n != "kernel_ms"]
    assert [getattr(sa, n) for n in fields] == [getattr(sb, n) for n in fields]
    a.close()
    b.close()


def test_compact_slabs_bands_async(heightfield_path):
    a = rt_amd.Context(0)
    b = rt_amd.Context(0, lb_compact=1)
    s = rt_amd.Scene(heightfield_path, 512, 288, 1)
    a.upload(s)
    b.upload(s)
    full = a.render_float(s.frame)
    assert bits_equal(b.render_float(s.frame), full)
    f = s.frame.copy()
    f.row_begin, f.row_end = 40, 203
    assert bits_equal(b.render_float(f), full[40:203])
    f = s.frame.copy()
    f.band_rows, f.band_count, f.band_index = 16, 3, 1
    rows = [r for r in range(288) if (r // 16) % 3 == 1]
    assert bits_equal(b.render_float(f), full[rows])
    o = torch.zeros((288, 512, 3), dtype=torch.float32, device="cuda")
    st = torch.cuda.current_stream()
    b.render_async(s.frame, 0, o.data_ptr(), st.cuda_stream)
    torch.cuda.synchronize()
    assert bits_equal(o.cpu().numpy(), full)
    a.close()
    b.close()


def test_compact_is_inert_for_small_lists():
    """Scenes of <= 1,024 triangles keep whole entries (the option only
    applies to big lists)."""
    s = rt_amd.Scene(scene(2), 320, 180, 3)
    a = rt_amd.Context(0)
    b = rt_amd.Context(0, lb_compact=1)
    a.upload(s)
    b.upload(s)
    assert np.array_equal(b.render(s.frame), a.render(s.frame))
    a.close()
    b.close()
