"""The lane-refill bounce kernel (RT_OPT_BOUNCE_REFILL, rt_refill_kernel):
persistent waves whose lanes take a new pixel when their ray tree ends.  It
runs radiance<MAXD>'s per-ray steps (Scene.cpp:1760-1822, ObtenirCouleur's
recursion) in a different lane order, so every image equals the one-pixel-
per-lane kernel's bits — which test_gpu_parity pins to the oracle."""
from __future__ import annotations

import numpy as np
import pytest

import rt_amd
from conftest import bits_equal, scene

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")


@pytest.mark.parametrize("n,w,h,depth", [(7, 320, 200, 5), (9, 333, 197, 5), (2, 256, 144, 5),
                                         (3, 160, 120, 3), (7, 64, 8, 1), (9, 8, 8, 20)])
def test_refill_renders_the_same_bits(n, w, h, depth):
    s = rt_amd.Scene(scene(n), w, h, depth)
    a = rt_amd.Context(0)
    a.upload(s)
    want = a.render_float(s.frame)
    want8 = a.render(s.frame)
    b = rt_amd.Context(0, bounce_refill=1)
    b.upload(s)
    assert b.get_option("bounce_refill") == 1
    assert bits_equal(b.render_float(s.frame), want)
    assert np.array_equal(b.render(s.frame), want8)
    a.close()
    b.close()


def test_refill_slabs_bands_and_async():
    s = rt_amd.Scene(scene(7), 256, 160, 5)
    a = rt_amd.Context(0)
    a.upload(s)
    full = a.render_float(s.frame)
    b = rt_amd.Context(0, bounce_refill=1)
    b.upload(s)
    f = s.frame.copy()
    f.row_begin, f.row_end = 24, 131
    assert bits_equal(b.render_float(f), full[24:131])
    f = s.frame.copy()
    f.band_rows, f.band_count, f.band_index = 16, 3, 2
    rows = [r for r in range(160) if (r // 16) % 3 == 2]
    assert bits_equal(b.render_float(f), full[rows])
    o = torch.empty((160, 256, 3), dtype=torch.float32, device="cuda")
    st = torch.cuda.current_stream()
    for _ in range(3):  # the work counter is reset by every launch
        o.zero_()
        b.render_async(s.frame, 0, o.data_ptr(), st.cuda_stream)
        torch.cuda.synchronize()
        assert bits_equal(o.cpu().numpy(), full)
    a.close()
    b.close()
