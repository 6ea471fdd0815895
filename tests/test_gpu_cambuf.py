"""The camera buffer built on the stream (round 3, rt_cambuf.h): per-tile
triangle lists binned by triangle screen boxes, with no host round trip.

* every list equals brute force — each tile with a list against every
  triangle, the camera wave test of the per-wave path (rt_debug_cb_verify) —
  for the reference's cameras and for moved, yawed, pitched, rolled and
  wide-angle ones, odd frame sizes, slabs and bands;
* rt_render_async of a moving camera builds the buffer itself (big lists)
  and renders the bits of a cold context (the reference's, pinned by
  test_gpu_parity);
* a capacity too small for the lists (RT_OPT_CB_CAPACITY) sends the tiles
  that do not fit down the per-wave path: the same image;
* the sequence path's per-slot buffers render cold-context bits.
The reference recomputes its camera for every frame (Scene.cpp:674 ->
:624-660); the lists only replace the per-wave culling of the camera rays
(ObtenirCouleur, Scene.cpp:1705-1738)."""
from __future__ import annotations

import ctypes

import numpy as np
import pytest

import rt_amd
from conftest import bits_equal, scene

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")


def _verify(ctx):
    L = rt_amd.lib()
    L.rt_debug_cb_verify.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    out = (ctypes.c_ulonglong * 3)()
    assert L.rt_debug_cb_verify(ctx._h, out) == 0, ctx._err()
    return list(out)


def _cb_info(ctx, n=10):
    L = rt_amd.lib()
    L.rt_debug_cb_info.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
    info = (ctypes.c_double * n)()
    assert L.rt_debug_cb_info(ctx._h, info, n) == 0
    return list(info)


def _rot(axis, deg):
    a = np.deg2rad(deg)
    c, s = np.cos(a), np.sin(a)
    i, j = [(1, 2), (2, 0), (0, 1)][axis]
    R = np.eye(3)
    R[i, i], R[i, j], R[j, i], R[j, j] = c, -s, s, c
    return R


def _turned(frame, R, move=(0.0, 0.0, 0.0), fov_scale=1.0):
    """The camera rotated by R about its own axes (orientation rows U V N),
    moved, and its film widened by fov_scale."""
    f = frame.copy()
    o = np.array(frame.orient[:], np.float64).reshape(4, 4)
    o[:3, :3] = R @ o[:3, :3]
    for i, v in enumerate(o.astype(np.float32).ravel()):
        f.orient[i] = float(v)
    for i in range(3):
        f.cam_pos[i] += move[i]
    f.half_w *= fov_scale
    f.half_h *= fov_scale
    return f


def _cameras(frame):
    return [frame,
            _turned(frame, _rot(1, 7.0), (3.0, 0.5, -2.0)),
            _turned(frame, _rot(0, -11.0) @ _rot(1, 23.0), (-4.0, 1.0, 2.0)),
            _turned(frame, _rot(2, 35.0)),                          # roll
            _turned(frame, _rot(0, 20.0), (0.0, -2.0, 0.0), 2.2),  # pitched, wide angle
            _turned(frame, _rot(1, 170.0))]                         # looking back


@pytest.mark.parametrize("which,w,h", [("scene2", 640, 360), ("scene2", 333, 197), ("scene3", 320, 240),
                                       ("scene1", 160, 120),
                                       ("hf", 640, 360), ("hf", 250, 131)])
def test_lists_equal_brute_force(heightfield_path, which, w, h):
    path = heightfield_path if which == "hf" else scene(int(which[-1]))
    s = rt_amd.Scene(path, w, h, 0)
    ctx = rt_amd.Context(0)
    ctx.upload(s)
    for i, f in enumerate(_cameras(s.frame)):
        ctx.prepare_camera(f)
        bad, pairs, listed = _verify(ctx)
        assert bad == 0, (i, bad, pairs, listed)
        assert listed > 0, i
    ctx.close()


@pytest.mark.parametrize("rows,bands", [((40, 176), None), (None, (16, 3, 1))])
def test_partial_frame_lists_equal_brute_force(heightfield_path, rows, bands):
    s = rt_amd.Scene(heightfield_path, 480, 270, 0)
    ctx = rt_amd.Context(0)
    ctx.upload(s)
    f = _turned(s.frame, _rot(1, 5.0), (1.0, 0.0, 1.0))
    if rows:
        f.row_begin, f.row_end = rows
    if bands:
        f.band_rows, f.band_count, f.band_index = bands
    ctx.prepare_camera(f)
    bad, pairs, listed = _verify(ctx)
    assert bad == 0 and listed > 0
    ctx.close()


def _cold(path, w, h, frames):
    s = rt_amd.Scene(path, w, h, 0)
    out = []
    for f in frames:
        c = rt_amd.Context(0)
        c.upload(s)
        out.append(c.render_float(f))
        c.close()
    return out


@pytest.mark.parametrize("which,ring", [("scene2", 0), ("hf", 1), ("hf", 0)])
def test_async_moving_camera_builds_and_matches(heightfield_path, which, ring):
    """Big lists: each new camera's state is built by the async render —
    in the async ring on the internal stream (ring 1), or in the context's
    own state on the caller's stream (ring 0)."""
    path = heightfield_path if which == "hf" else scene(2)
    w, h = 480, 270
    s = rt_amd.Scene(path, w, h, 0)
    frames = rt_amd.camera_path(s.frame, 6, yaw_deg=1.5, step=(0.6, 0.0, -0.4))
    want = _cold(path, w, h, frames)
    ctx = rt_amd.Context(0, async_ring=ring, camera_buffer=2)  # 2: async builds at any size
    ctx.upload(s)
    st = torch.cuda.current_stream()
    outs = []
    for f in frames:
        o = torch.empty((h, w, 3), dtype=torch.float32, device="cuda")
        ctx.render_async(f, 0, o.data_ptr(), st.cuda_stream)
        outs.append(o)
    torch.cuda.synchronize()
    info = _cb_info(ctx)
    if ring:  # the ring's slots: the context's own state untouched
        assert info[0] == 0.0
    else:  # the last camera's buffer, built by the async render (or rebuilt at
        # its next render if its guessed capacity fell short)
        assert info[1] > 0
        if info[0] == 1.0:
            assert _verify(ctx)[0] == 0
    for i, o in enumerate(outs):
        assert bits_equal(o.cpu().numpy(), want[i]), i
    ctx.close()


@pytest.mark.parametrize("cap", [1, 3000, 20000])
def test_overflowing_capacity_renders_the_same(heightfield_path, cap):
    w, h = 480, 270
    s = rt_amd.Scene(heightfield_path, w, h, 0)
    frames = rt_amd.camera_path(s.frame, 3, yaw_deg=2.0, step=(0.5, 0.0, 0.3))
    want = _cold(heightfield_path, w, h, frames)
    ctx = rt_amd.Context(0, cb_capacity=cap)
    ctx.upload(s)
    for i, f in enumerate(frames):
        assert bits_equal(ctx.render_float(f), want[i]), i
        bad, pairs, listed = _verify(ctx)
        assert bad == 0
        info = _cb_info(ctx)
        assert info[9] == cap
        if info[1] > cap:  # some tiles did not fit: they render by the per-wave path
            assert listed < (w // 8 + 1) * (h // 8 + 1)
    ctx.close()


def test_non_rotation_orientation_renders_without_buffer():
    """A scaled orientation is not a rotation: no camera buffer (the boxes
    need camera coordinates), the per-wave path, the same bits as a context
    with the camera buffer switched off."""
    s = rt_amd.Scene(scene(2), 320, 200, 0)
    f = s.frame.copy()
    for i in range(12):
        f.orient[i] *= 1.5
    a = rt_amd.Context(0)
    a.upload(s)
    got = a.render_float(f)
    assert _cb_info(a)[0] == 0.0
    b = rt_amd.Context(0, camera_buffer=0)
    b.upload(s)
    assert bits_equal(got, b.render_float(f))
    a.close()
    b.close()


@pytest.mark.parametrize("cbopt", [1, 2])
def test_sequence_slots_build_camera_buffers(heightfield_path, cbopt):
    w, h = 320, 200
    s = rt_amd.Scene(heightfield_path, w, h, 0)
    frames = rt_amd.camera_path(s.frame, 7, yaw_deg=1.0, step=(0.4, 0.0, -0.3))
    want = _cold(heightfield_path, w, h, frames)
    ctx = rt_amd.Context(0, camera_buffer=cbopt)
    ctx.upload(s)
    ring = torch.empty((len(frames), h, w, 3), dtype=torch.float32, device="cuda")
    for rep in range(2):  # the second call reuses the slots' buffers
        ring.zero_()
        ctx.render_sequence_async(frames, 0, 0, ring.data_ptr(), h * w * 12,
                                  torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        for i in range(len(frames)):
            assert bits_equal(ring[i].cpu().numpy(), want[i]), (rep, i)
    ctx.close()


def test_async_ring_two_streams_interleaved(heightfield_path):
    """The ring's slots under renders of alternating and repeated cameras
    on two streams, with no host sync between calls: every output equals
    a cold context's render of its camera."""
    w, h = 320, 200
    s = rt_amd.Scene(heightfield_path, w, h, 0)
    cams = rt_amd.camera_path(s.frame, 4, yaw_deg=2.0, step=(0.7, 0.0, -0.5))
    want = _cold(heightfield_path, w, h, cams)
    ctx = rt_amd.Context(0, camera_buffer=2, async_ring=1)
    ctx.upload(s)
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    order = [0, 1, 0, 2, 3, 3, 1, 2, 0, 3]
    outs = []
    for i, k in enumerate(order):
        st = s1 if i % 2 == 0 else s2
        o = torch.empty((h, w, 3), dtype=torch.float32, device="cuda")
        o.record_stream(st)
        ctx.render_async(cams[k], 0, o.data_ptr(), st.cuda_stream)
        outs.append((k, o))
        if i == 5:  # a synchronous render in the middle (the context's own state)
            assert bits_equal(ctx.render_float(cams[1]), want[1])
    ctx.sync()
    for i, (k, o) in enumerate(outs):
        assert bits_equal(o.cpu().numpy(), want[k]), (i, k)
    ctx.close()
