"""Envelope lists (RT_OPT_CB_ENVELOPE, round 5): a camera moving by
translation walks per-tile lists built once for a ball of camera positions
(rt_cull.h cone_record_env, rt_camhost.h cb_envelope_build).

* structure: after every frame of a translating camera, the envelope lists
  hold every triangle that frame's own exact list would hold, keyed at most
  its own dmin (rt_debug_env_verify against the frame's own camera
  records) — small and large steps, odd frame sizes, slabs and bands;
* images: the frames of the moving camera (async, synchronous and
  interleaved with repeats) are the reference's (tests/golden/cameras.json,
  made by oracle/_ref with each frame's explicit camera words), at 480x270
  and at full C3 size (1920x1080: frames 3 and 6 of tests/cameras.py
  moving()), and bit-equal to the per-wave path for steps the fixtures do
  not cover.
The reference recomputes its camera every frame (Scene.cpp:674 -> :624-660)
and traces every camera ray through the all-surface loop of ObtenirCouleur
(Scene.cpp:1705-1738); the lists only choose which triangles a tile tests."""
from __future__ import annotations

import ctypes
import gc
import hashlib

import numpy as np
import pytest

import cameras
import rt_amd
from conftest import CamRef, bits_equal, cam_golden

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")


def env_info(ctx):
    L = rt_amd.lib()
    L.rt_debug_env_info.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
    out = (ctypes.c_double * 7)()
    assert L.rt_debug_env_info(ctx._h, out, 7) == 0, ctx._err()
    return list(out)


def env_verify(ctx):
    L = rt_amd.lib()
    L.rt_debug_env_verify.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    out = (ctypes.c_ulonglong * 3)()
    assert L.rt_debug_env_verify(ctx._h, out) == 0, ctx._err()
    return list(out)


def translated(frame, step, n):
    out = []
    for k in range(n):
        f = frame.copy()
        for i in range(3):
            f.cam_pos[i] += step[i] * (k + 1)
        out.append(f)
    return out


@pytest.mark.parametrize("w,h,step", [(480, 270, (-0.29, 0.0, 0.17)), (333, 197, (2.5, -0.7, 1.5)),
                                      (640, 360, (0.0, 0.0, -4.0)), (250, 131, (0.05, 0.02, 0.0))])
def test_envelope_lists_hold_each_camera(heightfield_path, w, h, step):
    s = rt_amd.Scene(heightfield_path, w, h, 0)
    ctx = rt_amd.Context(0)
    ctx.upload(s)
    ref = rt_amd.Context(0, camera_buffer=0)  # the per-wave path
    ref.upload(s)
    st = torch.cuda.current_stream().cuda_stream
    served = 0
    for i, f in enumerate([s.frame] + translated(s.frame, step, 12)):
        o = torch.empty((h, w, 3), dtype=torch.float32, device="cuda")
        ctx.render_async(f, 0, o.data_ptr(), st)
        info = env_info(ctx)
        if i >= 1:
            assert info[0] == 1.0 and info[2] >= 1, (i, info)
            bad, pairs, listed = env_verify(ctx)
            assert bad == 0 and pairs > 0 and listed >= pairs, (i, bad, pairs, listed)
            served += 1
        assert bits_equal(o.cpu().numpy(), ref.render_float(f)), i
    info = env_info(ctx)
    assert info[3] >= served  # every moving frame walked the envelope lists
    assert info[2] <= 1 + served // 8 + 1, info  # one build per 8 frames of motion
    ctx.close()
    ref.close()


@pytest.mark.parametrize("rows,bands", [((40, 176), None), (None, (16, 3, 1))])
def test_envelope_partial_frames(heightfield_path, rows, bands):
    s = rt_amd.Scene(heightfield_path, 480, 270, 0)
    ctx = rt_amd.Context(0)
    ctx.upload(s)
    ref = rt_amd.Context(0, camera_buffer=0)
    ref.upload(s)
    base = s.frame.copy()
    if rows:
        base.row_begin, base.row_end = rows
    if bands:
        base.band_rows, base.band_count, base.band_index = bands
    for i, f in enumerate([base] + translated(base, (0.8, 0.1, -0.5), 6)):
        got = ctx.render_float(f)  # synchronous renders take the envelope too
        if i >= 1:
            assert env_verify(ctx)[0] == 0, i
        assert bits_equal(got, ref.render_float(f)), i
    assert env_info(ctx)[3] >= 6
    ctx.close()
    ref.close()


@pytest.mark.parametrize("which", ["hf", "scene7", "scene9", "scene2"])
def test_moving_camera_matches_reference(heightfield_path, which):
    """tests/cameras.py moving() frames (the bench's translated camera) through
    rt_render_async, rt_render, and async with each camera repeated (a repeat
    builds its own exact lists), against _ref."""
    r = CamRef(which, heightfield_path)
    frames = r.frames["moving"]
    for mode in ("async", "sync", "repeat"):
        ctx = rt_amd.Context(0)
        ctx.upload(r.scene)
        st = torch.cuda.current_stream().cuda_stream
        outs = []
        ctx.render_float(r.scene.frame)
        for f in frames:
            for rep in range(2 if mode == "repeat" else 1):
                if mode == "sync":
                    outs.append(ctx.render_float(f))
                else:
                    o = torch.empty((r.h, r.w, 3), dtype=torch.float32, device="cuda")
                    ctx.render_async(f, 0, o.data_ptr(), st)
                    outs.append(o)
        torch.cuda.synchronize()
        per = 2 if mode == "repeat" else 1
        for i in range(len(frames)):
            for rep in range(per):
                o = outs[per * i + rep]
                img = o if isinstance(o, np.ndarray) else o.cpu().numpy()
                assert r.matches(img, "moving", i), (which, mode, i, rep)
        if which == "hf":
            assert env_info(ctx)[3] >= len(frames) - 1, mode
        ctx.close()


def _digest_key(i):
    name, w, h, d, _ = cameras.MOVING_FULL
    return f"{name}_{w}x{h}_d{d}_moving{i}"


def _sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def test_moving_c3_full_size_matches_reference(heightfield_path):
    """C3 (the 50k heightfield at 1920x1080, depth 0): the bench's translated
    camera, 7 frames through rt_render_async (envelope lists) and through
    rt_render_sequence_async (the sequence slots' own lists); frames 3 and 6
    against _ref's whole-frame digests."""
    name, w, h, d, idx = cameras.MOVING_FULL
    s = rt_amd.Scene(heightfield_path, w, h, d)
    frames = cameras.moving(s.frame, max(idx) + 1)
    g = cam_golden()
    for i in idx:
        assert g[_digest_key(i)]["camera_words_sha256"] == cameras.words_sha(frames[i])
    ctx = rt_amd.Context(0)
    ctx.upload(s)
    st = torch.cuda.current_stream().cuda_stream
    ctx.render_float(s.frame)
    outs = []
    for f in frames:
        o = torch.empty((h, w, 3), dtype=torch.float32, device="cuda")
        ctx.render_async(f, 0, o.data_ptr(), st)
        outs.append(o)
    torch.cuda.synchronize()
    assert env_info(ctx)[3] >= len(frames) - 1
    for i in idx:
        assert _sha(outs[i].cpu().numpy()) == g[_digest_key(i)]["rgb_f32_sha256"], ("async", i)
    ring = torch.empty((len(frames), h, w, 4), dtype=torch.uint8, device="cuda")
    ctx.render_sequence_async(frames, ring.data_ptr(), h * w * 4, 0, 0, st)
    torch.cuda.synchronize()
    for i in idx:
        assert _sha(ring[i].cpu().numpy()) == g[_digest_key(i)]["rgba8_sha256"], ("sequence", i)
    ctx.close()


def test_envelope_off_and_capture(heightfield_path):
    """RT_OPT_CB_ENVELOPE 0 builds none; a hipGraph capture of a moving
    frame never walks envelope lists (the per-wave path or the camera's own
    lists), and replays the same image."""
    s = rt_amd.Scene(heightfield_path, 480, 270, 0)
    frames = translated(s.frame, (0.5, 0.0, 0.3), 4)
    a = rt_amd.Context(0, cb_envelope=0)
    a.upload(s)
    for f in frames:
        a.render_float(f)
    assert env_info(a)[2] == 0 and env_info(a)[3] == 0
    b = rt_amd.Context(0)
    b.upload(s)
    for f in frames[:3]:
        b.render_float(f)
    want = a.render_float(frames[3])
    b.prepare_camera(frames[3])
    o = torch.zeros((270, 480, 3), dtype=torch.float32, device="cuda")
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    gc.collect()
    gc.disable()  # (a collection could finalize a context mid-capture: test_gpu_streams.capture)
    try:
        with torch.cuda.graph(g):
            b.render_async(frames[3], 0, o.data_ptr(), torch.cuda.current_stream().cuda_stream)
    finally:
        gc.enable()
    g.replay()
    torch.cuda.synchronize()
    assert bits_equal(o.cpu().numpy(), want)
    a.close()
    b.close()
