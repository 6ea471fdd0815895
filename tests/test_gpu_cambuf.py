"""The camera buffer built on the stream (round 3, rt_cambuf.h) and moved
cameras against the reference.

* every list equals brute force — each tile with a list against every
  triangle, the camera wave test of the per-wave path (rt_debug_cb_verify) —
  for the reference's cameras and for moved, yawed, pitched, rolled and
  wide-angle ones, odd frame sizes, slabs and bands;
* every moved camera of tests/cameras.py (turned / moved / widened cameras
  and a camera path, on scene2, scene7 at depth 3, scene9 at depth 5 and the
  50k-triangle heightfield) renders the reference's frame bit for bit —
  oracle/_ref run with the frame's explicit camera words
  (tests/golden/cameras.json) — through the synchronous path, and through
  rt_render_async of a moving camera (which builds the buffer itself), the
  sequence path's per-slot buffers and two interleaved streams;
* a capacity too small for the lists (RT_OPT_CB_CAPACITY) sends the tiles
  that do not fit down the per-wave path: the same (reference) image.
The reference recomputes its camera for every frame (Scene.cpp:674 ->
:624-660); the lists only replace the per-wave culling of the camera rays
(ObtenirCouleur, Scene.cpp:1705-1738)."""
from __future__ import annotations

import ctypes

import pytest

import cameras
import rt_amd
from conftest import CamRef, bits_equal, scene

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


@pytest.mark.parametrize("which,w,h", [("scene2", 640, 360), ("scene2", 333, 197), ("scene3", 320, 240),
                                       ("scene1", 160, 120),
                                       ("hf", 640, 360), ("hf", 250, 131)])
def test_lists_equal_brute_force(heightfield_path, which, w, h):
    path = heightfield_path if which == "hf" else scene(int(which[-1]))
    s = rt_amd.Scene(path, w, h, 0)
    ctx = rt_amd.Context(0)
    ctx.upload(s)
    for i, f in enumerate(cameras.cameras(s.frame)):
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
    f = cameras.turned(s.frame, cameras.rot(1, 5.0), (1.0, 0.0, 1.0))
    if rows:
        f.row_begin, f.row_end = rows
    if bands:
        f.band_rows, f.band_count, f.band_index = bands
    ctx.prepare_camera(f)
    bad, pairs, listed = _verify(ctx)
    assert bad == 0 and listed > 0
    ctx.close()


@pytest.mark.parametrize("which,lc", [("scene2", 1), ("scene2", 0), ("scene7", 1), ("scene9", 1), ("hf", 1)])
@pytest.mark.parametrize("kind", ["cams", "path", "moving"])
def test_moved_cameras_equal_reference(heightfield_path, which, lc, kind):
    """Synchronous renders (float32 RGB and RGBA8) of every moved camera of
    the set, one context for all of them, against _ref's frames (scene2 with
    the launch-camera records and with the device camera buffer)."""
    r = CamRef(which, heightfield_path)
    ctx = rt_amd.Context(0, launch_camera=lc)
    ctx.upload(r.scene)
    for i, f in enumerate(r.frames[kind]):
        assert r.matches(ctx.render_float(f), kind, i), (which, kind, i)
        assert r.matches(ctx.render(f), kind, i), (which, kind, i, "rgba8")
    ctx.close()


@pytest.mark.parametrize("which,cbopt,lc", [("scene2", 1, 1), ("scene2", 1, 0), ("scene2", 2, 0), ("hf", 2, 1),
                                           ("hf", 1, 1), ("scene7", 1, 1), ("scene9", 1, 1)])
@pytest.mark.parametrize("kind", ["path", "moving"])
def test_async_moving_camera_matches_reference(heightfield_path, which, cbopt, lc, kind):
    """rt_render_async of a camera path, no host sync between frames: each
    new camera's records travel with the launch (scene2, lc 1), or its device
    state (and, with camera_buffer 2 or where it pays, its camera buffer) is
    built on the caller's stream; every frame is the reference's."""
    r = CamRef(which, heightfield_path)
    frames = r.frames[kind]
    ctx = rt_amd.Context(0, camera_buffer=cbopt, launch_camera=lc)
    ctx.upload(r.scene)
    st = torch.cuda.current_stream()
    outs = []
    for f in frames:
        o = torch.empty((r.h, r.w, 3), dtype=torch.float32, device="cuda")
        ctx.render_async(f, 0, o.data_ptr(), st.cuda_stream)
        outs.append(o)
    torch.cuda.synchronize()
    if cbopt == 2 and r.depth == 0 and not (lc and which == "scene2"):
        info = _cb_info(ctx)
        assert info[1] > 0  # the last camera's buffer, built by the async render
        if info[0] == 1.0:
            assert _verify(ctx)[0] == 0
    for i, o in enumerate(outs):
        assert r.matches(o.cpu().numpy(), kind, i), (which, i)
    ctx.close()


def test_moving_c3_full_size_matches_reference(heightfield_path):
    """C3 (the 50k heightfield at 1920x1080, depth 0) under the bench's
    translated camera (tests/cameras.py moving(), the per-frame move of a
    display loop, Main.cpp:229-250 -> LancerRayons, Scene.cpp:674): seven
    frames through rt_render_async (new cameras below 4 Mpx: the per-wave
    path; a camera repeated once builds its lists), through
    rt_render_sequence_async (the slots' own state) and synchronously (the
    camera buffer of each camera); frames 3 and 6 against _ref's whole-frame
    digests (tests/golden/cameras.json)."""
    import hashlib

    import numpy as np

    from conftest import cam_golden

    name, w, h, d, idx = cameras.MOVING_FULL
    s = rt_amd.Scene(heightfield_path, w, h, d)
    frames = cameras.moving(s.frame, max(idx) + 1)
    g = cam_golden()

    def key(i):
        return f"{name}_{w}x{h}_d{d}_moving{i}"

    def sha(a):
        return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()

    for i in idx:
        assert g[key(i)]["camera_words_sha256"] == cameras.words_sha(frames[i])
    ctx = rt_amd.Context(0)
    ctx.upload(s)
    st = torch.cuda.current_stream().cuda_stream
    outs = []
    for i, f in enumerate(frames):
        o = torch.empty((h, w, 3), dtype=torch.float32, device="cuda")
        ctx.render_async(f, 0, o.data_ptr(), st)
        outs.append(o)
        if i in idx:  # the same camera again: its second frame builds and walks its lists
            o2 = torch.empty((h, w, 3), dtype=torch.float32, device="cuda")
            ctx.render_async(f, 0, o2.data_ptr(), st)
            outs.append(o2)
    torch.cuda.synchronize()
    k = 0
    for i in range(len(frames)):
        reps = 2 if i in idx else 1
        for r_ in range(reps):
            if i in idx:
                assert sha(outs[k].cpu().numpy()) == g[key(i)]["rgb_f32_sha256"], ("async", i, r_)
            k += 1
    ring = torch.empty((len(frames), h, w, 4), dtype=torch.uint8, device="cuda")
    ctx.render_sequence_async(frames, ring.data_ptr(), h * w * 4, 0, 0, st)
    torch.cuda.synchronize()
    for i in idx:
        assert sha(ring[i].cpu().numpy()) == g[key(i)]["rgba8_sha256"], ("sequence", i)
        assert sha(ctx.render_float(frames[i])) == g[key(i)]["rgb_f32_sha256"], ("sync", i)
    ctx.close()


@pytest.mark.parametrize("cap", [1, 3000, 20000])
def test_overflowing_capacity_renders_the_same(heightfield_path, cap):
    r = CamRef("hf", heightfield_path)
    ctx = rt_amd.Context(0, cb_capacity=cap)
    ctx.upload(r.scene)
    for i, f in enumerate(r.frames["path"][:3]):
        assert r.matches(ctx.render_float(f), "path", i), i
        bad, pairs, listed = _verify(ctx)
        assert bad == 0
        info = _cb_info(ctx)
        assert info[9] == cap
        if info[1] > cap:  # some tiles did not fit: they render by the per-wave path
            assert listed < (r.w // 8 + 1) * (r.h // 8 + 1)
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


@pytest.mark.parametrize("which,cbopt,lc", [("hf", 1, 1), ("hf", 2, 1), ("scene2", 2, 0), ("scene2", 1, 1)])
def test_sequence_slots_build_camera_buffers(heightfield_path, which, cbopt, lc):
    r = CamRef(which, heightfield_path)
    frames = r.frames["path"]
    ctx = rt_amd.Context(0, camera_buffer=cbopt, launch_camera=lc)
    ctx.upload(r.scene)
    ring = torch.empty((len(frames), r.h, r.w, 3), dtype=torch.float32, device="cuda")
    for rep in range(2):  # the second call reuses the slots' buffers
        ring.zero_()
        ctx.render_sequence_async(frames, 0, 0, ring.data_ptr(), r.h * r.w * 12,
                                  torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        for i in range(len(frames)):
            assert r.matches(ring[i].cpu().numpy(), "path", i), (rep, i)
    ctx.close()


@pytest.mark.parametrize("cbopt", [2, 1])
def test_async_two_streams_interleaved(heightfield_path, cbopt):
    """Renders of alternating and repeated cameras on two streams, with no
    host sync between calls and a synchronous render in the middle: every
    output is the reference's frame of its camera (camera_buffer 1: a new
    camera per-wave, its repeat on the same stream building the lists)."""
    r = CamRef("hf", heightfield_path)
    cams = r.frames["path"][:4]
    ctx = rt_amd.Context(0, camera_buffer=cbopt)
    ctx.upload(r.scene)
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    order = [0, 1, 0, 2, 3, 3, 1, 2, 0, 3]
    outs = []
    for i, k in enumerate(order):
        st = s1 if i % 2 == 0 else s2
        o = torch.empty((r.h, r.w, 3), dtype=torch.float32, device="cuda")
        o.record_stream(st)
        ctx.render_async(cams[k], 0, o.data_ptr(), st.cuda_stream)
        outs.append((k, o))
        if i == 5:  # a synchronous render in the middle (the context's own state)
            assert r.matches(ctx.render_float(cams[1]), "path", 1)
    ctx.sync()
    for i, (k, o) in enumerate(outs):
        assert r.matches(o.cpu().numpy(), "path", k), (i, k)
    ctx.close()


def test_sequence_capture_builds_buffers_inside_the_graph(heightfield_path):
    """a sequence captured into a hipGraph whose slots build their
    camera buffers inside the capture (camera_buffer 2), replayed after
    uncaptured sequences that grow or reuse the slot buffers (a larger
    frame): every replay is the reference's camera path."""
    import gc

    r = CamRef("hf", heightfield_path)
    frames = r.frames["path"]
    ctx = rt_amd.Context(0, camera_buffer=2)
    ctx.upload(r.scene)
    st = torch.cuda.current_stream()
    out = torch.zeros((len(frames), r.h, r.w, 3), dtype=torch.float32, device="cuda")
    ctx.render_sequence_async(frames, 0, 0, out.data_ptr(), r.h * r.w * 12, st.cuda_stream)  # sizes the slots
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    gc.collect()
    gc.disable()
    try:
        with torch.cuda.graph(g):
            ctx.render_sequence_async(frames, 0, 0, out.data_ptr(), r.h * r.w * 12,
                                      torch.cuda.current_stream().cuda_stream)
    finally:
        gc.enable()
    big = rt_amd.Scene(r.path, 2 * r.w, 2 * r.h, 0)
    bframes = cameras.path(big.frame)
    tmp = torch.zeros((len(bframes), 2 * r.h, 2 * r.w, 3), dtype=torch.float32, device="cuda")
    for rep in range(2):
        out.zero_()
        g.replay()
        torch.cuda.synchronize()
        for i in range(len(frames)):
            assert r.matches(out[i].cpu().numpy(), "path", i), (rep, i)
        # uncaptured sequences in between: bigger frames grow the slots' arrays
        ctx.render_sequence_async(bframes, 0, 0, tmp.data_ptr(), 4 * r.h * r.w * 12, st.cuda_stream)
        ctx.render_sequence_async(frames[::-1], 0, 0, out.data_ptr(), r.h * r.w * 12, st.cuda_stream)
        torch.cuda.synchronize()
        for i in range(len(frames)):
            assert r.matches(out[len(frames) - 1 - i].cpu().numpy(), "path", i), (rep, "uncaptured", i)
    ctx.close()


def test_candidate_pairs_past_32_bits(tmp_path):
    """the pair offsets are 32-bit.  10,000 triangles that are
    never culled (edges > 110 units: the reference's det can be too inexact at
    its 0.01 gate, so no cone record) have whole-film boxes; at 7680 x 4320
    (518,400 tiles) that is 5.2 G candidate pairs > 2^32 - 1.  The build must
    flag every tile (per-wave path)
    instead of wrapping the offsets, and a slab of the frame must render
    like a context without the camera buffer."""
    import numpy as np

    rng = np.random.default_rng(7)
    lines = ["background: 10 20 30", "origin: 0 0 400", "eye: 0 0 0", "up: 0 1 0",
             "Lumiere:", "position: 0 300 300", "intens: 1", "color: 255 255 255"]
    for k in range(10000):
        c = rng.uniform(-60, 60, 3)
        lines += ["Poly:", "color: 200 100 50"]
        for i, d in enumerate(([-120, -5, -900], [120, -5, -900], [0, 80, -900])):
            p = c + np.array(d) + rng.uniform(-1, 1, 3)
            lines.append(f"point: {i} {p[0]:.2f} {p[1]:.2f} {p[2]:.2f}")
    path = tmp_path / "big_tris.dat"
    path.write_text("\n".join(lines) + "\n")
    s = rt_amd.Scene(str(path), 7680, 4320, 0)
    ctx = rt_amd.Context(0)
    ctx.upload(s)
    ctx.prepare_camera(s.frame)
    info = _cb_info(ctx, 11)
    assert info[10] == 1.0, info  # past 2^32 - 1: every tile flagged
    assert _verify(ctx)[2] == 0   # no tile has a list
    f = s.frame.copy()
    f.row_begin, f.row_end = 2160, 2168
    ref = rt_amd.Context(0, camera_buffer=0)
    ref.upload(s)
    assert bits_equal(ctx.render_float(f), ref.render_float(f))
    ctx.close()
    ref.close()


def test_launch_camera_mask_modes_on_one_stream(heightfield_path):
    """The launch-camera path's three mask modes on one stream (rt_camhost.h
    tiny_masks): camera A's first frame computes its tile masks, its second
    computes and stores them, its third reads them; a new camera B computes
    without storing, so A's stored masks stay valid and A's next frame reads
    them; B's second frame then overwrites them with B's.  Every frame is the
    reference's (scene2 moved cameras, RGBA8 and float RGB)."""
    r = CamRef("scene2", heightfield_path)
    cams = r.frames["cams"]
    order = [0, 0, 0, 1, 0, 0, 1, 1, 1, 0]
    ctx = rt_amd.Context(0, launch_camera=1)
    ctx.upload(r.scene)
    st = torch.cuda.Stream()
    outs = []
    with torch.cuda.stream(st):
        for i, k in enumerate(order):
            if i % 2:
                o = torch.empty((r.h, r.w, 4), dtype=torch.uint8, device="cuda")
                ctx.render_async(cams[k], o.data_ptr(), 0, st.cuda_stream)
            else:
                o = torch.empty((r.h, r.w, 3), dtype=torch.float32, device="cuda")
                ctx.render_async(cams[k], 0, o.data_ptr(), st.cuda_stream)
            outs.append((k, o))
    st.synchronize()
    for i, (k, o) in enumerate(outs):
        assert r.matches(o.cpu().numpy(), "cams", k), (i, k)
    ctx.close()


@pytest.mark.parametrize("kind", ["cams", "path"])
def test_async_repeat_builds_the_sorted_lists(heightfield_path, kind):
    """An async frame repeating the previous async frame's camera builds the
    camera buffer (the heightfield at 480x270 is below the 4 Mpx at which a
    new camera's async frame builds it): after each camera's second frame the
    buffer is that camera's and equals brute force, and every frame is the
    reference's."""
    r = CamRef("hf", heightfield_path)
    ctx = rt_amd.Context(0)
    ctx.upload(r.scene)
    # synchronous renders first: they read each build's size back, so the
    # capacity fits every camera (an async build that overflows is flagged
    # and rebuilt at its camera's next frame, by design)
    for i, f in enumerate(r.frames[kind][:4]):
        assert r.matches(ctx.render_float(f), kind, i), i
    st = torch.cuda.current_stream()
    for i, f in enumerate(r.frames[kind][:4]):
        for rep in range(2):
            o = torch.empty((r.h, r.w, 3), dtype=torch.float32, device="cuda")
            ctx.render_async(f, 0, o.data_ptr(), st.cuda_stream)
            torch.cuda.synchronize()
            assert r.matches(o.cpu().numpy(), kind, i), (i, rep)
        info = _cb_info(ctx)
        assert info[0] == 1.0, i  # built by the repeat
        bad, pairs, listed = _verify(ctx)
        assert bad == 0 and listed > 0, (i, bad)
    ctx.close()
