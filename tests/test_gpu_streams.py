"""Ordering of the per-camera device state across streams (include/rt.h,
ABI 4) and hipGraph capture of rt_render_async.

The context keeps per-camera state on the device (camera records, cone
records, the camera buffer).  Synchronous renders run on the context's own
stream, async renders on the caller's: every write of that state must come
after every render already enqueued that may read it, and every render after
the write it needs — with no host sync by the caller.  Each test interleaves
cameras and streams without a single synchronize between calls and compares
every output, bit for bit, with a cold context that renders each camera
alone (the reference's bits are pinned for those by test_gpu_parity.py)."""
from __future__ import annotations

import contextlib
import gc

import numpy as np
import pytest

import rt_amd
from conftest import bits_equal, scene

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")


@contextlib.contextmanager
def capture(g):
    """torch.cuda.graph without the garbage collector: a collection during
    the capture could finalize an unrelated context, whose rt_destroy
    synchronises streams — illegal while a stream is capturing."""
    gc.collect()
    gc.disable()
    try:
        with torch.cuda.graph(g):
            yield
    finally:
        gc.enable()


def _cameras(s, moves):
    out = []
    for dx, dz in moves:
        f = s.frame.copy()
        f.cam_pos[0] += dx
        f.cam_pos[2] += dz
        out.append(f)
    return out


def _cold(path, w, h, frames):
    """Each camera rendered by a fresh context (no state carried over)."""
    s = rt_amd.Scene(path, w, h, 0)
    want = []
    for f in frames:
        c = rt_amd.Context(0)
        c.upload(s)
        want.append(c.render_float(f))
        c.close()
    return want


@pytest.mark.parametrize("which", ["scene2", "heightfield"])
def test_async_sync_interleaved_without_host_sync(which, heightfield_path):
    """async(A) on s1, sync(B), async(B) on s1, async(A) on s2, ... in a loop,
    never synchronising: every image equals the cold context's."""
    path, w, h = (scene(2), 1920, 1080) if which == "scene2" else (heightfield_path, 960, 540)
    s = rt_amd.Scene(path, w, h, 0)
    cams = _cameras(s, [(0.0, 0.0), (9.5, -4.0), (-14.25, 6.5)])
    want = _cold(path, w, h, cams)
    ctx = rt_amd.Context(0)
    ctx.upload(s)
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    torch.cuda.synchronize()
    outs, host = [], []
    plan = []
    for k in range(4):
        a, b = k % 3, (k + 1) % 3
        plan += [("async", a, s1), ("sync", b, None), ("async", b, s1), ("async", a, s2), ("async", b, s2)]
    for kind, cam, st in plan:
        if kind == "sync":
            host.append((cam, ctx.render_float(cams[cam])))
        else:
            o = torch.empty((h, w, 3), dtype=torch.float32, device="cuda")
            # the allocation belongs to the current stream; keep it alive
            # until the end and tell the caching allocator about st
            o.record_stream(st)
            ctx.render_async(cams[cam], 0, o.data_ptr(), st.cuda_stream)
            outs.append((cam, o))
    ctx.sync()
    torch.cuda.synchronize()
    for i, (cam, o) in enumerate(outs):
        assert bits_equal(o.cpu().numpy(), want[cam]), f"async render {i} (camera {cam})"
    for i, (cam, img) in enumerate(host):
        assert bits_equal(img, want[cam]), f"sync render {i} (camera {cam})"


def test_async_prepass_seen_by_other_stream():
    """A camera first met by an async render is prepared on that stream; a
    render of the same camera on another stream right after must wait for it."""
    w, h = 640, 480
    s = rt_amd.Scene(scene(2), w, h, 0)
    cams = _cameras(s, [(3.0, 1.0), (-6.0, 2.0)])
    want = _cold(scene(2), w, h, cams)
    ctx = rt_amd.Context(0)
    ctx.upload(s)
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    torch.cuda.synchronize()
    outs = []
    for rep in range(3):
        for cam in (0, 1):
            for st in (s1, s2):
                o = torch.empty((h, w, 3), dtype=torch.float32, device="cuda")
                o.record_stream(st)
                ctx.render_async(cams[cam], 0, o.data_ptr(), st.cuda_stream)
                outs.append((cam, o))
    ctx.sync()
    for i, (cam, o) in enumerate(outs):
        assert bits_equal(o.cpu().numpy(), want[cam]), i


def test_prepare_camera_makes_async_fast():
    """rt_prepare_camera builds the camera buffer without rendering; the
    async render after it uses it (and renders the reference's bits)."""
    import ctypes

    w, h = 320, 240
    s = rt_amd.Scene(scene(2), w, h, 0)
    f = _cameras(s, [(2.5, 0.0)])[0]
    want = _cold(scene(2), w, h, [f])[0]
    ctx = rt_amd.Context(0)
    ctx.upload(s)
    ctx.prepare_camera(f)
    L = rt_amd.lib()
    L.rt_debug_cb_info.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
    info = (ctypes.c_double * 6)()
    assert L.rt_debug_cb_info(ctx._h, info, 6) == 0
    assert info[0] == 1.0 and info[1] > 0
    o = torch.empty((h, w, 3), dtype=torch.float32, device="cuda")
    ctx.render_async(f, 0, o.data_ptr(), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    assert bits_equal(o.cpu().numpy(), want)


# the refused capture leaves its graph empty, which torch warns about
@pytest.mark.filterwarnings("ignore:The CUDA Graph is empty")
def test_graph_capture_and_replay():
    """rt_render_async captured in a hipGraph (torch.cuda.CUDAGraph) replays
    the reference's image; capture of an unprepared camera is RT_E_STATE;
    a replay after other cameras were rendered and the captured one was
    prepared again is still exact (captured buffers are never freed)."""
    w, h = 480, 320
    s = rt_amd.Scene(scene(2), w, h, 0)
    cams = _cameras(s, [(0.0, 0.0), (11.0, -3.0), (-20.0, 9.0)])
    want = _cold(scene(2), w, h, cams)
    ctx = rt_amd.Context(0)
    ctx.upload(s)
    out = torch.zeros((h, w, 3), dtype=torch.float32, device="cuda")
    ctx.render_float(cams[0])  # prepares camera 0
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with capture(g):
        ctx.render_async(cams[0], 0, out.data_ptr(), torch.cuda.current_stream().cuda_stream)
    for _ in range(3):
        out.zero_()
        g.replay()
        torch.cuda.synchronize()
        assert bits_equal(out.cpu().numpy(), want[0])
    # an unprepared camera cannot be captured
    g2 = torch.cuda.CUDAGraph()
    with capture(g2):
        with pytest.raises(rt_amd.RtError) as e:
            ctx.render_async(cams[1], 0, out.data_ptr(), torch.cuda.current_stream().cuda_stream)
    assert e.value.code == -4
    # bigger frames of other cameras (buffers grow), then camera 0 again
    big = rt_amd.Scene(scene(2), 1280, 960, 0)
    ctx.render_float(_cameras(big, [(11.0, -3.0)])[0])
    assert bits_equal(ctx.render_float(cams[2]), want[2])
    ctx.prepare_camera(cams[0])
    out.zero_()
    g.replay()
    torch.cuda.synchronize()
    assert bits_equal(out.cpu().numpy(), want[0])


def test_options_round_trip_and_validation():
    ctx = rt_amd.Context(0)
    for name, v in (("light_buffer", 2), ("camera_buffer", 0), ("union_pretest", 0), ("lb_scale", 3.5),
                    ("dcov_near", 1.5), ("cb_inline_max_mb", 64)):
        ctx.set_option(name, v)
        assert ctx.get_option(name) == v
    for name, v in (("light_buffer", 3), ("lb_scale", -1), ("dcov_near", 0.5), ("cb_inline_max_mb", -2)):
        with pytest.raises(rt_amd.RtError):
            ctx.set_option(name, v)
    with pytest.raises(rt_amd.RtError):
        ctx.set_option(99, 1)
    with pytest.raises(rt_amd.RtError):
        ctx.set_far_ladder([4.0, 2.0])  # not rising
    with pytest.raises(rt_amd.RtError):
        ctx.set_far_ladder([2.0] * 9)
    ctx.set_far_ladder([2.0, 8.0])
    ctx.set_far_ladder(None)


@pytest.mark.parametrize("which,w,h,depth", [("scene2", 320, 240, 0), ("heightfield", 480, 320, 1),
                                             ("scene7", 200, 150, 3), ("scene9", 160, 120, 5)])
def test_sequence_matches_cold_renders(which, w, h, depth, heightfield_path):
    """rt_render_sequence_async over a camera path (yaw + translation per
    frame): every frame equals a fresh context's synchronous render."""
    path = heightfield_path if which == "heightfield" else scene(int(which[-1]))
    s = rt_amd.Scene(path, w, h, depth)
    frames = rt_amd.camera_path(s.frame, 5, yaw_deg=1.5, step=(2.0, 0.5, -1.0))
    cold = rt_amd.Context(0)
    cold.upload(s)
    want = [cold.render_float(f) for f in frames]
    ctx = rt_amd.Context(0)
    ctx.upload(s)
    out = torch.zeros((len(frames), h, w, 3), dtype=torch.float32, device="cuda")
    ctx.render_sequence_async(frames, 0, 0, out.data_ptr(), h * w * 12, torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    for i, f in enumerate(want):
        assert bits_equal(out[i].cpu().numpy(), f), i
    # the camera of the last frame is not left "current" by a sequence: a
    # synchronous render of it afterwards prepares it and is exact too
    assert bits_equal(ctx.render_float(frames[-1]), want[-1])


def test_sequences_on_two_streams_share_the_slots_safely():
    """Sequences of 7 frames (more than the 4 camera slots and internal
    streams a sequence keeps in flight) on two caller streams, back to back
    with no host sync: the second waits for the first's slots; every frame
    equals a fresh context's render."""
    w, h = 256, 192
    s = rt_amd.Scene(scene(2), w, h, 0)
    a = rt_amd.camera_path(s.frame, 7, yaw_deg=2.0, step=(1.5, 0.0, -2.0))
    b = rt_amd.camera_path(s.frame, 7, yaw_deg=-2.5, step=(-3.0, 0.5, 1.0))
    cold = rt_amd.Context(0)
    cold.upload(s)
    want_a = [cold.render(f) for f in a]
    want_b = [cold.render(f) for f in b]
    ctx = rt_amd.Context(0)
    ctx.upload(s)
    oa = torch.zeros((7, h, w, 4), dtype=torch.uint8, device="cuda")
    ob = torch.zeros((7, h, w, 4), dtype=torch.uint8, device="cuda")
    oc = torch.zeros((7, h, w, 4), dtype=torch.uint8, device="cuda")
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    torch.cuda.synchronize()
    for rep in range(3):
        ctx.render_sequence_async(a, oa.data_ptr(), h * w * 4, 0, 0, s1.cuda_stream)
        ctx.render_sequence_async(b, ob.data_ptr(), h * w * 4, 0, 0, s2.cuda_stream)
        ctx.render_sequence_async(a[::-1], oc.data_ptr(), h * w * 4, 0, 0, s1.cuda_stream)
        torch.cuda.synchronize()
        for i in range(7):
            assert np.array_equal(oa[i].cpu().numpy(), want_a[i]), (rep, "a", i)
            assert np.array_equal(ob[i].cpu().numpy(), want_b[i]), (rep, "b", i)
            assert np.array_equal(oc[i].cpu().numpy(), want_a[6 - i]), (rep, "c", i)
        oa.zero_(), ob.zero_(), oc.zero_()


def test_sequence_graph_replay_is_self_contained():
    """A camera path captured into a hipGraph replays the reference's frames
    even after other cameras and sequences were rendered on the context."""
    w, h = 320, 240
    s = rt_amd.Scene(scene(2), w, h, 0)
    frames = rt_amd.camera_path(s.frame, 6, yaw_deg=2.0, step=(1.5, 0.0, -2.0))
    other = rt_amd.camera_path(s.frame, 3, yaw_deg=-3.0, step=(-4.0, 1.0, 3.0))
    cold = rt_amd.Context(0)
    cold.upload(s)
    want = [cold.render(f) for f in frames]
    want_other = [cold.render(f) for f in other]
    ctx = rt_amd.Context(0)
    ctx.upload(s)
    out = torch.zeros((len(frames), h, w, 4), dtype=torch.uint8, device="cuda")
    tmp = torch.zeros((len(other), h, w, 4), dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with capture(g):
        ctx.render_sequence_async(frames, out.data_ptr(), h * w * 4, 0, 0, torch.cuda.current_stream().cuda_stream)
    for rep in range(3):
        out.zero_()
        g.replay()
        # other work on the same context between replays, no host sync
        ctx.render_async(other[rep], tmp[rep].data_ptr(), 0, torch.cuda.current_stream().cuda_stream)
        ctx.render_sequence_async(other, tmp.data_ptr(), h * w * 4, 0, 0, torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        for i, f in enumerate(want):
            assert np.array_equal(out[i].cpu().numpy(), f), (rep, i)
        for i, f in enumerate(want_other):
            assert np.array_equal(tmp[i].cpu().numpy(), f), (rep, i)
        assert np.array_equal(ctx.render(other[rep]), want_other[rep])


# the refused capture leaves its graph empty, which torch warns about
@pytest.mark.filterwarnings("ignore:The CUDA Graph is empty")
def test_capture_after_async_prepass_on_another_stream():
    """A camera first prepared by an async render on stream s1 (its state
    write pending there) cannot be captured on another stream — that would
    need a wait on an event outside the capture — until rt_sync; then it can,
    and the replay is exact."""
    w, h = 320, 240
    s = rt_amd.Scene(scene(2), w, h, 0)
    f = _cameras(s, [(5.0, -2.0)])[0]
    want = _cold(scene(2), w, h, [f])[0]
    ctx = rt_amd.Context(0)
    ctx.upload(s)
    s1 = torch.cuda.Stream()
    out = torch.zeros((h, w, 3), dtype=torch.float32, device="cuda")
    ctx.render_async(f, 0, out.data_ptr(), s1.cuda_stream)  # prepass on s1
    g = torch.cuda.CUDAGraph()
    with capture(g):
        with pytest.raises(rt_amd.RtError) as e:
            ctx.render_async(f, 0, out.data_ptr(), torch.cuda.current_stream().cuda_stream)
    assert e.value.code == -4
    ctx.sync()
    torch.cuda.synchronize()
    g2 = torch.cuda.CUDAGraph()
    with capture(g2):
        ctx.render_async(f, 0, out.data_ptr(), torch.cuda.current_stream().cuda_stream)
    out.zero_()
    g2.replay()
    torch.cuda.synchronize()
    assert bits_equal(out.cpu().numpy(), want)
