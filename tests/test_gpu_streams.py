"""Ordering of the per-camera device state across streams (include/rt.h,
ABI 4) and hipGraph capture of rt_render_async.

The context keeps per-camera state on the device (camera records, cone
records, the camera buffer).  Synchronous renders run on the context's own
stream, async renders on the caller's: every write of that state must come
after every render already enqueued that may read it, and every render after
the write it needs — with no host sync by the caller.  Each test interleaves
cameras and streams without a single synchronize between calls and compares
every output, bit for bit, with the reference's frame of its camera
(oracle/_ref with the frame's explicit camera words, tests/golden/cameras.json:
the moved cameras of tests/cameras.py at 480 x 270)."""
from __future__ import annotations

import contextlib
import gc

import pytest

import rt_amd
from conftest import CamRef, scene

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


@pytest.mark.parametrize("which,lc", [("scene2", 1), ("scene2", 0), ("hf", 1)])
def test_async_sync_interleaved_without_host_sync(which, lc, heightfield_path):
    """async(A) on s1, sync(B), async(B) on s1, async(A) on s2, ... in a loop,
    never synchronising: every image is the reference's (scene2: with the
    launch-camera records, and with the device camera state, lc 0)."""
    r = CamRef(which, heightfield_path)
    w, h = r.w, r.h
    cams = r.frames["cams"][:3]
    ctx = rt_amd.Context(0, launch_camera=lc)
    ctx.upload(r.scene)
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
        assert r.matches(o.cpu().numpy(), "cams", cam), f"async render {i} (camera {cam})"
    for i, (cam, img) in enumerate(host):
        assert r.matches(img, "cams", cam), f"sync render {i} (camera {cam})"


def test_async_prepass_seen_by_other_stream(heightfield_path):
    """A camera first met by an async render is prepared on that stream; a
    render of the same camera on another stream right after must wait for it
    (the device camera state: launch_camera 0)."""
    r = CamRef("scene2", heightfield_path)
    w, h = r.w, r.h
    cams = r.frames["cams"][1:3]
    ctx = rt_amd.Context(0, launch_camera=0)
    ctx.upload(r.scene)
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
        assert r.matches(o.cpu().numpy(), "cams", cam + 1), i


def test_prepare_camera_makes_async_fast(heightfield_path):
    """rt_prepare_camera builds the camera buffer without rendering; the
    async render after it uses it (and renders the reference's bits)."""
    import ctypes

    r = CamRef("scene2", heightfield_path)
    w, h = r.w, r.h
    f = r.frames["cams"][1]
    ctx = rt_amd.Context(0)
    ctx.upload(r.scene)
    ctx.prepare_camera(f)
    L = rt_amd.lib()
    L.rt_debug_cb_info.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
    info = (ctypes.c_double * 6)()
    assert L.rt_debug_cb_info(ctx._h, info, 6) == 0
    assert info[0] == 1.0 and info[1] > 0
    o = torch.empty((h, w, 3), dtype=torch.float32, device="cuda")
    ctx.render_async(f, 0, o.data_ptr(), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    assert r.matches(o.cpu().numpy(), "cams", 1)


# the refused capture leaves its graph empty, which torch warns about
@pytest.mark.filterwarnings("ignore:The CUDA Graph is empty")
def test_graph_capture_and_replay(heightfield_path):
    """rt_render_async captured in a hipGraph (torch.cuda.CUDAGraph) replays
    the reference's image; capture of an unprepared camera is RT_E_STATE
    (device camera state: launch_camera 0); a replay after other cameras were
    rendered and the captured one was prepared again is still exact (captured
    buffers are never freed)."""
    r = CamRef("scene2", heightfield_path)
    w, h = r.w, r.h
    cams = r.frames["cams"][:3]
    ctx = rt_amd.Context(0, launch_camera=0)
    ctx.upload(r.scene)
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
        assert r.matches(out.cpu().numpy(), "cams", 0)
    # an unprepared camera cannot be captured
    g2 = torch.cuda.CUDAGraph()
    with capture(g2):
        with pytest.raises(rt_amd.RtError) as e:
            ctx.render_async(cams[1], 0, out.data_ptr(), torch.cuda.current_stream().cuda_stream)
    assert e.value.code == -4
    # bigger frames of other cameras (buffers grow), then camera 0 again
    big = rt_amd.Scene(scene(2), 1280, 960, 0)
    ctx.render_float(_cameras(big, [(11.0, -3.0)])[0])
    assert r.matches(ctx.render_float(cams[2]), "cams", 2)
    ctx.prepare_camera(cams[0])
    out.zero_()
    g.replay()
    torch.cuda.synchronize()
    assert r.matches(out.cpu().numpy(), "cams", 0)


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


@pytest.mark.parametrize("which", ["scene2", "hf", "scene7", "scene9"])
@pytest.mark.parametrize("kind", ["path", "cams"])
def test_sequence_matches_reference(which, kind, heightfield_path):
    """rt_render_sequence_async over a camera path (yaw + translation per
    frame) or the turned / moved / widened cameras: every frame is the
    reference's (scene7 at depth 3, scene9 at depth 5: the bounce kernels)."""
    r = CamRef(which, heightfield_path)
    w, h = r.w, r.h
    frames = r.frames[kind]
    ctx = rt_amd.Context(0)
    ctx.upload(r.scene)
    out = torch.zeros((len(frames), h, w, 3), dtype=torch.float32, device="cuda")
    ctx.render_sequence_async(frames, 0, 0, out.data_ptr(), h * w * 12, torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    for i in range(len(frames)):
        assert r.matches(out[i].cpu().numpy(), kind, i), i
    # the camera of the last frame is not left "current" by a sequence: a
    # synchronous render of it afterwards prepares it and is exact too
    assert r.matches(ctx.render_float(frames[-1]), kind, len(frames) - 1)


def test_sequences_on_two_streams_share_the_slots_safely(heightfield_path):
    """Sequences of 6 frames (more than the 4 camera slots and internal
    streams a sequence keeps in flight) on two caller streams, back to back
    with no host sync: the second waits for the first's slots; every RGBA8
    frame is the reference's."""
    r = CamRef("scene2", heightfield_path)
    w, h = r.w, r.h
    a, b = r.frames["path"], r.frames["cams"]
    n = len(a)
    oa = torch.zeros((n, h, w, 4), dtype=torch.uint8, device="cuda")
    ob = torch.zeros((len(b), h, w, 4), dtype=torch.uint8, device="cuda")
    oc = torch.zeros((n, h, w, 4), dtype=torch.uint8, device="cuda")
    ctx = rt_amd.Context(0)
    ctx.upload(r.scene)
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    torch.cuda.synchronize()
    for rep in range(3):
        ctx.render_sequence_async(a, oa.data_ptr(), h * w * 4, 0, 0, s1.cuda_stream)
        ctx.render_sequence_async(b, ob.data_ptr(), h * w * 4, 0, 0, s2.cuda_stream)
        ctx.render_sequence_async(a[::-1], oc.data_ptr(), h * w * 4, 0, 0, s1.cuda_stream)
        torch.cuda.synchronize()
        for i in range(n):
            assert r.matches(oa[i].cpu().numpy(), "path", i), (rep, "a", i)
            assert r.matches(oc[i].cpu().numpy(), "path", n - 1 - i), (rep, "c", i)
        for i in range(len(b)):
            assert r.matches(ob[i].cpu().numpy(), "cams", i), (rep, "b", i)
        oa.zero_(), ob.zero_(), oc.zero_()


def test_sequence_graph_replay_is_self_contained(heightfield_path):
    """A camera path captured into a hipGraph replays the reference's frames
    even after other cameras and sequences were rendered on the context."""
    r = CamRef("scene2", heightfield_path)
    w, h = r.w, r.h
    frames = r.frames["path"]
    other = r.frames["cams"][1:4]
    ctx = rt_amd.Context(0)
    ctx.upload(r.scene)
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
        for i in range(len(frames)):
            assert r.matches(out[i].cpu().numpy(), "path", i), (rep, i)
        for i in range(len(other)):
            assert r.matches(tmp[i].cpu().numpy(), "cams", i + 1), (rep, i)
        assert r.matches(ctx.render(other[rep]), "cams", rep + 1)


# the refused capture leaves its graph empty, which torch warns about
@pytest.mark.filterwarnings("ignore:The CUDA Graph is empty")
def test_launch_camera_captures_any_camera(heightfield_path):
    """With the camera records in the launch (tiny scenes) there is no
    per-camera device state: a never-rendered camera is captured directly
    and every replay — after other cameras on other streams — is exact."""
    r = CamRef("scene2", heightfield_path)
    w, h = r.w, r.h
    cams = r.frames["cams"]
    ctx = rt_amd.Context(0)
    ctx.upload(r.scene)
    outs = [torch.zeros((h, w, 3), dtype=torch.float32, device="cuda") for _ in cams]
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with capture(g):
        for f, o in zip(cams, outs):
            ctx.render_async(f, 0, o.data_ptr(), torch.cuda.current_stream().cuda_stream)
    s1 = torch.cuda.Stream()
    tmp = torch.zeros((h, w, 3), dtype=torch.float32, device="cuda")
    for rep in range(2):
        for o in outs:
            o.zero_()
        g.replay()
        ctx.render_async(r.frames["path"][rep + 1], 0, tmp.data_ptr(), s1.cuda_stream)
        torch.cuda.synchronize()
        for i, o in enumerate(outs):
            assert r.matches(o.cpu().numpy(), "cams", i), (rep, i)
        assert r.matches(tmp.cpu().numpy(), "path", rep + 1)


def test_capture_after_async_prepass_on_another_stream(heightfield_path):
    """A camera first prepared by an async render on stream s1 (its state
    write pending there) cannot be captured on another stream — that would
    need a wait on an event outside the capture — until rt_sync; then it can,
    and the replay is exact."""
    r = CamRef("scene2", heightfield_path)
    w, h = r.w, r.h
    f = r.frames["cams"][2]
    ctx = rt_amd.Context(0, launch_camera=0)
    ctx.upload(r.scene)
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
    assert r.matches(out.cpu().numpy(), "cams", 2)
