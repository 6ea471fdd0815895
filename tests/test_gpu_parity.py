"""Parity of the HIP path (librt_amd.so through the C ABI) with the reference.

Checkers: the golden fixtures (made from the reference's own sources, see
tests/golden/make_golden.py) and the oracle restatement.  Bar: RGBA8 within
1 LSB per channel (north star); in practice the float32 RGB is compared
bit-for-bit and every deviation is reported (PHONG_ULP below is the only
allowance: ocml powf vs glibc powf on Phong highlights)."""
from __future__ import annotations

import hashlib
import os

import numpy as np
import pytest

import rt_amd
from conftest import REPO, bits_equal, rgba8, scene, ulp_diff

pytestmark = pytest.mark.gpu

# Only scene4 has a specular (Phong) term -> powf.  glibc's powf and ROCm's
# ocml powf are both faithfully (not correctly) rounded, so a highlight may
# differ by an ulp or two in float; RGBA8 must still be within 1 LSB.
PHONG_SCENES = {4}
PHONG_ULP = 8


@pytest.fixture(scope="module")
def ctx():
    return rt_amd.Context(0)


def render(ctx, path, w, h, depth, as_float=True, rows=None, flags=0):
    s = rt_amd.Scene(path, w, h, depth)
    ctx.upload(s)
    f = s.frame.copy()
    f.flags = flags
    if rows:
        f.row_begin, f.row_end = rows
    return ctx.render_float(f) if as_float else ctx.render(f)


def check(got, want, i):
    if i in PHONG_SCENES:
        assert ulp_diff(got, want) <= PHONG_ULP
    else:
        assert bits_equal(got, want), f"max |d| {np.abs(got - want).max()} ulps {ulp_diff(got, want)}"
    assert np.abs(rgba8(got).astype(int) - rgba8(want).astype(int)).max() <= 1


@pytest.mark.parametrize("i", range(1, 10))
@pytest.mark.parametrize("depth", [0, 1, 3, 5])
def test_scene_images(ctx, golden_images, i, depth):
    got = render(ctx, scene(i), 64, 48, depth)
    check(got, golden_images[f"scene{i}_64x48_d{depth}"], i)


@pytest.mark.parametrize("wh", [(1, 1), (13, 7), (67, 33)])
def test_ragged_sizes(ctx, golden_images, wh):
    w, h = wh
    check(render(ctx, scene(5), w, h, 3), golden_images[f"scene5_{w}x{h}_d3"], 5)


def test_rgba8_is_quantised_float(ctx):
    for i in (1, 4, 7):
        s = rt_amd.Scene(scene(i), 96, 64, 5)
        ctx.upload(s)
        f = ctx.render_float(s.frame)
        q = ctx.render(s.frame)
        assert np.array_equal(q, rgba8(f))


@pytest.mark.parametrize("name,i,w,h,depth", [
    ("scene2_1080p_d0", 2, 1920, 1080, 0),
    ("scene2_1080p_d3", 2, 1920, 1080, 3),
    ("scene7_2160p_d5", 7, 3840, 2160, 5),
    ("scene9_2160p_d5", 9, 3840, 2160, 5),
])
def test_big_frame_windows(ctx, golden_images, name, i, w, h, depth):
    full = render(ctx, scene(i), w, h, depth)
    keys = [k for k in golden_images.files if k.startswith(name + "_win_")]
    assert keys
    for k in keys:
        r0, r1, c0, c1 = map(int, k.rsplit("_win_", 1)[1].split("_"))
        check(full[r0:r1, c0:c1], golden_images[k], i)


@pytest.fixture(scope="module")
def c3_column():
    """_ref windows down the whole C3 frame (tests/golden/make_c3_column_golden.py)."""
    return np.load(os.path.join(REPO, "tests", "golden", "c3_column.npz"))


def _hf_windows(golden_images, c3_column):
    out = [(k, golden_images[k]) for k in golden_images.files if k.startswith("hf_1080p_d1_win_")]
    out += [(k, c3_column[k]) for k in c3_column.files]
    assert len(out) > 40
    return out


def test_heightfield_windows(ctx, golden_images, c3_column, heightfield_path):
    full = render(ctx, heightfield_path, 1920, 1080, 1)
    for k, want in _hf_windows(golden_images, c3_column):
        r0, r1, c0, c1 = map(int, k.rsplit("_win_", 1)[1].split("_"))
        check(full[r0:r1, c0:c1], want, 0)


def test_heightfield_without_plane_silhouette(ctx, tmp_path):
    """The mesh against the sky (no ground plane): waves on its silhouette
    shade only some lanes, so the big-list kernel's LDS-staged light-buffer
    walk runs on partial waves there.  120 _ref windows
    (tests/golden/make_hf_sky_golden.py), 7 of them across the silhouette."""
    from rt_amd import synth

    lines = synth.heightfield_dat().split("\n")
    i = lines.index("Plane: plane_1")
    j = i + 1
    while j < len(lines) and lines[j].startswith(" "):
        j += 1
    path = tmp_path / "hf_sky.dat"
    path.write_text("\n".join(lines[:i] + lines[j:]))
    full = render(ctx, str(path), 1920, 1080, 1)
    bg = np.array([0.0, 0.0, 150 / 255.0], dtype=np.float32)
    mixed = 0
    with np.load(os.path.join(REPO, "tests", "golden", "hf_sky.npz")) as z:
        for k in z.files:
            r0, r1, c0, c1 = map(int, k.rsplit("_win_", 1)[1].split("_"))
            want = z[k]
            check(full[r0:r1, c0:c1], want, 0)
            sky = int((np.abs(want.reshape(-1, 3) - bg).sum(1) < 1e-6).sum())
            mixed += 0 < sky < want.shape[0] * want.shape[1]
    assert mixed >= 5


def test_small_big_list_frames_walk_two_entries_per_round(golden_images, c3_column, heightfield_path):
    """RT_OPT_LB_UNROLL: under 4 Mpx the big-list kernel walks the light
    buffer's per-lane lists two entries per round (WAVE bit 2048): C3 against
    the reference's windows, the same bits as the one-entry walk, and the
    kernel label names the variant that ran."""
    a, b = rt_amd.Context(0), rt_amd.Context(0, lb_unroll=0)
    s = rt_amd.Scene(heightfield_path, 1920, 1080, 1)
    for c in (a, b):
        c.upload(s)
    full = a.render_float(s.frame)
    assert a.stats().kernel == "rt_trace_kernel<0,1,2062>", a.stats().kernel
    assert bits_equal(full, b.render_float(s.frame))
    assert b.stats().kernel == "rt_trace_kernel<0,1,14>", b.stats().kernel
    for k, want in _hf_windows(golden_images, c3_column):
        r0, r1, c0, c1 = map(int, k.rsplit("_win_", 1)[1].split("_"))
        check(full[r0:r1, c0:c1], want, 0)
    f = s.frame.copy()
    f.cam_pos[0] += 3.0  # a new camera: the per-wave path's variant (no camera buffer yet)
    torch = pytest.importorskip("torch")
    o = torch.empty((1080, 1920, 3), dtype=torch.float32, device="cuda")
    a.render_async(f, 0, o.data_ptr(), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    assert bits_equal(o.cpu().numpy(), b.render_float(f))


@pytest.mark.parametrize("mode,stripe", [(0, 0), (2, 0), (2, 3), (2, 4), (3, 0)])
def test_xcd_deal_modes_render_the_same(golden_images, c3_column, heightfield_path, mode, stripe):
    """RT_OPT_XCD_DEAL: the big-list kernels' tile-to-XCD dealing (padded
    grids in modes 2 and 3) only moves tiles between workgroups: C3 at full
    size against the reference's windows, a slab off the tile grid, a band
    set and the reflective mesh's wavefront level 0 — all equal to mode 1
    (stripes of 3 and 4 tiles: 240 tile columns are not a multiple of 24)."""
    from rt_amd import synth

    a, b = rt_amd.Context(0, xcd_deal=1), rt_amd.Context(0, xcd_deal=mode, xcd_stripe=stripe)
    s = rt_amd.Scene(heightfield_path, 1920, 1080, 1)
    for c in (a, b):
        c.upload(s)
    full = b.render_float(s.frame)
    for k, want in _hf_windows(golden_images, c3_column):
        r0, r1, c0, c1 = map(int, k.rsplit("_win_", 1)[1].split("_"))
        check(full[r0:r1, c0:c1], want, 0)
    frames = []
    f = s.frame.copy()
    f.row_begin, f.row_end = 203, 1077
    frames.append(f)
    f = s.frame.copy()
    f.band_rows, f.band_count, f.band_index = 16, 3, 2
    frames.append(f)
    f = s.frame.copy()
    f.width, f.height, f.row_end = 1000, 1000, 1000  # tiles not a multiple of 8 either way
    f.inv_w, f.inv_h = 1.0 / 1000, 1.0 / 1000
    frames.append(f)
    for f in frames:
        assert bits_equal(b.render_float(f), a.render_float(f))
    hf = synth.write_heightfield("/tmp/rt_amd_xcd_hfr.dat", cols=60, rows=30, reflect=0.5)
    s2 = rt_amd.Scene(hf, 1920, 1080, 3)
    for c in (a, b):
        c.upload(s2)
    assert bits_equal(b.render_float(s2.frame), a.render_float(s2.frame))


@pytest.mark.parametrize("near,far", [(1.5, [64.0]), (1.5, [1.6]), (1.05, [1.1, 1.3, 2.0, 4.0]),
                                      (1.02, [1.05, 1.1, 1.2, 1.4, 1.8, 2.5, 4.0, 8.0]), (1.25, [])])
def test_heightfield_far_buffer(golden_images, c3_column, heightfield_path, near, far):
    """Big lists: lanes beyond the light buffer's distance walk the light's
    far buffers level by level, lanes beyond the last the per-lane loop over
    every triangle.  The distances shrunk (RT_OPT_DCOV_NEAR, rt_set_far_ladder,
    x the farthest triangle) so that many lanes take every level: still the
    reference's bits."""
    c = rt_amd.Context(0, dcov_near=near, far_ladder=far)
    full = render(c, heightfield_path, 1920, 1080, 1)
    for k, want in _hf_windows(golden_images, c3_column):
        r0, r1, c0, c1 = map(int, k.rsplit("_win_", 1)[1].split("_"))
        check(full[r0:r1, c0:c1], want, 0)


def test_scene2_1080p_digest_and_counts(ctx, digests):
    full = render(ctx, scene(2), 1920, 1080, 0, flags=rt_amd.FLAG_STATS)
    st = ctx.stats()
    assert hashlib.sha256(full.tobytes()).hexdigest() == digests["scene2_1920x1080_d0_rgb_f32_sha256"]
    assert hashlib.sha256(rgba8(full).tobytes()).hexdigest() == digests["scene2_1920x1080_d0_rgba8_sha256"]
    # ray counts of the reference's CPU loop at this config (gprof)
    assert st.primary_rays == 2_073_600
    assert st.shadow_rays == 5_618_440
    assert st.bounce_rays == 0


def test_timed_kernel_label_after_three_renders():
    """bench.py's roofline.kernel is rt_stats.kernel of a timed launch: for
    the C2 camera on one stream the first frame computes the tile masks
    (<0,1,101>), the second stores them (<0,1,229>), every later frame reads
    them (<0,1,37>, the kernel rocprof times in the bench's loop)."""
    torch = pytest.importorskip("torch")
    s = rt_amd.Scene(scene(2), 1920, 1080, 3)
    c = rt_amd.Context(0)
    c.upload(s)
    out = torch.empty((1080, 1920, 4), dtype=torch.uint8, device="cuda")
    stream = torch.cuda.current_stream().cuda_stream
    labels = []
    for _ in range(4):
        c.render_async(s.frame, out.data_ptr(), 0, stream)
        labels.append(c.stats().kernel)
    torch.cuda.synchronize()
    assert labels == ["rt_trace_tiny<0,1,101>", "rt_trace_tiny<0,1,229>",
                      "rt_trace_tiny<0,1,37>", "rt_trace_tiny<0,1,37>"], labels


@pytest.mark.parametrize("i,depth", [(2, 0), (7, 3), (1, 0)])
def test_counted_kernel_renders_the_same(ctx, i, depth):
    """The RT_FLAG_STATS launch runs the COUNT kernel variant: same image, and
    its test tallies lie between 0 and the brute-force count."""
    plain = render(ctx, scene(i), 320, 200, depth)
    counted = render(ctx, scene(i), 320, 200, depth, flags=rt_amd.FLAG_STATS)
    st = ctx.stats()
    assert bits_equal(plain, counted)
    s = rt_amd.Scene(scene(i), 320, 200, depth)
    n = s.n_surfaces
    tests = st.triangle_tests + st.plane_tests + st.quadric_tests
    assert 0 < tests <= (st.primary_rays + st.bounce_rays + st.shadow_rays) * n * 64


def test_scene2_depth_inert_full_size(ctx):
    """C4 property at full size: scene2 has no Kr/Kt, so depth 5 == depth 0."""
    a = render(ctx, scene(2), 3840, 2160, 5, as_float=False)
    b = render(ctx, scene(2), 3840, 2160, 0, as_float=False)
    assert np.array_equal(a, b) and (a[..., 3] == 255).all()


@pytest.mark.parametrize("nslabs", [2, 3, 8])
def test_row_slabs_reassemble(ctx, nslabs):
    """The multi-GPU partition: slabs rendered separately == the full frame."""
    w, h = 200, 150
    s = rt_amd.Scene(scene(7), w, h, 3)
    ctx.upload(s)
    full = ctx.render(s.frame)
    parts = []
    for r in range(nslabs):
        f = s.frame.copy()
        f.row_begin, f.row_end = r * h // nslabs, (r + 1) * h // nslabs
        parts.append(ctx.render(f))
    assert np.array_equal(np.concatenate(parts, 0), full)


@pytest.mark.gpu
@pytest.mark.parametrize("sc,depth,w,h", [(2, 3, 200, 150), (7, 3, 120, 90), (9, 5, 96, 70)])
@pytest.mark.parametrize("nranks,band_rows", [(2, 16), (3, 16), (8, 16), (3, 32)])
def test_row_bands_reassemble(ctx, sc, depth, w, h, nranks, band_rows):
    """Cyclic row bands (rt_frame.band_rows, ABI 3): every rank's packed band
    set, un-permuted, == the full frame (float RGB, bit for bit)."""
    s = rt_amd.Scene(scene(sc), w, h, depth)
    ctx.upload(s)
    full = ctx.render_float(s.frame)
    got = np.full_like(full, np.nan)
    for r in range(nranks):
        f = s.frame.copy()
        f.band_rows, f.band_count, f.band_index = band_rows, nranks, r
        part = ctx.render_float(f)
        assert part.shape[0] == rt_amd.band_rows(h, band_rows, nranks, r)
        for q in range(part.shape[0] // band_rows):
            a = (q * nranks + r) * band_rows
            e = min(h, a + band_rows)
            got[a:e] = part[q * band_rows: q * band_rows + (e - a)]
    assert bits_equal(got, full)


@pytest.mark.gpu
def test_bad_band_layout_rejected(ctx):
    s = rt_amd.Scene(scene(2), 64, 64, 0)
    ctx.upload(s)
    for br, n, i in ((8, 2, 0), (16, 0, 0), (16, 2, 2), (16, 2, -1)):
        f = s.frame.copy()
        f.band_rows, f.band_count, f.band_index = br, n, i
        with pytest.raises(rt_amd.RtError):
            ctx.render(f)


def test_camera_buffer_follows_the_camera():
    """The camera buffer (per-tile lists, built per camera by synchronous
    renders) must never serve a stale camera: after the camera moves, the
    async path renders without it until a synchronous render rebuilds it —
    every image bit-identical to a context that never had one."""
    torch = pytest.importorskip("torch")
    s = rt_amd.Scene(scene(2), 160, 120, 0)
    frames = []
    for dx in (0.0, 7.5, -12.25):
        f = s.frame.copy()
        f.cam_pos[0] += dx
        frames.append(f)
    ref = rt_amd.Context(0, camera_buffer=0, launch_camera=0)
    ref.upload(s)
    want = [ref.render_float(f) for f in frames]
    c = rt_amd.Context(0, launch_camera=0)  # the device camera buffer (launch records: no state to go stale)
    c.upload(s)
    out = torch.zeros((120, 160, 3), dtype=torch.float32, device="cuda")
    stream = torch.cuda.current_stream().cuda_stream
    for k, (f, w) in enumerate(zip(frames, want)):
        c.render_async(f, 0, out.data_ptr(), stream)  # stale (or no) buffer: not used
        torch.cuda.synchronize()
        assert bits_equal(out.cpu().numpy(), w), k
        assert bits_equal(c.render_float(f), w), k  # rebuilt for this camera
        c.render_async(f, 0, out.data_ptr(), stream)  # current: used
        torch.cuda.synchronize()
        assert bits_equal(out.cpu().numpy(), w), k


@pytest.mark.parametrize("w,h", [(1920, 1080), (333, 197), (8, 8), (1, 1), (640, 17)])
@pytest.mark.parametrize("i", [1, 2, 3, 4, 5, 6])
def test_launch_camera_equals_device_camera_state(i, w, h):
    """Tiny scenes' launch-camera records (RT_OPT_LAUNCH_CAMERA) against the
    device camera buffer and the per-wave path: the same float32 bits — at
    the reference camera, slabs off the 8-row grid, bands, a wide-angle film
    (the boxes' tile bound above one radian: no boxes) and a scaled, non
    rotation orientation (no boxes)."""
    s = rt_amd.Scene(scene(i), w, h, 0)
    a = rt_amd.Context(0)
    b = rt_amd.Context(0, launch_camera=0)
    p = rt_amd.Context(0, launch_camera=0, camera_buffer=0)
    for c in (a, b, p):
        c.upload(s)
    frames = [s.frame]
    if h >= 20:
        f = s.frame.copy()
        f.row_begin, f.row_end = 3, h - 5
        frames.append(f)
        f = s.frame.copy()
        f.band_rows, f.band_count, f.band_index = 16, 3, 1
        frames.append(f)
    f = s.frame.copy()
    f.half_w *= 40.0
    f.half_h *= 40.0
    frames.append(f)
    f = s.frame.copy()
    for q in range(12):
        f.orient[q] *= 1.25
    frames.append(f)
    for k, f in enumerate(frames):
        want = p.render_float(f)
        # three renders of each frame on the context's stream: the camera's
        # first frame computes its tile masks, the second stores them, the
        # third reads them back (off-grid slabs and bands included)
        for rep in range(3):
            assert bits_equal(a.render_float(f), want), (i, w, h, k, rep)
        assert bits_equal(b.render_float(f), want), (i, w, h, k)
    # host output in row chunks (each chunk a launch of its own), three times
    a.set_option("host_chunk_mb", max(1e-4, w * h * 12 / 8 / 1048576.0 / 1.01))
    try:
        f = s.frame.copy()
        f.cam_pos[1] += 0.25  # a camera new to the stream
        want = p.render_float(f)
        for rep in range(3):
            assert bits_equal(a.render_float(f), want), (i, w, h, "chunked", rep)
    finally:
        a.set_option("host_chunk_mb", 8)


def test_camera_buffer_after_bounce_frame(tmp_path):
    """A big scene rendered first with bounces (no camera buffer, so camera
    records only for <= 256 triangles), then at depth 0 from the same
    camera: the camera buffer must be built from complete records."""
    from rt_amd import synth

    path = synth.write_heightfield(str(tmp_path / "hfr.dat"), cols=40, rows=20, reflect=0.5)
    s = rt_amd.Scene(path, 320, 240, 3)
    c = rt_amd.Context(0)
    c.upload(s)
    c.render_float(s.frame)  # bounce kernel first
    f0 = s.frame.copy()
    f0.max_bounces = 0
    got = c.render_float(f0)
    ref = rt_amd.Context(0)
    ref.upload(s)
    assert bits_equal(got, ref.render_float(f0))


def test_async_device_outputs(ctx):
    torch = pytest.importorskip("torch")
    s = rt_amd.Scene(scene(6), 128, 96, 3)
    ctx.upload(s)
    rgba = torch.zeros((96, 128, 4), dtype=torch.uint8, device="cuda")
    rgb = torch.zeros((96, 128, 3), dtype=torch.float32, device="cuda")
    ctx.render_async(s.frame, rgba.data_ptr(), rgb.data_ptr(), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    assert np.array_equal(rgba.cpu().numpy(), ctx.render(s.frame))
    assert bits_equal(rgb.cpu().numpy(), ctx.render_float(s.frame))


def test_device_pointer_sync_render(ctx):
    torch = pytest.importorskip("torch")
    s = rt_amd.Scene(scene(3), 64, 64, 0)
    ctx.upload(s)
    out = torch.zeros((64, 64, 4), dtype=torch.uint8, device="cuda")
    assert rt_amd.lib().rt_render(ctx._h, rt_amd.ctypes.byref(s.frame), out.data_ptr()) == 0
    assert np.array_equal(out.cpu().numpy(), ctx.render(s.frame))


def test_deep_bounces_and_limits(ctx, oracle):
    # scene9: two facing mirrors (Kr 0.99) — depth 20 is the reference's default m_NbRebondsMax
    got = render(ctx, scene(9), 48, 32, 20)
    want = oracle.render(scene(9), 48, 32, 20)
    assert bits_equal(got, want)
    with pytest.raises(rt_amd.RtError) as e:
        render(ctx, scene(9), 8, 8, 40)
    assert e.value.code == -6


def test_bad_frame_rejected(ctx):
    s = rt_amd.Scene(scene(1), 16, 16, 0)
    ctx.upload(s)
    f = s.frame.copy()
    f.row_end = 17
    with pytest.raises(rt_amd.RtError):
        ctx.render(f)


def test_wave_primitives_selftest(ctx):
    """The DPP wave reductions and the wave cone the culling relies on, checked
    on the device against plain loops (rt_debug_selftest, 4,096 workgroups)."""
    import ctypes

    L = rt_amd.lib()
    f = L.rt_debug_selftest
    f.restype = ctypes.c_int
    f.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_uint)]
    fails = ctypes.c_uint(99)
    assert f(0, 4096, ctypes.byref(fails)) == 0
    assert fails.value == 0


@pytest.mark.parametrize("which", ["scene2", "heightfield"])
def test_camera_buffer_covers_only_the_ranks_rows(which, heightfield_path):
    """A slab (or band set) render builds the camera buffer for its own tile
    rows only — 1/n of the lists for 1/n of the frame — and still renders
    the full frame's bits for those rows."""
    import ctypes

    path = scene(2) if which == "scene2" else heightfield_path
    s = rt_amd.Scene(path, 1920, 1080, 0)
    c = rt_amd.Context(0, launch_camera=0)  # scene2's device camera buffer
    c.upload(s)
    L = rt_amd.lib()
    L.rt_debug_cb_info.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]

    def entries():
        info = (ctypes.c_double * 6)()
        assert L.rt_debug_cb_info(c._h, info, 6) == 0 and info[0] == 1.0
        return info[1]

    full = c.render_float(s.frame)
    n_full = entries()
    f = s.frame.copy()
    f.row_begin, f.row_end = 136, 272  # rank 1 of 8 (slab_rows)
    assert bits_equal(c.render_float(f), full[136:272])
    assert 0 < entries() < n_full / 4
    f = s.frame.copy()
    f.band_rows, f.band_count, f.band_index = 16, 8, 3
    part = c.render_float(f)
    assert 0 < entries() < n_full / 4
    for q in range(part.shape[0] // 16):
        a = (q * 8 + 3) * 16
        e = min(1080, a + 16)
        assert bits_equal(part[q * 16: q * 16 + (e - a)], full[a:e])
