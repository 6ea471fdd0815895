"""Bounce rays through the exact BVH (rt_bvh.h; VERDICT r04 item 2, SURVEY.md
§8(f) row 3): the reflective heightfield — the 50k-triangle mesh with
`reflect: 0.5` on every triangle (bench c3r / c5r) — against windows the
reference's own code rendered (tests/golden/hf_reflect.npz,
make_hf_reflect_golden.py), bit for bit in float32, through every entry
point; and the BVH walk against brute force for adversarial rays (grazing,
axis-aligned, far, degenerate) on the device."""
from __future__ import annotations

import ctypes
import os

import numpy as np
import pytest

import rt_amd
from conftest import GOLDEN, bits_equal

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def hfr_golden():
    with np.load(os.path.join(GOLDEN, "hf_reflect.npz")) as z:
        return {k: z[k] for k in z.files}


def _parse(k):
    size, d, rest = k.split("_", 3)[1], int(k.split("_")[2][1:]), k.rsplit("_win_", 1)[1]
    w, h = map(int, size.split("x"))
    return w, h, d, tuple(map(int, rest.split("_")))


def _groups(golden):
    g = {}
    for k, v in golden.items():
        w, h, d, win = _parse(k)
        g.setdefault((w, h, d), []).append((win, v, k))
    return g


@pytest.fixture(scope="module")
def hfr(heightfield_r05_path):
    ctx = rt_amd.Context(0)
    scenes = {}

    def get(w, h, d):
        if (w, h, d) not in scenes:
            scenes[(w, h, d)] = rt_amd.Scene(heightfield_r05_path, w, h, d)
        return scenes[(w, h, d)]

    ctx.upload(get(1920, 1080, 3))
    yield ctx, get
    ctx.close()


def _bvh_info(ctx):
    L = rt_amd.lib()
    L.rt_debug_bvh_info.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
    out = (ctypes.c_double * 5)()
    assert L.rt_debug_bvh_info(ctx._h, out, 5) == 0
    return list(out)


def test_bvh_built_for_the_reflective_mesh(hfr):
    ctx, _ = hfr
    built, inner, leaves, depth, ms = _bvh_info(ctx)
    assert built == 1.0 and leaves >= 50_000 / 4 and depth <= 24
    assert inner == leaves - 1  # a binary tree


@pytest.mark.parametrize("wavefront", [1, 0])
@pytest.mark.parametrize("size", [(1920, 1080, 3), (1920, 1080, 1), (1920, 1080, 6), (7680, 4320, 3)])
def test_reflective_heightfield_matches_reference(hfr, hfr_golden, size, wavefront):
    """The wavefront levels (RT_OPT_WAVEFRONT 1, the default) and the BVH
    megakernel (0), each against the reference's windows."""
    ctx, get = hfr
    w, h, d = size
    s = get(w, h, d)
    f = s.frame.copy()
    f.flags = rt_amd.FLAG_STATS
    ctx.set_option("wavefront", wavefront)
    try:
        full = ctx.render_float(f)
    finally:
        ctx.set_option("wavefront", 1)
    st = ctx.stats()
    if wavefront:  # level 0 = the big-list depth-0 kernel emitting children, then the levels
        # (under 4 Mpx its variant with the two-entry light-buffer walk, WAVE bit 2048)
        wave0 = 2574 if w * h < 4_000_000 else 526
        assert st.kernel.startswith(f"wavefront rt_trace_kernel<0,1,{wave0}>"), st.kernel
    else:
        # the BVH megakernel ran (reflect-only: its chain variant, WAVE bit 1024)
        assert st.kernel.endswith(",1,1294>"), st.kernel
    assert st.bounce_rays > 0
    # bounce rays test <= 1% of the 50,000 triangles each
    assert st.bounce_triangle_tests <= 0.01 * 50_000 * st.bounce_rays, (st.bounce_triangle_tests, st.bounce_rays)
    n = 0
    for win, want, k in _groups(hfr_golden)[(w, h, d)]:
        r0, r1, c0, c1 = win
        assert bits_equal(full[r0:r1, c0:c1], want), k
        n += 1
    assert n >= 6


def test_brute_force_bounce_kernel_agrees(hfr, hfr_golden):
    """RT_OPT_BVH 0 (every triangle per bounce ray) on two windows' rows."""
    ctx, get = hfr
    s = get(1920, 1080, 3)
    ctx.set_option("bvh", 0)
    try:
        for (win, want, k) in _groups(hfr_golden)[(1920, 1080, 3)][10:12]:
            r0, r1, c0, c1 = win
            f = s.frame.copy()
            f.row_begin, f.row_end = r0, r1
            f.flags = rt_amd.FLAG_STATS
            part = ctx.render_float(f)
            st = ctx.stats()
            assert ",270>" not in st.kernel
            assert bits_equal(part[:, c0:c1], want), k
    finally:
        ctx.set_option("bvh", 1)


def test_async_sequence_and_slabs_match(hfr, hfr_golden):
    import torch

    ctx, get = hfr
    s = get(1920, 1080, 3)
    want = {win: v for win, v, _ in _groups(hfr_golden)[(1920, 1080, 3)]}
    full = ctx.render_float(s.frame)
    ref8 = ctx.render(s.frame)
    stream = torch.cuda.current_stream().cuda_stream
    dev = torch.empty((1080, 1920, 4), dtype=torch.uint8, device="cuda")
    # a moved camera first (async builds no camera buffer for it), then back
    g = s.frame.copy()
    g.cam_pos[0] += 3.0
    ctx.render_async(g, dev.data_ptr(), 0, stream)
    ctx.render_async(s.frame, dev.data_ptr(), 0, stream)
    ctx.render_async(s.frame, dev.data_ptr(), 0, stream)
    torch.cuda.synchronize()
    assert np.array_equal(dev.cpu().numpy(), ref8)
    ring = torch.empty((2, 1080, 1920, 4), dtype=torch.uint8, device="cuda")
    ctx.render_sequence_async([s.frame, s.frame], ring.data_ptr(), 1080 * 1920 * 4, 0, 0, stream)
    torch.cuda.synchronize()
    assert np.array_equal(ring[1].cpu().numpy(), ref8)
    # slabs off the tile grid, and bands
    parts = []
    for r0, r1 in ((0, 301), (301, 777), (777, 1080)):
        f = s.frame.copy()
        f.row_begin, f.row_end = r0, r1
        parts.append(ctx.render_float(f))
    assert bits_equal(np.concatenate(parts, 0), full)
    for (r0, r1, c0, c1), v in want.items():
        assert bits_equal(full[r0:r1, c0:c1], v)


def test_wavefront_frames_on_two_streams(hfr):
    """Async wavefront frames of different cameras alternating between two
    streams (the queues are shared: each frame waits for the other stream's
    last one) equal synchronous renders."""
    import torch

    ctx, get = hfr
    s = get(1920, 1080, 3)
    cams = []
    for k in range(4):
        g = s.frame.copy()
        g.cam_pos[0] += 2.0 * k
        g.cam_pos[2] -= 1.5 * k
        cams.append(g)
    want = [ctx.render(g) for g in cams]
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    outs = [torch.empty((1080, 1920, 4), dtype=torch.uint8, device="cuda") for _ in cams]
    for k, g in enumerate(cams):
        st = s1 if k % 2 == 0 else s2
        ctx.render_async(g, outs[k].data_ptr(), 0, st.cuda_stream)
    torch.cuda.synchronize()
    for k in range(len(cams)):
        assert np.array_equal(outs[k].cpu().numpy(), want[k]), k


def test_wavefront_stats_count_the_bounce_rays(hfr):
    ctx, get = hfr
    s = get(1920, 1080, 3)
    f = s.frame.copy()
    f.flags = rt_amd.FLAG_STATS
    out = {}
    for wf in (1, 0):
        ctx.set_option("wavefront", wf)
        ctx.render(f)
        st = ctx.stats()
        out[wf] = (st.primary_rays, st.bounce_rays, st.shadow_rays, st.bounce_triangle_tests, st.bvh_nodes_visited)
    ctx.set_option("wavefront", 1)
    assert out[1][:3] == out[0][:3]  # the same rays, however scheduled
    # the same walks but for the stragglers the wave finishes together
    assert out[0][3] <= out[1][3] <= 1.5 * out[0][3], out


def _rays_on_mesh(rng, s, n):
    """Origins on random triangles of the mesh (p0 + u e1 + v e2 in float32,
    the way a hit point is made), plus the triangles' float records."""
    types, geom = s.arrays()[0], s.arrays()[1]
    tri = np.nonzero(types == rt_amd.TRIANGLE)[0]
    k = rng.choice(tri, n)
    g = geom[k].astype(np.float32)
    p0, p1, p2 = g[:, 0:3], g[:, 3:6], g[:, 6:9]
    e1, e2 = (p1 - p0).astype(np.float32), (p2 - p0).astype(np.float32)
    u = rng.random(n).astype(np.float32)
    v = (rng.random(n) * (1 - u)).astype(np.float32)
    O = (p0 + u[:, None] * e1 + v[:, None] * e2).astype(np.float32)
    nrm = np.cross(e1.astype(np.float64), e2.astype(np.float64))
    nrm /= np.linalg.norm(nrm, axis=1, keepdims=True)
    return O, e1, e2, nrm


def _unit(v):
    v = np.asarray(v, np.float32)
    ln = np.sqrt((v[:, 0] * v[:, 0] + v[:, 1] * v[:, 1] + v[:, 2] * v[:, 2]).astype(np.float32))
    return (v * (np.float32(1.0) / ln)[:, None]).astype(np.float32)


def _adversarial(s, seed=5):
    rng = np.random.default_rng(seed)
    n = 32768
    sets = {}
    O, e1, e2, nrm = _rays_on_mesh(rng, s, n)
    sets["mesh_random"] = (O, _unit(rng.normal(size=(n, 3))))
    # grazing: in the triangle's plane, lifted by 1e-7 .. 1e-2 rad
    w = rng.normal(size=(n, 3))
    w -= np.einsum("ij,ij->i", w, nrm)[:, None] * nrm
    w /= np.linalg.norm(w, axis=1, keepdims=True)
    el = np.exp(rng.uniform(np.log(1e-7), np.log(1e-2), n)) * np.where(rng.random(n) < 0.5, 1, -1)
    sets["mesh_grazing"] = (O, _unit(np.cos(el)[:, None] * w + np.sin(el)[:, None] * nrm))
    # axis-aligned and one-zero-component directions (inv = +-inf in the slab test)
    axes = np.array([[1, 0, 0], [-1, 0, 0], [0, 1, 0], [0, -1, 0], [0, 0, 1], [0, 0, -1],
                     [0.6, 0.8, 0], [0, -0.6, 0.8], [-0.8, 0, -0.6]], np.float32)
    sets["mesh_axes"] = (O, axes[rng.integers(0, len(axes), n)])
    # straight down through a mesh vertex (ties between the triangles that
    # share it: the file-index compare) and origins on vertex coordinate
    # planes (box faces) moving inside them
    types, geom = s.arrays()[0], s.arrays()[1]
    vt = geom[rng.choice(np.nonzero(types == rt_amd.TRIANGLE)[0], n)][:, 0:3].astype(np.float32)
    sets["vertex_drop"] = (vt + np.array([0, 3, 0], np.float32), np.tile(np.array([[0, -1, 0]], np.float32), (n, 1)))
    sets["on_faces"] = (vt + np.array([0, 0.5, 0], np.float32), axes[rng.integers(0, 6, n)])
    # from far away, aimed at random mesh points
    far = (rng.normal(size=(n, 3)) * np.exp(rng.uniform(np.log(50), np.log(5e3), n))[:, None]).astype(np.float32)
    sets["far"] = (far, _unit(O - far))
    # reflected directions off the hit triangles (what the kernel traces)
    d_in = _unit(rng.normal(size=(n, 3)) - np.array([0, 2, 0]))
    nf = nrm.astype(np.float32)
    dn = (d_in[:, 0] * nf[:, 0] + d_in[:, 1] * nf[:, 1] + d_in[:, 2] * nf[:, 2]).astype(np.float32)
    sets["reflected"] = (O, (d_in - (np.float32(2.0) * dn)[:, None] * nf).astype(np.float32))
    # degenerate: zero, long, NaN, infinite (every triangle is tested for these)
    m = 256
    bad_d = np.zeros((m, 3), np.float32)
    bad_d[m // 4: m // 2] = 3.0
    bad_d[m // 2: 3 * m // 4] = np.nan
    bad_o = O[:m].copy()
    bad_o[3 * m // 4:, 1] = np.inf
    bad_d[3 * m // 4:] = _unit(rng.normal(size=(m // 4, 3)))
    sets["degenerate"] = (bad_o, bad_d)
    return sets


def _check_rays(ctx, O, D):
    L = rt_amd.lib()
    L.rt_debug_bvh_rays.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p,
                                    ctypes.c_void_p, ctypes.c_void_p]
    rays = np.ascontiguousarray(np.concatenate([O, D], 1).astype(np.float32))
    n = rays.shape[0]
    idx = np.zeros((n, 2), np.int32)
    t = np.zeros((n, 2), np.float32)
    tally = np.zeros(2, np.uint64)
    rc = L.rt_debug_bvh_rays(ctx._h, rays.ctypes.data, n, idx.ctypes.data, t.ctypes.data, tally.ctypes.data)
    assert rc == 0, ctx._err()
    return idx, t, tally


def _check_rays_wave(ctx, O, D):
    L = rt_amd.lib()
    L.rt_debug_bvh_rays_wave.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p,
                                         ctypes.c_void_p]
    rays = np.ascontiguousarray(np.concatenate([O, D], 1).astype(np.float32))
    n = rays.shape[0]
    idx = np.zeros(n, np.int32)
    t = np.zeros(n, np.float32)
    assert L.rt_debug_bvh_rays_wave(ctx._h, rays.ctypes.data, n, idx.ctypes.data, t.ctypes.data) == 0, ctx._err()
    return idx, t


def test_bvh_walk_equals_brute_force_on_adversarial_rays(hfr):
    ctx, get = hfr
    s = get(1920, 1080, 3)
    for name, (O, D) in _adversarial(s).items():
        idx, t, tally = _check_rays(ctx, O, D)
        same = (idx[:, 0] == idx[:, 1]) & (t[:, 0].view(np.uint32) == t[:, 1].view(np.uint32))
        bad = np.nonzero(~same)[0]
        assert bad.size == 0, (name, bad[:5], idx[bad[:5]], t[bad[:5]])
        # the wave-cooperative walk (the wavefront's stragglers) on the first 4,096
        wi, wt = _check_rays_wave(ctx, O[:4096], D[:4096])
        same = (wi == idx[:4096, 1]) & (wt.view(np.uint32) == t[:4096, 1].view(np.uint32))
        assert same.all(), (name, np.nonzero(~same)[0][:5])
        if name not in ("degenerate",):
            hits = int((idx[:, 1] >= 0).sum())
            assert hits > 0, name
        if name not in ("degenerate", "far"):
            # the walk tests a small fraction of the 50,000 triangles (rays
            # from far away: the margins grow with the distance, see rt_bvh.h)
            assert tally[0] <= 0.02 * 50_000 * len(O), (name, tally)


@pytest.mark.parametrize("seed", [11, 12])
def test_bvh_walk_equals_brute_force_on_random_meshes(tmp_path, seed):
    """Random triangle soups (slivers, long edges, 400-unit triangles, a
    reflective material) with planes and quadrics: the BVH walk and brute
    force agree on every ray."""
    rng = np.random.default_rng(seed)
    lines = ["background: 10 10 30", "origin: 0 0 80", "eye: 0 0 0", "up: 0 1 0",
             "Lumiere: l", "        position: 10 50 40", "        intens: 0.8"]
    n = 700
    for i in range(n):
        c = rng.uniform(-40, 40, 3)
        sc = [0.05, 2.0, 30.0, 400.0][i % 4] if i % 7 else 0.5
        pts = c + rng.normal(size=(3, 3)) * sc
        if i % 5 == 0:  # sliver
            pts[2] = pts[0] + (pts[1] - pts[0]) * 0.5 + rng.normal(size=3) * 1e-3
        lines.append(f"Poly: t{i}")
        for j in range(3):
            lines.append(f"        point: {j} {pts[j][0]:.4f} {pts[j][1]:.4f} {pts[j][2]:.4f}")
        lines.append("        color: 200 100 50")
        lines.append("        reflect: 0.6")
    lines += ["Plane: p", "        v_linear: 0 1 0", "        v_const: 45", "        color: 10 200 10"]
    lines += ["Quad: q", "        v_quad: 1 1 1", "        v_const: -25", "        color: 10 10 200",
              "        reflect: 0.3"]
    path = tmp_path / f"soup{seed}.dat"
    path.write_text("\n".join(lines) + "\n")
    s = rt_amd.Scene(str(path), 64, 64, 3)
    ctx = rt_amd.Context(0)
    ctx.upload(s)
    assert _bvh_info(ctx)[0] == 1.0
    m = 65536
    O = rng.uniform(-60, 60, (m, 3)).astype(np.float32)
    D = _unit(rng.normal(size=(m, 3)))
    D[: m // 8] = np.array([1, 0, 0], np.float32)  # axis-aligned
    idx, t, tally = _check_rays(ctx, O, D)
    same = (idx[:, 0] == idx[:, 1]) & (t[:, 0].view(np.uint32) == t[:, 1].view(np.uint32))
    assert same.all(), np.nonzero(~same)[0][:5]
    assert (idx[:, 1] >= 0).sum() > m // 4
    ctx.close()


# ---- the wavefront levels' 2-child segments: refraction, and a
# negative min_energy (every node spawns both children, Kt = 0 included)
def _oracle_windows(oracle, path, w, h, depth, min_energy, wins, threads=8):
    out = []
    for (r0, r1, c0, c1) in wins:
        rc, p = oracle.load(path, w, h, depth)
        assert rc == 0
        oracle.L.oracle_set_params(p, depth, min_energy, 1.0)
        img = np.zeros((r1 - r0, c1 - c0, 3), np.float32)
        oracle.L.oracle_render_window(p, r0, r1, c0, c1, img.ctypes.data, threads)
        oracle.L.oracle_free(p)
        out.append(img)
    return out


_WINS = [(0, 8, 0, 64), (300, 308, 900, 964), (500, 508, 1200, 1264), (700, 716, 400, 432), (1072, 1080, 1856, 1920),
         (540, 548, 0, 1920)]


def _three_ways(path, w, h, depth, min_energy, oracle):
    s = rt_amd.Scene(path, w, h, depth, min_energy=min_energy)
    got = {}
    for wf in (1, 0):
        c = rt_amd.Context(0, wavefront=wf)
        c.upload(s)
        f = s.frame.copy()
        f.flags = rt_amd.FLAG_STATS
        got[wf] = c.render_float(f)
        st = c.stats()
        assert st.kernel.startswith("wavefront") == bool(wf), st.kernel
        assert st.bounce_rays > 0
        c.close()
    assert bits_equal(got[1], got[0])
    for (r0, r1, c0, c1), want in zip(_WINS, _oracle_windows(oracle, path, w, h, depth, min_energy, _WINS)):
        assert bits_equal(got[1][r0:r1, c0:c1], want), (r0, r1, c0, c1)


@pytest.mark.parametrize("depth", [3, 5])
def test_refractive_mesh_wavefront_megakernel_oracle(tmp_path, oracle, depth):
    """Every triangle reflects, every other one also refracts (Kt 0.4, ior
    1.5; the opaque half keeps the light buffer, which the BVH kernels need):
    2-child nodes, inside/out IOR flips, the refracted branch's sort key — at
    1920 x 1080."""
    from rt_amd import synth

    lines, k = [], 0
    for line in synth.heightfield_dat(cols=40, rows=20, reflect=0.3).split("\n"):
        lines.append(line)
        if line.startswith("        reflect:"):
            if k % 2 == 0:
                lines.append("        refract: 0.4 1.5")
            k += 1
    path = tmp_path / "hf_refr.dat"
    path.write_text("\n".join(lines))
    _three_ways(str(path), 1920, 1080, depth, 0.01, oracle)


def test_negative_min_energy_spawns_both_children(tmp_path, oracle):
    """A reflect-only mesh with min_energy < 0: K * energy > min_energy holds
    for Kt = 0 too, so every hit spawns two children (the queues must be
    sized for 2 per node, not 1)."""
    from rt_amd import synth

    path = synth.write_heightfield(str(tmp_path / "hf_neg.dat"), cols=12, rows=6, reflect=0.5)
    _three_ways(path, 1920, 1080, 3, -1.0, oracle)


@pytest.mark.parametrize("sort", [0, 2, 3, 6, 7])
def test_wavefront_sort_orders_render_the_same(hfr, hfr_golden, sort):
    """RT_OPT_WF_SORT (the counting sorts of each level's live rays by parent
    bin and by hit bin or, bit 2, the hit's light-buffer cell) only changes
    which wave takes which ray: the
    reflective heightfield at 1920 x 1080 d3 and d6 against the reference's
    windows, bit for bit, and the refracting mesh against the default."""
    ctx, get = hfr
    ctx.set_option("wf_sort", sort)
    try:
        for d in (3, 6):
            full = ctx.render_float(get(1920, 1080, d).frame)
            for win, want, k in _groups(hfr_golden)[(1920, 1080, d)]:
                r0, r1, c0, c1 = win
                assert bits_equal(full[r0:r1, c0:c1], want), k
    finally:
        ctx.set_option("wf_sort", 1)


def test_straggler_overlap_renders_the_same(hfr, hfr_golden):
    """RT_OPT_WF_OVERLAP (the stragglers' walks and shading on a second
    stream beside each level's shade launch) on and off: the same images, and
    the reference's windows at d3 and d6 with it off."""
    ctx, get = hfr
    for d in (3, 6):
        f = get(1920, 1080, d).frame
        on = ctx.render_float(f)
        ctx.set_option("wf_overlap", 0)
        try:
            off = ctx.render_float(f)
        finally:
            ctx.set_option("wf_overlap", 1)
        assert bits_equal(on, off), d
        for win, want, k in _groups(hfr_golden)[(1920, 1080, d)]:
            r0, r1, c0, c1 = win
            assert bits_equal(off[r0:r1, c0:c1], want), k


def test_refractive_mesh_sort_orders(tmp_path):
    from rt_amd import synth

    lines, k = [], 0
    for line in synth.heightfield_dat(cols=40, rows=20, reflect=0.3).split("\n"):
        lines.append(line)
        if line.startswith("        reflect:"):
            if k % 2 == 0:
                lines.append("        refract: 0.4 1.5")
            k += 1
    path = tmp_path / "hf_refr.dat"
    path.write_text("\n".join(lines))
    s = rt_amd.Scene(str(path), 1920, 1080, 4)
    imgs = []
    for sort, ovl in ((0, 1), (1, 1), (2, 1), (3, 1), (7, 1), (1, 0), (3, 0)):
        c = rt_amd.Context(0, wf_sort=sort, wf_overlap=ovl)
        c.upload(s)
        imgs.append(c.render_float(s.frame))
        assert c.stats().kernel.startswith("wavefront")
        c.close()
    for im in imgs[1:]:
        assert bits_equal(im, imgs[0])
