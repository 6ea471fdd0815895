// rt_cull.h — wave-level (packet) culling: wave cones, cone / edge / cluster records
// and their prepass kernels.
// Part of the device code of rt_kernels.hip (one translation unit: the
// kernels are templates instantiated by its host half); built with the
// same exactness flags (no FMA contraction, IEEE div/sqrt).
#ifndef RT_AMD_RT_CULL_H
#define RT_AMD_RT_CULL_H

#include "rt_primitives.h"

#pragma clang fp contract(off)

namespace rt {

// ------------------------------------------------ wave-level (packet) culling
// When all 64 lanes of a wave are active (checked at run time, so the result
// never depends on how the compiler shaped the control flow), the wave's
// rays from a common apex (the camera, or one light for shadow rays) fit in
// one cone [w, W] (w: the centre lane's direction, cos W = min over lanes).
// A triangle whose cone [v, T] from the same apex satisfies
// angle(w, v) > W + T cannot be reached by any lane (spherical triangle
// inequality), so 64 triangles are culled per wave instruction — one lane
// per triangle — and only the ballot's survivors are tested exactly.  The
// per-lane predicates above remain the definition; the margins here only
// widen them (cos W lowered, sin W raised, cos(W + T) lowered by 2e-6 and by
// the shadow ray's direction slack).
__device__ __forceinline__ bool wave_full() { return __builtin_amdgcn_read_exec() == ~0ull; }

template <int CTRL>
__device__ __forceinline__ float dppf(float v)
{
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, false));
}
__device__ __forceinline__ float readlanef(float v, int lane)
{
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), lane));
}
// Min / max over all 64 lanes (full exec only): quad, half-row and row
// exchanges by DPP, then the four row results.
__device__ __forceinline__ float wave_min(float v)
{
    v = fminf(v, dppf<0xB1>(v));   // quad_perm [1,0,3,2]
    v = fminf(v, dppf<0x4E>(v));   // quad_perm [2,3,0,1]
    v = fminf(v, dppf<0x141>(v));  // row_half_mirror
    v = fminf(v, dppf<0x140>(v));  // row_mirror
    return fminf(fminf(readlanef(v, 0), readlanef(v, 16)), fminf(readlanef(v, 32), readlanef(v, 48)));
}
__device__ __forceinline__ float wave_max(float v)
{
    v = fmaxf(v, dppf<0xB1>(v));
    v = fmaxf(v, dppf<0x4E>(v));
    v = fmaxf(v, dppf<0x141>(v));
    v = fmaxf(v, dppf<0x140>(v));
    return fmaxf(fmaxf(readlanef(v, 0), readlanef(v, 16)), fmaxf(readlanef(v, 32), readlanef(v, 48)));
}
// Sum over all 64 lanes (full exec only), for the stats tallies.
__device__ __forceinline__ unsigned long long wave_sum_u64(unsigned long long v)
{
    // the stats launch is untimed: 64 scalar reads are simple and exact
    unsigned long long t = 0;
    for (int l = 0; l < 64; ++l) {
        const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)v, l);
        const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(v >> 32), l);
        t += ((unsigned long long)hi << 32) | lo;
    }
    return t;
}

struct WaveCone {
    Vec3 w;
    float cosW, sinW, chord;  // chord = |d - w| bound = 2 sin(W/2)
    bool ok;
};
// Cone of the live lanes' unit directions d (apex shared).  ok = false when
// no lane is live or the spread exceeds 60 degrees (then W + T could pass pi).
__device__ __forceinline__ WaveCone wave_cone(const Vec3 d, bool live)
{
    WaveCone c;
    const unsigned long long lm = __ballot(live);
    c.ok = lm != 0;
    if (!c.ok) return c;
    const int ref = ((lm >> 36) & 1ull) ? 36 : (int)__builtin_ctzll(lm);
    c.w = make3(readlanef(d.x, ref), readlanef(d.y, ref), readlanef(d.z, ref));
    float cd = dot(d, c.w);
    cd = live ? (cd == cd ? cd : -1.0f) : 1.0f;
    c.cosW = wave_min(cd) - 1e-6f;
    c.ok = c.cosW >= 0.5f;
    c.sinW = __builtin_amdgcn_sqrtf(fmaxf(0.0f, 1.0f - c.cosW * c.cosW)) + 1e-6f;
    c.chord = __builtin_amdgcn_sqrtf(2.0f * (1.0f - c.cosW)) + 1e-6f;
    return c;
}
// May some ray of the wave cone reach the triangle cone [c0.xyz, c0.w; c1.w]?
// ang = extra angular slack.
// ang = extra angular slack, applied as a wider wave cone W + ang:
// cos(W + a) >= cosW - a sinW - a^2/2 and sin(W + a) <= sinW + a cosW, both
// within a^2 of the true values, so the test is cos(W + a + T) minus the
// rounding margin to within ~1e-10 — the angle-space form the cluster
// records rely on (rt_cluster_prepass).
__device__ __forceinline__ bool cone_overlap(const WaveCone& wc, const float4 c0, float sinT, float ang,
                                             float margin = 2e-6f)
{
    const float cw = wc.cosW - ang * wc.sinW - 0.5f * ang * ang;
    const float sw = wc.sinW + ang * wc.cosW;
    const float lim = cw * c0.w - sw * sinT - margin;
    return !(c0.w > 0.0f) | (dot(wc.w, make3(c0.x, c0.y, c0.z)) >= lim);
}

// May some ray of the wave cone pass on the inner side (up to the margin
// in e.w) of one edge plane [e.xyz, e.w]?  For every d in the cone
// d . n <= w . n + |d - w| <= w . n + chord(W) (+ ang for the widened cone).
__device__ __forceinline__ bool edge_open(const WaveCone& wc, const float4 e, float ang)
{
    const float c = dot(wc.w, make3(e.x, e.y, e.z));
    return !(c + wc.chord + 2e-6f + ang < e.w);
}
__device__ __forceinline__ bool edges_open(const WaveCone& wc, const float4* e, float ang)
{
    return edge_open(wc, e[0], ang) & edge_open(wc, e[1], ang) & edge_open(wc, e[2], ang);
}

// Per-wave LDS windows (dynamic LDS, one per wave): the light-buffer walk's
// staged entries (rt_shade.h lb_walk_lds: kLbLdsCap entries of a, b,
// c per wave) and the camera-list walk's staged records (a, b:
// kLbLdsCap / 2 records of 64 B per wave).  The two walks never overlap in a
// wave.
#ifndef RT_LB_LDS_CAP
#define RT_LB_LDS_CAP 64
#endif
constexpr int kLbLdsCap = RT_LB_LDS_CAP;  // entries per wave window
// The wave's window in the launch's dynamic LDS (kLdsWaveBytes per wave of
// the workgroup, trace_dims on the host): a[cap], b[cap] float4, c[cap] float2.
constexpr size_t kLdsWaveBytes = (size_t)kLbLdsCap * 40;
struct LdsWin {
    float4* a;
    float4* b;
    float2* c;
};
__device__ __forceinline__ LdsWin lds_window()
{
    extern __shared__ float4 rt_lds_dyn[];
    float4* a = rt_lds_dyn + (threadIdx.x >> 6) * (kLbLdsCap * 5 / 2);
    return LdsWin{a, a + kLbLdsCap, reinterpret_cast<float2*>(a + 2 * kLbLdsCap)};
}

__device__ __forceinline__ void wave_lds_sync()
{
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// One batch of 64 triangles [k0, k0 + 64) for the wave's camera rays: one
// lane per triangle against the wave cone, exact tests on the survivors.
// STAGE (big lists: the clustered per-wave path, whose kernels have LDS
// windows): each survivor's lane loads its tri[] record into the wave's
// window first — one load round trip for the batch instead of one per
// survivor — and the wave tests them from LDS in the same (ascending) order.
template <bool STAGE = false>
__device__ __forceinline__ void camera_wave_batch(const SceneDev& S, const WaveCone& wc, int k0, const Vec3 O,
                                                  const Vec3 D, float& bt, int& bi, Counters& cnt,
                                                  float far = INFINITY)
{
    const int k = k0 + (int)(threadIdx.x & 63);
    float4 c0 = make_float4(0.f, 0.f, 0.f, 1.f), c1 = make_float4(0.f, 0.f, 0.f, 0.f);  // no reach
    if (k < S.n_tri) {
        c0 = S.cone_cam[2 * k];
        c1 = S.cone_cam[2 * k + 1];
    }
    // far: every lane already holds a hit nearer than this, so a triangle
    // whose hits all lie at t >= dmin > far cannot win
    bool reach = cone_overlap(wc, c0, c1.w, 0.0f) & !(far < c1.x);
    // edge records only for sphere survivors
    if (S.use_edges && reach) reach = edges_open(wc, S.cone_cam + 2 * S.n_tri + 3 * k, 0.0f);
    RT_EV(cnt, 1);
    unsigned long long m = __ballot(reach);
    if constexpr (STAGE) {
        if (!m) return;
        const LdsWin win = lds_window();
        const int rk = (int)__builtin_amdgcn_mbcnt_hi((unsigned)(m >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)m, 0u));
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        if (reach) {
            const float4* r = S.tri + 3 * k;
            const float4 a = r[0], b = r[1], c = r[2];
            win.a[rk] = a;
            win.b[rk] = b;
            win.c[rk] = make_float2(c.x, c.y);
        }
        wave_lds_sync();
        const int n = __popcll(m);
        for (int j = 0; j < n; ++j) {
            RT_EV(cnt, 2);
            const float4 a = win.a[j], b = win.b[j];
            const float2 c = win.c[j];
            ++cnt.tri;
            const Vec3 e1 = make3(a.w, b.x, b.y), e2 = make3(b.z, b.w, c.x);
            const TriU r = tri_u(make3(a.x, a.y, a.z), e1, e2, O, D);
            if (!__any(r.ok)) continue;
            float t;
            const bool ok = tri_vt(r, e1, e2, D, t);
            take_min(ok, t, __float_as_int(c.y), bt, bi);
        }
        return;
    }
    while (m) {
        const int kk = k0 + (int)__builtin_ctzll(m);
        m &= m - 1;
        RT_EV(cnt, 2);
        if (S.use_tricam) {
            const float4* r = S.tricam + 4 * kk;
            camera_tri(r[0], r[1], r[2], r[3], D, bt, bi, cnt);
        } else {
            const TriRec tr = load_tri(S, kk);
            ++cnt.tri;
            const TriU r = tri_u(tr.p0, tr.e1, tr.e2, O, D);
            if (!__any(r.ok)) continue;
            float t;
            const bool ok = tri_vt(r, tr.e1, tr.e2, D, t);
            take_min(ok, t, tr.idx, bt, bi);
        }
    }
}

// Closest hit for camera rays, wave-culled (full wave, cone ok).
template <bool CLU>
__device__ __forceinline__ int closest_hit_camera_wave(const SceneDev& S, const WaveCone& wc, const Vec3 O,
                                                       const Vec3 D, float& best_t, Counters& cnt)
{
    float bt = -1.0f;
    int bi = -1;
    const int lane = (int)(threadIdx.x & 63);
    // planes first: their hits bound the early exit below (the minimum over
    // (t, index) does not depend on the order)
    for (int k = 0; k < S.n_plane; ++k) {
        const float4 a = S.plane[2 * k], b = S.plane[2 * k + 1];
        float t;
        ++cnt.pla;
        const bool ok = hit_plane(make_float4(0.f, a.x, a.y, a.z), make_float4(a.w, 0.f, 0.f, 0.f), O, D, t);
        take_min(ok, t, __float_as_int(b.x), bt, bi);
    }
    if constexpr (CLU) {
        // Clusters of 64 first (a cluster record implies every member's
        // test), nearest first (rt_cluster_sort: by dmin, the id in q1.y):
        // once every lane holds a hit nearer than the next cluster's dmin,
        // nothing farther can win.
        for (int c0i = 0; c0i < S.n_clu; c0i += 64) {
            const float far = wave_max(bi >= 0 ? bt : INFINITY);
            if (far < S.clu_cam[2 * c0i + 1].x) break;
            const int cl = c0i + lane;
            float4 q0 = make_float4(0.f, 0.f, 0.f, 1.f), q1 = make_float4(INFINITY, 0.f, 0.f, 0.f);  // no reach
            if (cl < S.n_clu) {
                q0 = S.clu_cam[2 * cl];
                q1 = S.clu_cam[2 * cl + 1];
            }
            const int id = __float_as_int(q1.y);
            RT_EV(cnt, 0);
            unsigned long long cm = __ballot(cone_overlap(wc, q0, q1.w, 0.0f, 4e-6f) & !(far < q1.x));
            while (cm) {
                const int b = (int)__builtin_ctzll(cm);
                cm &= cm - 1;
                const int cid = __builtin_amdgcn_readlane(id, b);
                camera_wave_batch<true>(S, wc, 64 * cid, O, D, bt, bi, cnt,
                                                    wave_max(bi >= 0 ? bt : INFINITY));
            }
        }
    } else {
        // the union record of all triangles first (small lists): one wave test
        bool any_tri = true;
        if (S.uni) {
            const float far = wave_max(bi >= 0 ? bt : INFINITY);
            any_tri = cone_overlap(wc, S.uni[0], S.uni[1].w, 0.0f, 4e-6f) & !(far < S.uni[1].x);
        }
        if (any_tri)
            for (int k0 = 0; k0 < S.n_tri; k0 += 64) camera_wave_batch(S, wc, k0, O, D, bt, bi, cnt);
    }
    for (int k = 0; k < S.n_quad; ++k) {
        const float4* r = S.quad + 3 * k;
        const float4 a = r[0], b = r[1], c = r[2];
        float t;
        ++cnt.qua;
        const bool ok = hit_quadric(make_float4(0.f, a.x, a.y, a.z), make_float4(a.w, b.x, b.y, b.z),
                                    make_float4(b.w, c.x, c.y, 0.f), O, D, t);
        take_min(ok, t, __float_as_int(c.z), bt, bi);
    }
    best_t = bt;
    return bi;
}

// Scene.cpp:1543-1552: the primary ray direction of pixel (pxc, pyc):
// (float)(2*PixX) * InvW - 1, then * HalfW; times the orientation; then
// Vecteur3.h Normaliser with the exact fast sqrt / reciprocal sequences
// (rt_fastmath.h; the IEEE results whichever path the wave takes, so the bits
// do not depend on the wave's other lanes).
__device__ __forceinline__ Vec3 camera_dir(const FrameDev& F, int pxc, int pyc)
{
    const Vec3 d0 = make3((2 * pxc * F.inv_w - 1) * F.half_w, (2 * pyc * F.inv_h - 1) * F.half_h, -1.0f);
    Mat4 M;
#pragma unroll
    for (int i = 0; i < 16; ++i) M.m[i >> 2][i & 3] = F.orient[i];
    const Vec3 dm = d0 * M;
    const float len = sqrt_w(dm.x * dm.x + dm.y * dm.y + dm.z * dm.z);
    return len > kEps ? dm * recip_w(len) : make3(0.f, 0.f, 0.f);
}

// Camera-list walk from LDS (the big-list kernel; the small-list kernel
// measured slower with it): the wave stages the next W records of
// its list with one load per lane (for lists of indices, the index then its
// record: two latencies per window instead of per entry) and walks them from
// LDS — same entries, same order, same exit.
constexpr unsigned kCbLdsW = 32;
static_assert(2 * kCbLdsW <= kLbLdsCap, "camera window exceeds the wave's LDS");

// Closest hit for camera rays from the tile's camera-buffer list (the wave
// is the tile: full, rows aligned).  Planes and quadrics first (their hits
// tighten the exit); then the list in cluster order, leaving once every
// lane holds a hit nearer than the entry's key (no later entry can report a
// nearer or equal hit: t >= dmin > best, as in the cluster early exit).
// INLINE (big lists): walk the inline records when the buffer has them.
template <bool INLINE>
__device__ __forceinline__ int closest_hit_camera_list(const SceneDev& S, int tile, const Vec3 O, const Vec3 D,
                                                       float& best_t, Counters& cnt)
{
    float bt = -1.0f;
    int bi = -1;
    for (int k = 0; k < S.n_plane; ++k) {
        const float4 a = S.plane[2 * k], b = S.plane[2 * k + 1];
        float t;
        ++cnt.pla;
        const bool ok = hit_plane(make_float4(0.f, a.x, a.y, a.z), make_float4(a.w, 0.f, 0.f, 0.f), O, D, t);
        take_min(ok, t, __float_as_int(b.x), bt, bi);
    }
    for (int k = 0; k < S.n_quad; ++k) {
        const float4* r = S.quad + 3 * k;
        const float4 a = r[0], b = r[1], c = r[2];
        float t;
        ++cnt.qua;
        const bool ok = hit_quadric(make_float4(0.f, a.x, a.y, a.z), make_float4(a.w, b.x, b.y, b.z),
                                    make_float4(b.w, c.x, c.y, 0.f), O, D, t);
        take_min(ok, t, __float_as_int(c.z), bt, bi);
    }
    const unsigned e0 = S.cb_off[tile], e1 = S.cb_off[tile + 1];
    if constexpr (INLINE) {
        constexpr unsigned W = kCbLdsW;
        const int lane = (int)(threadIdx.x & 63);
        const LdsWin win = lds_window();
        const bool inl = INLINE && S.cb_rec;
        for (unsigned w0 = e0; w0 < e1; w0 += W) {
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            const bool live = (unsigned)lane < W && w0 + lane < e1;
            const unsigned n = e1 - w0 < W ? e1 - w0 : W;
            float4 a, b, c, d;
            if (live) {
                if (inl) {
                    const float4* r = S.cb_rec + 4 * (size_t)(w0 + lane);
                    a = r[0];
                    b = r[1];
                    c = r[2];
                    d = r[3];
                } else {
                    const int2 en = S.cb_ent[w0 + lane];
                    const float4* r = S.tricam + 4 * (size_t)en.x;
                    a = r[0];
                    b = r[1];
                    c = r[2];
                    d = r[3];
                    d.z = __int_as_float(en.y);
                }
            }
            if (live) {
                win.a[2 * lane] = a;
                win.a[2 * lane + 1] = b;
                win.b[2 * lane] = c;
                win.b[2 * lane + 1] = d;
            }
            wave_lds_sync();
            bool stop = false;
            for (unsigned j = 0; j < n; ++j) {
                const float4 d = win.b[2 * j + 1];
                if (!__any((bi < 0) | !(bt < d.z))) {
                    stop = true;
                    break;
                }
                RT_EV(cnt, 2);
                camera_tri(win.a[2 * j], win.a[2 * j + 1], win.b[2 * j], d, D, bt, bi, cnt);
            }
            if (stop) break;
        }
        best_t = bt;
        return bi;
    }
    if (INLINE && S.cb_rec) {  // records inline: one scalar load round trip per entry
        for (unsigned e = e0; e < e1; ++e) {
            const float4* r = S.cb_rec + 4 * (size_t)e;
            const float4 a = r[0], b = r[1], c = r[2], d = r[3];  // key in d.z
            if (!__any((bi < 0) | !(bt < d.z))) break;
            RT_EV(cnt, 2);
            camera_tri(a, b, c, d, D, bt, bi, cnt);
        }
    } else {
        for (unsigned e = e0; e < e1; ++e) {
            const int2 en = S.cb_ent[e];
            if (!__any((bi < 0) | !(bt < __int_as_float(en.y)))) break;
            RT_EV(cnt, 2);
            const float4* r = S.tricam + 4 * en.x;
            camera_tri(r[0], r[1], r[2], r[3], D, bt, bi, cnt);
        }
    }
    best_t = bt;
    return bi;
}

// Camera records in the launch (tiny scenes, WAVE bit 32).  For a scene of
// at most kTinyMax triangles the host computes, per camera, every triangle's
// camera cone and edge records (cone_record, in double), its tricam record
// (the values Triangle.cpp:139-160 computes for a ray from the camera) and
// its dmin (no reported hit nearer), sorted nearest first, and passes them BY
// VALUE with the kernel launch — no camera prepass, no per-camera arrays:
// the records arrive by scalar loads from the kernel-argument segment.
// A tile's triangles are a bit mask: triangle j is kept iff the camera wave
// test passes for a cone that holds every ray of the tile — axis = the
// direction of the tile's lane 36 (pixel (8tx + 4, py0 + 4), clamped like
// every lane, so every lane's pixel lies within 4 pixels of it in each
// axis), half-angle = wbound, the analytic bound on that spread (the host's
// tile_wbound).  That is the camera buffer's test with the tile's measured
// cone replaced by a provably wider one, so the kept set holds every
// triangle any ray of the tile can be reported hitting.  A camera's first two
// frames on a stream (WAVE bit 64) compute each tile's mask in the trace
// kernel itself — lane j tests triangle j, one ballot —, the second also
// stores it (bit 128, rt_camhost.h tiny_masks); its later frames on that
// stream read it (one scalar load).
constexpr int kTinyMax = 20;
struct TinyCam {
    int n;       // listed triangles (never-hit ones left out)
    int masked;  // 1: tile masks hold (rows aligned to the tile grid); 0: test every listed triangle
    int tiles_x, tiles_y;
    float cosW, sinW, chord, pad;  // the tile cone's width (wbound), as wave_cone would hold it
    unsigned* mask;                // per tile of the full frame: bit j = keep triangle j
    // per triangle, nearest first: the mask planes (cone, edge 0, edge 1,
    // edge 2 paired as TinyLane holds them), the tricam record [0] [1] [2]
    // [3 = tq, file index, dmin, unused]
    float4 rec[8 * kTinyMax];
};

// The tile's mask, computed by the wave: lane j < n tests triangle j against
// the tile cone around lane 36's direction (full wave: depth-0 kernels run
// every lane).  The camera wave test (cone_overlap, edges_open) at the fixed
// tile width is four half-space tests of that direction: dot(w, p.xyz) >=
// p.w, with the planes and thresholds made on the host (tiny_build, margins
// widened by 1e-6 over the wave test's, which covers the fused products
// here), so the test is two packed FMA chains and four compares.  The
// lane's planes are loaded at the top of the kernel (tiny_lane_load), so
// their latency hides under the ray set-up.
struct TinyLane {
    float4 q[4];  // planes (0, 1) and (2, 3) paired: [x0 x1 y0 y1] [z0 z1 w0 w1] [x2 x3 y2 y3] [z2 z3 w2 w3]
};
// Only the lanes of listed triangles load (each wave reads n x 64 B through
// its CU's L1, not 64 x 64 B: A/B -1.4% on a moving C2 camera).
__device__ __forceinline__ TinyLane tiny_lane_load(const TinyCam& T)
{
    const int lane = (int)(threadIdx.x & 63);
    TinyLane L{};
    if (lane < T.n) {
        const float4* r = T.rec + 8 * lane;
        L = TinyLane{{r[0], r[1], r[2], r[3]}};
    }
    return L;
}
__device__ __forceinline__ unsigned tiny_tile_mask(const TinyCam& T, const TinyLane& L, const Vec3 D)
{
    typedef float f2 __attribute__((ext_vector_type(2)));
    const float wx = readlanef(D.x, 36), wy = readlanef(D.y, 36), wz = readlanef(D.z, 36);
    const f2 X = {wx, wx}, Y = {wy, wy}, Z = {wz, wz};
    f2 a = Z * f2{L.q[1].x, L.q[1].y}, b = Z * f2{L.q[3].x, L.q[3].y};
    a = __builtin_elementwise_fma(Y, f2{L.q[0].z, L.q[0].w}, a);
    b = __builtin_elementwise_fma(Y, f2{L.q[2].z, L.q[2].w}, b);
    a = __builtin_elementwise_fma(X, f2{L.q[0].x, L.q[0].y}, a);
    b = __builtin_elementwise_fma(X, f2{L.q[2].x, L.q[2].y}, b);
    const bool keep = ((int)(threadIdx.x & 63) < T.n) & (a.x >= L.q[1].z) & (a.y >= L.q[1].w) & (b.x >= L.q[3].z) &
                      (b.y >= L.q[3].w);
    return (unsigned)__ballot(keep);
}

// Closest hit for camera rays from the launch's records: planes and quadrics
// first, then the tile's kept triangles nearest first (tile < 0 or no masks:
// every listed triangle), leaving once every lane holds a hit nearer than
// the next dmin (t >= dmin > best: no later triangle can win or tie).
// SELF: the wave computed the tile's mask (tmask, tiny_tile_mask); else it
// reads the stored one.
template <bool SELF>
__device__ __forceinline__ int closest_hit_camera_tiny(const SceneDev& S, const TinyCam& T, int tile, unsigned tmask,
                                                       const Vec3 O, const Vec3 D, float& best_t, Counters& cnt)
{
    unsigned m = T.n >= 32 ? ~0u : (1u << T.n) - 1u;
    if (T.masked && tile >= 0) {
        if constexpr (SELF) {
            m = tmask;
        } else {
            m = T.mask[tile];  // wave-uniform (scalar) load
        }
    }
    float bt = -1.0f;
    int bi = -1;
    for (int k = 0; k < S.n_plane; ++k) {
        const float4 a = S.plane[2 * k], b = S.plane[2 * k + 1];
        float t;
        ++cnt.pla;
        const bool ok = hit_plane(make_float4(0.f, a.x, a.y, a.z), make_float4(a.w, 0.f, 0.f, 0.f), O, D, t);
        take_min(ok, t, __float_as_int(b.x), bt, bi);
    }
    for (int k = 0; k < S.n_quad; ++k) {
        const float4* r = S.quad + 3 * k;
        const float4 a = r[0], b = r[1], c = r[2];
        float t;
        ++cnt.qua;
        const bool ok = hit_quadric(make_float4(0.f, a.x, a.y, a.z), make_float4(a.w, b.x, b.y, b.z),
                                    make_float4(b.w, c.x, c.y, 0.f), O, D, t);
        take_min(ok, t, __float_as_int(c.z), bt, bi);
    }
    while (m) {
        const int j = (int)__builtin_ctz(m);
        m &= m - 1u;
        const float4* r = T.rec + 8 * j + 4;
        const float4 d = r[3];
        if (!__any((bi < 0) | !(bt < d.z))) break;
        camera_tri(r[0], r[1], r[2], d, D, bt, bi, cnt);
    }
    best_t = bt;
    return bi;
}

// Primary rays: wave-culled when the whole wave is here, else per lane.
// WAVE: 0 per lane only, 1 wave-level culling, 2 wave-level two-level
// (clustered) culling.
// tile >= 0: the wave is that camera-buffer tile (WAVE bit 8).
template <int WAVE>
__device__ __forceinline__ int closest_hit_primary(const SceneDev& S, const Vec3 O, const Vec3 D, float& t,
                                                   Counters& cnt, int tile = -1, const TinyCam* T = nullptr,
                                                   unsigned tmask = 0)
{
    if constexpr ((WAVE & 32) != 0) return closest_hit_camera_tiny<(WAVE & 64) != 0>(S, *T, tile, tmask, O, D, t, cnt);
    if ((WAVE & 8) && tile >= 0 && wave_full())
        return closest_hit_camera_list<(WAVE & 2) != 0>(S, tile, O, D, t, cnt);
    if ((WAVE & 3) > 0 && wave_full()) {
        const WaveCone wc = wave_cone(D, true);
        if (wc.ok) return closest_hit_camera_wave<(WAVE & 3) == 2>(S, wc, O, D, t, cnt);
    }
    return S.use_tricam ? closest_hit_camera(S, O, D, t, cnt) : closest_hit<true>(S, O, D, t, cnt);
}

// tricam[k] for camera position C: the camera-ray triangle values that
// depend only on the origin (written by rt_cone_prepass's camera launch).
__host__ __device__ inline void camera_record(const float4* __restrict__ tri, int k, float cx, float cy, float cz,
                                              float4* __restrict__ tricam)
{
    const float4 a = tri[3 * k], b = tri[3 * k + 1], c = tri[3 * k + 2];
    const Vec3 p0 = make3(a.x, a.y, a.z), e1 = make3(a.w, b.x, b.y), e2 = make3(b.z, b.w, c.x);
    const Vec3 Sv = make3(cx, cy, cz) - p0;
    const Vec3 Q = cross(Sv, e1);
    const float tq = dot(e2, Q);
    float4* o = tricam + 4 * k;
    o[0] = make_float4(e1.x, e1.y, e1.z, e2.x);
    o[1] = make_float4(e2.y, e2.z, Sv.x, Sv.y);
    o[2] = make_float4(Sv.z, Q.x, Q.y, Q.z);
    o[3] = make_float4(tq, c.y, 0.f, 0.f);
}

// Cone records for apex A (one thread per triangle, in double).
//
// Culling a triangle for a ray that misses its bounding cone is exact only if
// the reference's float test could not have reported a hit for that ray
// either.  Its rounding (Triangle.cpp:127-172 in f32, eps = 2^-24) gives,
// with S = origin - p0, L = longest edge, N = e1 x e2, a = |D . N|/|N|:
//   u, v, u+v  within  x = k (rho + 2 delta)  of their exact values,
//   delta = 9 eps |S| L / |det|,  rho = 7 eps L^2 / |det| + 3 eps,
//   k = 1/(1 - rho_cap),  rho_cap = rho at the reference's |det| >= 0.01 gate,
// so a reported hit means the ray crosses the plane within 3 x L of the
// triangle, i.e. within G/a + tau, G = gS |S| + gL, tau = 9 k eps L (coef[]
// holds gS, gL, rho_cap).  The cone is built on the sphere grown by a margin
// m, so a culled ray is safe where G/a + tau <= m (well conditioned); where
// it is nearly parallel to the plane it crosses it far away instead:
// dist(X, tri) >= h/a - (h + dv + r), h = the apex's distance to the plane.
// One of the two holds for EVERY a iff
//   h >= G (m + Rp) / (m - tau)            (Rp = h + dv + r),
// which fixes m per pair: 1% of r, or what this needs (up to 10 r; beyond
// that the pair is never culled).  Shadow rays have |S| <= dist + dv + r, so
// the condition holds up to a distance cap (c1.z; m is sized so that the
// cap reaches dtarget).  In the well conditioned case the reference's t errs
// by <= m/3: dmin absorbs it for a sphere beyond P, a second cap on dist for
// a sphere behind the light.  Rounding of the cull test itself: radius
// + 2e-5 dv, cosine - 2e-5.
//
//   camera: c0 = [dir to centre, cosT]   c1 = [dmin, 0, 0, sinT]
//   light : c0 = [dir to centre, cosT]   c1 = [dmin, 2/dmin, dcap, sinT]
//   edges : [n_e, lim] for the three edges (wave-level test only; stored
//           after the n_tri [c0 c1] pairs)
// (sinT >= sin of the angle whose cosine is cosT, for the wave-level test)
// "always test": cosT = -2, sinT = 2, dmin = dcap = -inf, lim = -4.
//
// Edge planes: the plane through A and edge e of the triangle, unit normal
// n_e pointing at the third vertex.  A reported hit puts the crossing X
// within m of the triangle (above), so on the inner side of every edge plane
// up to m, at distance >= s_min = dv - r - m from A: the direction d from A
// has d . n_e >= -m / s_min =: lim for all three edges.  A wave whose cone
// has max d . n_e < lim for some edge reaches no point of the triangle.
// Distance from point a to the triangle (v0, v1, v2), in double (closest
// point by the triangle's Voronoi regions).
__host__ __device__ inline double point_triangle_dist(const double* a, const double (*v)[3])
{
    double ab[3], ac[3], ap[3], cl[3];
    for (int i = 0; i < 3; ++i) {
        ab[i] = v[1][i] - v[0][i];
        ac[i] = v[2][i] - v[0][i];
        ap[i] = a[i] - v[0][i];
    }
    auto dot3 = [](const double* x, const double* y) { return x[0] * y[0] + x[1] * y[1] + x[2] * y[2]; };
    auto at = [&](double s, double t) {
        for (int i = 0; i < 3; ++i) cl[i] = v[0][i] + s * ab[i] + t * ac[i];
    };
    const double d1 = dot3(ab, ap), d2 = dot3(ac, ap);
    double bp[3], cp[3];
    for (int i = 0; i < 3; ++i) {
        bp[i] = a[i] - v[1][i];
        cp[i] = a[i] - v[2][i];
    }
    const double d3 = dot3(ab, bp), d4 = dot3(ac, bp), d5 = dot3(ab, cp), d6 = dot3(ac, cp);
    const double va = d3 * d6 - d5 * d4, vb = d5 * d2 - d1 * d6, vc = d1 * d4 - d3 * d2;
    if (d1 <= 0 && d2 <= 0) at(0, 0);
    else if (d3 >= 0 && d4 <= d3) at(1, 0);
    else if (vc <= 0 && d1 >= 0 && d3 <= 0) at(d1 / (d1 - d3), 0);
    else if (d6 >= 0 && d5 <= d6) at(0, 1);
    else if (vb <= 0 && d2 >= 0 && d6 <= 0) at(0, d2 / (d2 - d6));
    else if (va <= 0 && (d4 - d3) >= 0 && (d5 - d6) >= 0) {
        const double w = (d4 - d3) / ((d4 - d3) + (d5 - d6));
        for (int i = 0; i < 3; ++i) cl[i] = v[1][i] + w * (v[2][i] - v[1][i]);
    } else {
        const double den = 1.0 / (va + vb + vc);
        at(vb * den, vc * den);
    }
    double q = 0;
    for (int i = 0; i < 3; ++i) q += (a[i] - cl[i]) * (a[i] - cl[i]);
    return sqrt(q);
}

__host__ __device__ inline void cone_record(const float4* __restrict__ tri, const float4* __restrict__ sph,
                                            const float4* __restrict__ nrm, const float4* __restrict__ coef, int n,
                                            float ax, float ay, float az, int camera, float dtarget,
                                            float4* __restrict__ out, float4* __restrict__ tricam, int k)
{
    // the camera's tricam records in the same launch (one kernel less per
    // camera: ~5 us of a moving frame's chain at C3)
    if (tricam) camera_record(tri, k, ax, ay, az, tricam);
    const float4 s = sph[k], nr = nrm[k], cf = coef[k], p0 = tri[3 * k];
    const double vx = (double)s.x - ax, vy = (double)s.y - ay, vz = (double)s.z - az;
    const double dv = sqrt(vx * vx + vy * vy + vz * vz);
    const double r0 = s.w, L = nr.w, gS = cf.x, gL = cf.y, rho_cap = cf.z;
    const double h = fabs(nr.x * ((double)ax - p0.x) + nr.y * ((double)ay - p0.y) + nr.z * ((double)az - p0.z));
    // float normal (the additive term, and 1e-3 h); the shadow ray's line
    // passes within 1e-6 dist of A, <= 1e-2 h while dist <= 1e4 h (the cap below)
    const double h_eff = 0.989 * h - 1e-6 * (dv + r0);
    const double tau = 18.0 * 0x1p-24 * L;                // k <= 2
    const double Rp = 1.011 * h + dv + r0 + 1e-6 * dv;
    // |S| bound and the G the margin must cover
    const double G = gS * ((camera ? 0.0 : (double)dtarget * 1.0001) + dv + r0) + gL;
    double m = 0.01 * r0;
    if (h_eff > 1.01 * G) m = fmax(m, 1.001 * (h_eff * tau + 1.01 * G * Rp) / (h_eff - 1.01 * G));
    const double rc = r0 + m + 2e-5 * dv;  // cone radius
    float4 c0 = make_float4(0.f, 0.f, 0.f, -2.0f);
    float4 c1 = make_float4(-INFINITY, 0.f, -INFINITY, 2.0f);
    bool never = false;
    // dmin: a reported hit's plane crossing X lies within m of the triangle
    // and its t within m/3 of X's, so no hit is reported nearer the apex than
    // (nearest point of the triangle) - 4m/3.  The triangle's own nearest
    // point (>= the sphere's, dv - r0), less the cone's 2e-5 dv rounding slack.
    double dnear = dv - r0;
    {
        const float4 t1 = tri[3 * k + 1], t2 = tri[3 * k + 2];
        const double Vt[3][3] = {{p0.x, p0.y, p0.z},
                                 {(double)p0.x + p0.w, (double)p0.y + t1.x, (double)p0.z + t1.y},
                                 {(double)p0.x + t1.z, (double)p0.y + t1.w, (double)p0.z + t2.x}};
        const double Ap[3] = {ax, ay, az};
        const double dt = point_triangle_dist(Ap, Vt);
        if (dt == dt) dnear = fmax(dnear, dt * (1.0 - 1e-9));
    }
    // m <= 10 r: wider cones cost more than the pairs they would cull
    // (a wide member cone widens its cluster's cone and floods light-buffer
    // cells; measured with m <= dv/2 for lights: C3 +7%, C5 +4%)
    if (rho_cap >= 0.0 && h_eff > 1.01 * G && m <= 10.0 * r0 && m > 2.0 * tau && dv - rc > m / 3.0 + 0.02 &&
        isfinite(dv) && isfinite(gS) && isfinite(gL)) {
        const double phi = 1.01 * (m + Rp) / (m - tau);
        // cosine margin 2e-6 >= the per-lane test's rounding: float dot
        // (3 x 2^-24), float unit c0 (1e-7), |L| - 1 (3 x 2^-24), float cosT
        // (6e-8): 5.4e-7 in all
        const double cosT = sqrt(1.0 - (rc / dv) * (rc / dv)) - 2e-6;
        const float4 cone = make_float4((float)(vx / dv), (float)(vy / dv), (float)(vz / dv), (float)cosT);
        const float sinT = (float)(sqrt(fmax(0.0, 1.0 - (double)cone.w * cone.w)) + 1e-7);
        if (camera) {
            if (h_eff >= (gS * (dv + r0) + gL) * phi) {
                // dmin: no reported hit of this triangle has t < dmin (the
                // near-regime t error is <= m/3) — the closest-hit early exit
                const double dmin = (dnear - 4.0 * m / 3.0 - 2e-5 * dv) * (1.0 - 1e-5);
                c0 = cone;
                c1 = make_float4((float)dmin, 0.f, 0.f, sinT);
            }
        } else {
            const double dmin = (dnear - 4.0 * m / 3.0 - 2e-5 * dv) * (1.0 - 1e-5);
            const double dcap1 = ((h_eff / phi - gL) / gS - dv - r0) / 1.0001;
            const double rhoN = fmin(m / (3.0 * L), rho_cap);  // rho where well conditioned
            const double dcap2 =
                rhoN > 0.0 ? ((dv - rc) * (1.0 - rhoN) - m / 3.0) / rhoN / 1.01 : INFINITY;
            const double dcap = fmin(fmin(dcap1, dcap2), 1e4 * h);
            if (dcap > 0.0) {
                c0 = cone;
                c1 = make_float4((float)dmin, (float)(2.0 / dmin), (float)(dcap * (1.0 - 1e-6)), sinT);
            }
        }
    }
    // Never reported: the reference rejects |det| < 0.01, so a hit needs
    // a = |D . N^| >= amin = (0.01 - 7 eps L^2) / |N|, and then the line's
    // crossing X with the plane lies within M = G/amin + tau of the triangle
    // (the bound above, for every a >= amin).  The line passes within
    // dl = 1e-6 |S| of the apex (exactly through it for camera rays), so
    // |X - apex| <= (h + dl)/amin + dl: when that keeps X farther than
    // r0 + M from the sphere centre, no ray from the apex (shadow rays up to
    // the cap) can be reported — whatever its direction.  Such a pair gets a
    // record no test passes (cosT 2, dmin +inf), also in place of a cone
    // record whose cap falls short of dtarget.
    const bool weak = !(c0.w > 0.0f) || (!camera && !(c1.z >= dtarget));
    if (weak && rho_cap >= 0.0 && cf.w > 0.0f && isfinite(dv) && isfinite(gS) && isfinite(gL)) {
        const double nn = cf.w;
        const double amin = (0.0099999 - 7.07 * 0x1p-24 * L * L) / (nn * (1.0 + 1e-6));
        if (amin > 0.0) {
            const double smax = (camera ? 0.0 : (double)dtarget * 1.0001) + dv + r0;
            const double M = 1.01 * ((gS * smax + gL) / amin + tau);
            const double dl = camera ? 0.0 : 1e-6 * (double)dtarget * 1.0001;
            const double hup = 1.01 * h + 1e-5 * (dv + r0);
            if (dv - r0 - M - (hup + dl) / amin - dl > 1e-3 * dv + 0.01) {
                never = true;
                c0 = make_float4((float)(vx / dv), (float)(vy / dv), (float)(vz / dv), 2.0f);
                c1 = make_float4(INFINITY, 0.f, camera ? 0.f : dtarget, 0.f);
            }
        }
    }
    float4 ce[3];
    for (int e = 0; e < 3; ++e) ce[e] = make_float4(0.f, 0.f, 0.f, -4.0f);
    if (c0.w > 0.0f && !never) {  // a culled pair: add its edge planes
        const float4 b1 = tri[3 * k + 1], c2r = tri[3 * k + 2];
        const double V[3][3] = {{p0.x, p0.y, p0.z},
                                {(double)p0.x + p0.w, (double)p0.y + b1.x, (double)p0.z + b1.y},
                                {(double)p0.x + b1.z, (double)p0.y + b1.w, (double)p0.z + c2r.x}};
        const double smin = dv - r0 - m;
        const float lim = (float)(-m / smin - 1e-5);
        bool good = smin > 0.0;
        for (int e = 0; e < 3 && good; ++e) {
            const int i = e, j = (e + 1) % 3, q = (e + 2) % 3;
            const double ax_ = V[i][0] - ax, ay_ = V[i][1] - ay, az_ = V[i][2] - az;
            const double bx_ = V[j][0] - ax, by_ = V[j][1] - ay, bz_ = V[j][2] - az;
            double nx = ay_ * bz_ - az_ * by_, ny = az_ * bx_ - ax_ * bz_, nz = ax_ * by_ - ay_ * bx_;
            const double nn = sqrt(nx * nx + ny * ny + nz * nz);
            const double side = nx * (V[q][0] - ax) + ny * (V[q][1] - ay) + nz * (V[q][2] - az);
            if (!(nn > 0.0) || !isfinite(nn) || side == 0.0) {
                good = false;
                break;
            }
            const double sg = side > 0.0 ? 1.0 : -1.0;
            ce[e] = make_float4((float)(sg * nx / nn), (float)(sg * ny / nn), (float)(sg * nz / nn), lim);
        }
        if (!good)
            for (int e = 0; e < 3; ++e) ce[e] = make_float4(0.f, 0.f, 0.f, -4.0f);
    }
    out[2 * k] = c0;
    out[2 * k + 1] = c1;
    float4* oe = out + 2 * (size_t)n + 3 * k;
    oe[0] = ce[0];
    oe[1] = ce[1];
    oe[2] = ce[2];
}
__global__ void rt_cone_prepass(const float4* __restrict__ tri, const float4* __restrict__ sph,
                                const float4* __restrict__ nrm, const float4* __restrict__ coef, int n, float ax,
                                float ay, float az, int camera, float dtarget, float4* __restrict__ out,
                                float4* __restrict__ tricam)
{
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k < n) cone_record(tri, sph, nrm, coef, n, ax, ay, az, camera, dtarget, out, tricam, k);
}

// Cluster records for one apex (one thread per 64-triangle cluster, in
// double), from the members' [c0 c1] records.  A member's wave test passes
// only if  w . v_k >= cos(W' + T_k) - 3e-6  (W' = W widened by the angular
// slack, T_k = acos(cosT_k), 2e-6 margin + 1e-6 rounding), i.e. only if
// angle(w, v_k) <= W' + T_k + d0 with d0 = arccos(1 - 3e-6) < 2.5e-3.  Then
// angle(w, a) <= W' + T_k + d0 + angle(a, v_k) <= W' + T_c for
//   T_c = max_k (angle(a, v_k) + T_k) + 2.5e-3,
// and the cluster test (the same form, its slack >= every member's) passes:
// a surviving member always has a surviving cluster.  A member that is
// always tested (cosT <= 0), or T_c >= 80 degrees, makes the cluster always
// tested.  For lights: dmin = min, 2/dmin = max, dcap = min over the members.
// csize: members per cluster (64; or n for the union record of small lists).
// One wave per cluster (4 per 256-thread block): lane i takes members
// k0 + i, k0 + i + 64, ...; the axis sum is a fixed butterfly in double (the
// record is deterministic; any axis works: T_c is measured from the float
// axis the test uses).  Round 3: one thread per cluster took 54 us at C3
// (782 clusters on 13 waves, 64 dependent loads each), this ~2 us.
__device__ __forceinline__ double wave_sum_dbl(double v)
{
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    return v;
}
__device__ __forceinline__ double wave_min_dbl(double v)
{
    for (int o = 32; o > 0; o >>= 1) v = fmin(v, __shfl_xor(v, o));
    return v;
}
__device__ __forceinline__ double wave_max_dbl(double v)
{
    for (int o = 32; o > 0; o >>= 1) v = fmax(v, __shfl_xor(v, o));
    return v;
}
__device__ __forceinline__ void cluster_record(const float4* __restrict__ cone, int n, int c, int csize,
                                               float4* __restrict__ out)
{
    const int lane = (int)(threadIdx.x & 63);
    const long long k0 = (long long)csize * c, k1 = min((long long)n, k0 + csize);
    double ax = 0, ay = 0, az = 0, dmin = INFINITY, inv = 0.0, dcap = INFINITY;
    bool always = false;
    for (long long k = k0 + lane; k < k1; k += 64) {
        const float4 c0 = cone[2 * k], c1 = cone[2 * k + 1];
        always |= !(c0.w > 0.0f);
        const double vn = sqrt((double)c0.x * c0.x + (double)c0.y * c0.y + (double)c0.z * c0.z);
        ax += c0.x / vn;
        ay += c0.y / vn;
        az += c0.z / vn;
        dmin = fmin(dmin, (double)c1.x);
        inv = fmax(inv, (double)c1.y);
        dcap = fmin(dcap, (double)c1.z);
    }
    always = __any(always);
    ax = wave_sum_dbl(ax);
    ay = wave_sum_dbl(ay);
    az = wave_sum_dbl(az);
    dmin = wave_min_dbl(dmin);
    inv = wave_max_dbl(inv);
    dcap = wave_min_dbl(dcap);
    const double an = sqrt(ax * ax + ay * ay + az * az);
    float4 q0 = make_float4(0.f, 0.f, 0.f, -2.0f);
    float4 q1 = make_float4(-INFINITY, 0.f, -INFINITY, 2.0f);
    if (!always && an > 0.0 && isfinite(an)) {
        // the float axis the test uses, normalised in double for the angles
        const float4 a = make_float4((float)(ax / an), (float)(ay / an), (float)(az / an), 0.f);
        const double al = sqrt((double)a.x * a.x + (double)a.y * a.y + (double)a.z * a.z);
        double Tc = 0.0;
        for (long long k = k0 + lane; k < k1; k += 64) {
            const float4 c0 = cone[2 * k];
            const double vx = c0.x, vy = c0.y, vz = c0.z;
            const double cx = a.y * vz - a.z * vy, cy = a.z * vx - a.x * vz, cz = a.x * vy - a.y * vx;
            const double ang = atan2(sqrt(cx * cx + cy * cy + cz * cz), a.x * vx + a.y * vy + a.z * vz);
            Tc = fmax(Tc, ang + acos(fmin(1.0, (double)c0.w)));
        }
        Tc = wave_max_dbl(Tc);
        Tc = Tc * (1.0 + 1e-9) + 2.5e-3 + 1e-6 + 4.0 * fabs(al - 1.0);
        if (Tc < 1.396) {  // 80 degrees
            q0 = make_float4(a.x, a.y, a.z, (float)(cos(Tc) - 1e-7));
            q1 = make_float4((float)(dmin * (1.0 - 1e-6)), (float)(inv * (1.0 + 1e-6)), (float)(dcap * (1.0 - 1e-6)),
                             (float)(sin(Tc) + 1e-7));
        }
    }
    if (lane == 0) {
        out[2 * c] = q0;
        out[2 * c + 1] = q1;
    }
}
__global__ __launch_bounds__(256) void rt_cluster_prepass(const float4* __restrict__ cone, int n, int nclu,
                                                          float4* __restrict__ out, int csize = 64)
{
    const int c = (int)(blockIdx.x * 4 + (threadIdx.x >> 6));
    if (c < nclu) cluster_record(cone, n, c, csize, out);  // wave-uniform
}
inline unsigned cluster_blocks(int nclu) { return (unsigned)((nclu + 3) / 4); }

// Small lists' per-camera records in ONE launch (one workgroup): every
// triangle's camera cone record (and tricam record), then — after the
// barrier, in the same workgroup — the union record over them; the same
// functions as rt_cone_prepass + rt_cluster_prepass, so the same bits, with
// one launch (and its dispatch gap) less per moving camera.
constexpr int kCameraSmallMax = 1024;  // triangles (the small-list bound)
__global__ __launch_bounds__(256) void rt_camera_small(const float4* __restrict__ tri, const float4* __restrict__ sph,
                                                       const float4* __restrict__ nrm,
                                                       const float4* __restrict__ coef, int n, float ax, float ay,
                                                       float az, float4* __restrict__ cone_out,
                                                       float4* __restrict__ tricam, float4* __restrict__ uni)
{
    for (int k = (int)threadIdx.x; k < n; k += (int)blockDim.x)
        cone_record(tri, sph, nrm, coef, n, ax, ay, az, 1, 0.0f, cone_out, tricam, k);
    __syncthreads();
    if (threadIdx.x < 64) cluster_record(cone_out, n, 0, n, uni);
}

// Camera cluster records in increasing dmin (rank sort; ties by id), the
// cluster id in q1.y (unused by camera tests).  One wave per cluster, 64
// keys per ballot (round 3; one thread per cluster walking every key took
// 107 us at C3).  A NaN key ranks as -inf (a total order: distinct ranks).
__device__ __forceinline__ float cluster_key(float k) { return k == k ? k : -INFINITY; }
__global__ __launch_bounds__(256) void rt_cluster_sort(const float4* __restrict__ in, int nclu,
                                                       float4* __restrict__ out)
{
    const int lane = (int)(threadIdx.x & 63);
    const int c = (int)(blockIdx.x * 4 + (threadIdx.x >> 6));
    if (c >= nclu) return;  // wave-uniform
    const float key = cluster_key(in[2 * c + 1].x);
    unsigned rank = 0;
    for (int j0 = 0; j0 < nclu; j0 += 64) {
        const int j = j0 + lane;
        bool lt = false;
        if (j < nclu) {
            const float kj = cluster_key(in[2 * j + 1].x);
            lt = (kj < key) | ((kj == key) & (j < c));
        }
        rank += (unsigned)__popcll(__ballot(lt));
    }
    if (lane == 0) {
        float4 q1 = in[2 * c + 1];
        q1.y = __int_as_float(c);
        out[2 * rank] = in[2 * c];
        out[2 * rank + 1] = q1;
    }
}

}  // namespace rt
#endif  // RT_AMD_RT_CULL_H
