// rt_kernels.hip — the hot path on gfx950 (MI355X) and the device half of the
// C ABI (include/rt.h).
//
// What runs here replaces, per pixel, the reference's CPU loop
// (Scene.cpp:1538-1561) -> ObtenirCouleur (:1705) -> ObtenirCouleurSurIntersection
// (:1740, plus the commented reflect/refract block :1779-1823 when
// max_bounces > 0) -> ObtenirFiltreDeSurface (:1842), and the primitive tests
// CTriangle/CPlan/CQuadrique::Intersection (Triangle.cpp:127, Plan.cpp:128,
// Quadrique.cpp:160).  It is NOT a translation of shaders/rayTracing.glsl.
//
// Execution model:
//  * one wave64 = one 8x8 pixel tile, lane l -> (l&7, l>>3); a 256-thread
//    workgroup covers 16x16 pixels (4 tiles);
//  * the surface list is walked in FILE ORDER by every lane of the wave in
//    lockstep, so the surface index, its type switch and its 64-byte record are
//    wave-uniform: records arrive through the scalar data cache (s_load) into
//    SGPRs and feed the VALU directly — no per-lane gather, no LDS round trip;
//  * closest hit keeps (t, index) only; the hit normal is rebuilt once for the
//    winner (bit-identical: same expressions, same inputs);
//  * shadow rays multiply the transmittance filter in file order and leave the
//    surface loop as soon as every active lane's filter is exactly +0 (only
//    when the host proved all filter factors are non-negative and finite, so
//    the skipped factors could not have changed a single bit);
//  * bounces (depth > 0) run as an explicit per-lane DFS with a compile-time
//    sized frame stack instead of recursion, folding each node's colour
//    bottom-up in the reference's order: ((local + C_refl*Kr) + C_refr*Kt);
//  * no FMA contraction, IEEE f32 division and sqrt.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdlib>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/rt.h"
#include "rt_fastmath.h"
#include "rt_math.h"

#pragma clang fp contract(off)

#ifndef RT_TRI_UNROLL
#define RT_TRI_UNROLL 1
#endif
#define RT_PRAGMA(x) _Pragma(#x)
#define RT_UNROLL(n) RT_PRAGMA(unroll n)

namespace rt {

// ------------------------------------------------------------ device layout
// 64-byte surface record, FILE ORDER (4 x float4):
//   word 0         : kind (int bits)
//   triangle       : p0 [1..3]  e1=p1-p0 [4..6]  e2=p2-p0 [7..9]  n [10..12]
//   plane          : n [1..3]   cst [4]
//   quadric        : quad [1..3] mix [4..6] lin [7..9] cst [10]
//   words 13..15   : shadow filter factor  colour * Kt  (Scene.cpp:1857-1858)
// Edges are the reference's own per-test subtractions (Triangle.cpp:135-136)
// hoisted to upload time: same operands, same IEEE subtraction, same bits.
// Material (3 x float4): [r g b Ka] [Kd Ks shin Kr] [Kt ior 0 0]
// Light    (2 x float4): [x y z I]  [r g b 0]
// Cone records per apex, rt_cone_prepass: kConeRec float4 per triangle, as
// [2 x n_tri: c0 c1 per triangle][3 x n_tri: the three edge planes].
constexpr int kConeRec = 5;
#ifndef RT_EDGES
#define RT_EDGES 1
#endif

struct SceneDev {
    const float4* __restrict__ geom;    // file order, 64-byte records (above)
    const float4* __restrict__ mat;
    const float4* __restrict__ lights;
    // Per-kind arrays for the closest-hit and any-hit loops (48/32/48 bytes),
    // each carrying its FILE index; opaque surfaces come first in each array.
    //   tri  : [p0 e1.x] [e1.y e1.z e2.x e2.y] [e2.z idx 0 0]
    //   plane: [n cst]   [idx 0 0 0]
    //   quad : [quad mix.x] [mix.y mix.z lin.x lin.y] [lin.z cst idx 0]
    const float4* __restrict__ tri;
    const float4* __restrict__ plane;
    const float4* __restrict__ quad;
    const int* __restrict__ translucent;  // file indices with a non-zero filter factor, file order
    // Camera-ray form of tri[] for the frame's camera position C (same order):
    //   [e1 e2.x] [e2.y e2.z S.x S.y] [S.z Q] [tQ idx 0 0]
    // with S = C - p0, Q = S x e1, tQ = e2 . Q — exactly the values
    // Triangle.cpp:139-160 computes for a ray whose origin is C, so they are
    // computed once per camera instead of once per pixel.
    const float4* __restrict__ tricam;
    // Camera records are 64 B (vs 40 B); while the triangle list fits the
    // scalar cache they win (C2: -3%), past it the extra misses lose (C3: +10%,
    // tools/ab_variants.py), so the host enables them for small lists only.
    int use_tricam;
    // wave-level edge-plane test on sphere survivors (small triangle lists:
    // loose spheres of large triangles; on big lists it costs more than it
    // culls — C2 -22%, C3 +14%, tools/ab_variants.py)
    int use_edges;
    // Bounding-cone culling (exact: it only skips triangles no lane's ray can
    // reach).  Per (apex, triangle), 2 float4: [dir-to-sphere-centre, cosT]
    // [distance from the apex to the sphere, 1/that, 0, 0], where the sphere
    // bounds the triangle (inflated for float slop) and cosT is the cosine of
    // the half-angle it subtends from the apex minus a margin.  Apex = the
    // camera (cone_cam) or light l (cone_light + kConeRec*n_tri*l).
    const float4* __restrict__ cone_cam;
    const float4* __restrict__ cone_light;
    // Two-level culling for big lists: one [c0 c1] record per apex and
    // 64-triangle cluster (tri[] is in cluster order, kd_order), built by
    // rt_cluster_prepass from its members' records; n_clu = 0: off.
    const float4* __restrict__ clu_cam;
    const float4* __restrict__ clu_light;
    int n_clu;
    int n_surf, n_lights;
    int n_tri, n_plane, n_quad;
    int n_tri_opaque, n_plane_opaque, n_quad_opaque;
    int n_translucent;
    // 1: every filter factor is finite and >= +0, so a ray that meets any
    //    fully opaque surface (factor exactly (0,0,0)) has a filter of exactly
    //    (+0,+0,+0) whatever the order — opaque surfaces are then an any-hit
    //    test (stop at the first hit, by kind), and only the translucent ones
    //    are multiplied, in file order.  0: the file-order product over all.
    int shadow_split;
    // Light buffer (shadow cells): per light, a cube map of lb_R x lb_R cells
    // per face around the light; cell c lists (64-byte entries, nearest to
    // the light first) every opaque triangle whose light cone record can
    // reach a ray whose direction falls in c (rt_lb_* kernels).
    // lb_off[meta.off + c] .. [+ c + 1] index lb_ent; lb_dcap holds, per
    // light, the triangles whose cull is not valid up to meta.dcov (sorted by
    // that distance cap).  lb_R = 0: off.
    int lb_R;
    const unsigned* __restrict__ lb_off;
    const float4* __restrict__ lb_ent;
    const float4* __restrict__ lb_dcap;
    const float4* __restrict__ lb_meta;  // per light: [off base, dcap base, n dcap, dcov] (ints as float bits)
    // Small lists (no clusters): ONE cluster record over all triangles for
    // the camera (uni[0..1]) and over the opaque ones for each light
    // (uni[2 + 2l ..]); nullptr: none.
    const float4* __restrict__ uni;
    // Camera buffer (depth-0 kernels, WAVE bit 8): per 8x8 tile of the full
    // frame (tile = row/8 * cb_tiles_x + col/8), the triangles the tile's
    // wave cone can reach (the camera wave test), with a key = min dmin of
    // the entry and every later one; cb_flag[tile] != 0: no list (per-wave
    // path).  Built once per camera (rt_cb_build).  cb_tiles_x = 0: none.
    const unsigned* __restrict__ cb_off;
    const int2* __restrict__ cb_ent;
    const unsigned* __restrict__ cb_flag;
    int cb_tiles_x;
};

struct FrameDev {
    float cam[3];
    float orient[16];
    float half_w, half_h, inv_w, inv_h;
    float bg[3];
    int width, height, row_begin, row_end;
    int max_bounces;
    float min_energy, scene_ior;
    int flags;
    int band_rows, band_count, band_index;  // band_rows > 0: cyclic row bands (rt.h)
};

struct StatsDev {
    unsigned long long primary, bounce, shadow, skipped, tri, pla, qua, pad;
};
// Stats tallies land in kStatSlots copies (by block) so the atomics of a
// launch spread over many addresses instead of serialising on one.
constexpr int kStatSlots = 256;
constexpr unsigned kXcds = 8;  // MI355X: 8 XCDs, one L2 each
#ifndef RT_XCD_CHUNK
#define RT_XCD_CHUNK 4
#endif

// Per-lane tallies (RT_FLAG_STATS): rays, and the exact ray-primitive tests
// the lane's wave executed (a wave-level test counts once per lane).
struct Counters {
    unsigned primary = 0, bounce = 0, shadow = 0, skipped = 0;
    unsigned tri = 0, pla = 0, qua = 0;
#ifdef RT_PROF  // diagnostic build (tools/prof_sections.py): shader clocks per section
    unsigned long long pt[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    unsigned long long last = 0;
    unsigned ev[8] = {0, 0, 0, 0, 0, 0, 0, 0};  // event counts (wave-uniform)
#endif
};
#ifdef RT_PROF
#define RT_MARK(cnt, i)                                           \
    do {                                                          \
        __builtin_amdgcn_sched_barrier(0);                        \
        const unsigned long long t_ = __builtin_amdgcn_s_memtime(); \
        __builtin_amdgcn_sched_barrier(0);                        \
        (cnt).pt[i] += t_ - (cnt).last;                           \
        (cnt).last = t_;                                          \
    } while (0)
__device__ unsigned long long rt_prof_acc[8];
#define RT_EV(cnt, i) (++(cnt).ev[i])
__device__ unsigned long long rt_prof_ev[8];
// per-tile record (16 x u32: total clocks lo/hi, 8 section clocks >> 8, events 1 2 4 5 6 7)
__device__ unsigned* rt_prof_tiles;
__device__ int rt_prof_ntiles;
#else
#define RT_EV(cnt, i) ((void)0)
#define RT_MARK(cnt, i) \
    do {                \
    } while (0)
#endif

// ----------------------------------------------------- exact fast reciprocal
// IEEE 1.0f/x in 3 VALU instead of the ~10-instruction division expansion:
// rcp_nr (rt_fastmath.h: v_rcp_f32 then one FMA Newton step), checked by
// tools/fastmath_check.hip against 1.0f/x on gfx950 for EVERY float with |x|
// in [2^-125, 2^125] (4,194,304,002 values, 0 mismatches; v_rcp_f32 alone:
// 448,837,500 mismatches).  Outside that range (and for NaN/Inf) the wave
// takes the IEEE division.  (The same header's exact division and sqrt
// sequences were measured too: their domain guards cost more than they save
// in this kernel, so the compiler's IEEE expansions stay.)
// For Det: lanes with |Det| < EPSILON are rejected whatever InvDet is
// (Triangle.cpp:141-142), so only the others must be in range.
__device__ __forceinline__ float recip_det(float det)
{
    const float a = fabsf(det);
    const bool need_ieee = !(a <= 0x1p125f) & !(a < kEps);
    if (__builtin_expect(__any(need_ieee), 0)) return 1.0f / det;
    return rcp_nr(det);
}

// --------------------------------------------------------- primitive tests
// Each returns whether the reference's Intersection() would set a surface,
// and the distance it would report.

// Triangle.cpp:127-172 (Moller-Trumbore).  Early outs become predicates.
__device__ __forceinline__ bool hit_triangle(const float4 a, const float4 b, const float4 c,
                                             const Vec3 O, const Vec3 D, float& t)
{
    const Vec3 p0 = make3(a.y, a.z, a.w);
    const Vec3 e1 = make3(b.x, b.y, b.z);
    const Vec3 e2 = make3(b.w, c.x, c.y);
    const Vec3 P = cross(D, e2);
    const float det = dot(e1, P);
    const float inv = recip_det(det);
    const Vec3 S = O - p0;
    const float u = dot(S, P) * inv;
    const Vec3 Q = cross(S, e1);
    const float v = dot(D, Q) * inv;
    t = dot(e2, Q) * inv;
    return !(fabsf(det) < kEps) & !((u < 0) | (u > 1)) & !((v < 0) | (u + v > 1));
}

// Plan.cpp:128-144
__device__ __forceinline__ bool hit_plane(const float4 a, const float4 b, const Vec3 O, const Vec3 D,
                                          float& t)
{
    const Vec3 n = make3(a.y, a.z, a.w);
    const float vd = dot(n, D);
    t = -(dot(n, O) + b.x) / vd;
    return fabsf(vd) > kEps;
}

// Quadrique.cpp:171-194 — the three coefficients, expression trees verbatim.
struct QuadCoef {
    float A, B, C;
};
__device__ __forceinline__ QuadCoef quad_coef(const float4 a, const float4 b, const float4 c,
                                              const Vec3 o, const Vec3 d)
{
    const Vec3 q = make3(a.y, a.z, a.w);
    const Vec3 m = make3(b.x, b.y, b.z);
    const Vec3 l = make3(b.w, c.x, c.y);
    const float cst = c.z;
    QuadCoef k;
    k.A = d.x * (q.x * d.x + m.z * d.y + m.y * d.z) + d.y * (q.y * d.y + m.x * d.z) + d.z * (q.z * d.z);
    k.B = d.x * (q.x * o.x + 0.5f * (m.z * o.y + m.y * o.z + l.x)) +
          d.y * (q.y * o.y + 0.5f * (m.z * o.x + m.x * o.z + l.y)) +
          d.z * (q.z * o.z + 0.5f * (m.y * o.x + m.x * o.y + l.z));
    k.C = o.x * (q.x * o.x + m.z * o.y + m.y * o.z + l.x) + o.y * (q.y * o.y + m.x * o.z + l.y) +
          o.z * (q.z * o.z + l.z) + cst;
    return k;
}
// Quadrique.cpp:196-248 (root choice: min, else max if min < EPS, accept if !(t<0);
// degenerate A == 0 branch always reports -0.5*(C/B)).
__device__ __forceinline__ bool hit_quadric(const float4 a, const float4 b, const float4 c,
                                            const Vec3 O, const Vec3 D, float& t)
{
    const QuadCoef k = quad_coef(a, b, c, O, D);
    if (k.A != 0.0f) {
        const float Ka = -k.B / k.A;
        const float Kb = k.C / k.A;
        float delta = Ka * Ka - Kb;
        const bool pos = delta > 0;
        delta = sqrtf(delta);
        const float t0 = Ka - delta;
        const float t1 = Ka + delta;
        float dist = t0 < t1 ? t0 : t1;
        if (dist < kEps) dist = t0 > t1 ? t0 : t1;
        t = dist;
        return pos && !(dist < 0);
    }
    t = -0.5f * (k.C / k.B);
    return true;
}

// Quadrique.cpp:214-237 / :243-246 — rebuilt only for the winning quadric.
__device__ __forceinline__ Vec3 quadric_normal(const float4 a, const float4 b, const float4 c,
                                               const Vec3 O, const Vec3 D, float t)
{
    const QuadCoef k = quad_coef(a, b, c, O, D);
    const Vec3 q = make3(a.y, a.z, a.w);
    const Vec3 m = make3(b.x, b.y, b.z);
    const Vec3 l = make3(b.w, c.x, c.y);
    if (k.A != 0.0f) {
        const Vec3 hp = O + t * D;
        Vec3 n;
        n.x = 2.0f * q.x * hp.x + m.y * hp.z + m.z * hp.y + l.x;
        n.y = 2.0f * q.y * hp.y + m.x * hp.z + m.z * hp.x + l.y;
        n.z = 2.0f * q.z * hp.z + m.x * hp.y + m.y * hp.x + l.z;
        return normalize(n);
    }
    return normalize(l);
}

__device__ __forceinline__ int kind_of(const float4 a) { return __float_as_int(a.x); }

// Lexicographic (distance, file index) minimum: the reference keeps the first
// surface in file order among equal distances (strict '<', Scene.cpp:1713),
// which is exactly min over (t, index).  That lets each kind run in its own
// loop without changing a single winner.
__device__ __forceinline__ void take_min(bool ok, float t, int idx, float& bt, int& bi)
{
    if (ok & (t > kEps) & ((bi < 0) | (t < bt) | ((t == bt) & (idx < bi)))) {
        bt = t;
        bi = idx;
    }
}

// Triangle test split at the u bound so a wave can drop a triangle that no
// lane's ray crosses the u-range of (exact: the skipped values could only have
// produced rejections).
struct TriU {
    Vec3 S, P;
    float inv, u;
    bool ok;
};
__device__ __forceinline__ TriU tri_u(const Vec3 p0, const Vec3 e1, const Vec3 e2, const Vec3 O, const Vec3 D)
{
    TriU r;
    r.P = cross(D, e2);
    const float det = dot(e1, r.P);
    r.inv = recip_det(det);
    r.S = O - p0;
    r.u = dot(r.S, r.P) * r.inv;
    r.ok = !(fabsf(det) < kEps) & !((r.u < 0) | (r.u > 1));
    return r;
}
__device__ __forceinline__ bool tri_vt(const TriU& r, const Vec3 e1, const Vec3 e2, const Vec3 D, float& t)
{
    const Vec3 Q = cross(r.S, e1);
    const float v = dot(D, Q) * r.inv;
    t = dot(e2, Q) * r.inv;
    return r.ok & !((v < 0) | (r.u + v > 1));
}

struct TriRec {
    Vec3 p0, e1, e2;
    int idx;
};
__device__ __forceinline__ TriRec load_tri(const SceneDev& S, int k)
{
    const float4* r = S.tri + 3 * k;
    const float4 a = r[0], b = r[1], c = r[2];
    return TriRec{make3(a.x, a.y, a.z), make3(a.w, b.x, b.y), make3(b.z, b.w, c.x), __float_as_int(c.y)};
}

// Scene.cpp:1705-1715: closest hit over every surface.  Returns the winning
// FILE index (-1 = miss) and its distance.
template <bool CAMERA>
__device__ __forceinline__ int closest_hit(const SceneDev& S, const Vec3 O, const Vec3 D, float& best_t, Counters& cnt)
{
    float bt = -1.0f;
    int bi = -1;
    RT_UNROLL(RT_TRI_UNROLL)
    for (int k = 0; k < S.n_tri; ++k) {
        if constexpr (CAMERA) {  // rays from the camera: skip triangles outside every lane's cone
            const float4 c = S.cone_cam[2 * k];
            if (!__any(dot(D, make3(c.x, c.y, c.z)) >= c.w)) continue;
        }
        const TriRec tr = load_tri(S, k);
        ++cnt.tri;
        const TriU r = tri_u(tr.p0, tr.e1, tr.e2, O, D);
        if (!__any(r.ok)) continue;
        float t;
        const bool ok = tri_vt(r, tr.e1, tr.e2, D, t);
        take_min(ok, t, tr.idx, bt, bi);
    }
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
        // repack into the file-order record layout hit_quadric reads
        const bool ok = hit_quadric(make_float4(0.f, a.x, a.y, a.z), make_float4(a.w, b.x, b.y, b.z),
                                    make_float4(b.w, c.x, c.y, 0.f), O, D, t);
        take_min(ok, t, __float_as_int(c.z), bt, bi);
    }
    best_t = bt;
    return bi;
}

// One camera-ray triangle test: exact u first, the rest only if some lane of
// the wave is inside the u bounds.
__device__ __forceinline__ void camera_tri(const float4 a, const float4 b, const float4 c, const float4 d,
                                           const Vec3 D, float& bt, int& bi, Counters& cnt)
{
    ++cnt.tri;
    const Vec3 e1 = make3(a.x, a.y, a.z), e2 = make3(a.w, b.x, b.y);
    const Vec3 Sv = make3(b.z, b.w, c.x), Q = make3(c.y, c.z, c.w);
    const Vec3 P = cross(D, e2);
    const float det = dot(e1, P);
    const float inv = recip_det(det);
    const float u = dot(Sv, P) * inv;
    const bool okU = !(fabsf(det) < kEps) & !((u < 0) | (u > 1));
    if (!__any(okU)) return;
    const float v = dot(D, Q) * inv;
    const float t = d.x * inv;
    take_min(okU & !((v < 0) | (u + v > 1)), t, __float_as_int(d.y), bt, bi);
}

// Closest hit for camera rays (origin = the camera for every lane), per-lane
// culling (partial waves): the per-triangle values that depend only on the
// origin come from tricam[].
__device__ __forceinline__ int closest_hit_camera(const SceneDev& S, const Vec3 O, const Vec3 D, float& best_t,
                                                  Counters& cnt)
{
    float bt = -1.0f;
    int bi = -1;
    for (int k = 0; k < S.n_tri; ++k) {
        const float4 cc = S.cone_cam[2 * k];
        if (!__any(dot(D, make3(cc.x, cc.y, cc.z)) >= cc.w)) continue;
        const float4* r = S.tricam + 4 * k;
        camera_tri(r[0], r[1], r[2], r[3], D, bt, bi, cnt);
    }
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
    best_t = bt;
    return bi;
}

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

// One batch of 64 triangles [k0, k0 + 64) for the wave's camera rays: one
// lane per triangle against the wave cone, exact tests on the survivors.
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
    if (RT_EDGES && S.use_edges && reach) reach = edges_open(wc, S.cone_cam + 2 * S.n_tri + 3 * k, 0.0f);
    RT_EV(cnt, 1);
    unsigned long long m = __ballot(reach);
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
                camera_wave_batch(S, wc, 64 * cid, O, D, bt, bi, cnt, wave_max(bi >= 0 ? bt : INFINITY));
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

// Closest hit for camera rays from the tile's camera-buffer list (the wave
// is the tile: full, rows aligned).  Planes and quadrics first (their hits
// tighten the exit); then the list in cluster order, leaving once every
// lane holds a hit nearer than the entry's key (no later entry can report a
// nearer or equal hit: t >= dmin > best, as in the cluster early exit).
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
    const unsigned e1 = S.cb_off[tile + 1];
    for (unsigned e = S.cb_off[tile]; e < e1; ++e) {
        const int2 en = S.cb_ent[e];
        if (!__any((bi < 0) | !(bt < __int_as_float(en.y)))) break;
        RT_EV(cnt, 2);
        const float4* r = S.tricam + 4 * en.x;
        camera_tri(r[0], r[1], r[2], r[3], D, bt, bi, cnt);
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
                                                   Counters& cnt, int tile = -1)
{
    if ((WAVE & 8) && tile >= 0 && wave_full()) return closest_hit_camera_list(S, tile, O, D, t, cnt);
    if ((WAVE & 3) > 0 && wave_full()) {
        const WaveCone wc = wave_cone(D, true);
        if (wc.ok) return closest_hit_camera_wave<(WAVE & 3) == 2>(S, wc, O, D, t, cnt);
    }
    return S.use_tricam ? closest_hit_camera(S, O, D, t, cnt) : closest_hit<true>(S, O, D, t, cnt);
}

// tricam[] for camera position C (one thread per triangle).
__global__ void rt_camera_prepass(const float4* __restrict__ tri, int n, float cx, float cy, float cz,
                                  float4* __restrict__ tricam)
{
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n) return;
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
__device__ double point_triangle_dist(const double* a, const double (*v)[3])
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

__global__ void rt_cone_prepass(const float4* __restrict__ tri, const float4* __restrict__ sph,
                                const float4* __restrict__ nrm, const float4* __restrict__ coef, int n, float ax,
                                float ay, float az, int camera, float dtarget, float4* __restrict__ out)
{
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n) return;
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
__global__ void rt_cluster_prepass(const float4* __restrict__ cone, int n, int nclu, float4* __restrict__ out,
                                   int csize = 64)
{
    const int c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= nclu) return;
    const int k0 = csize * c, k1 = min(n, k0 + csize);
    double ax = 0, ay = 0, az = 0, dmin = INFINITY, inv = 0.0, dcap = INFINITY;
    bool always = false;
    for (int k = k0; k < k1; ++k) {
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
    const double an = sqrt(ax * ax + ay * ay + az * az);
    float4 q0 = make_float4(0.f, 0.f, 0.f, -2.0f);
    float4 q1 = make_float4(-INFINITY, 0.f, -INFINITY, 2.0f);
    if (!always && an > 0.0 && isfinite(an)) {
        // the float axis the test uses, normalised in double for the angles
        const float4 a = make_float4((float)(ax / an), (float)(ay / an), (float)(az / an), 0.f);
        const double al = sqrt((double)a.x * a.x + (double)a.y * a.y + (double)a.z * a.z);
        double Tc = 0.0;
        for (int k = k0; k < k1; ++k) {
            const float4 c0 = cone[2 * k];
            const double vx = c0.x, vy = c0.y, vz = c0.z;
            const double cx = a.y * vz - a.z * vy, cy = a.z * vx - a.x * vz, cz = a.x * vy - a.y * vx;
            const double ang = atan2(sqrt(cx * cx + cy * cy + cz * cz), a.x * vx + a.y * vy + a.z * vz);
            Tc = fmax(Tc, ang + acos(fmin(1.0, (double)c0.w)));
        }
        Tc = Tc * (1.0 + 1e-9) + 2.5e-3 + 1e-6 + 4.0 * fabs(al - 1.0);
        if (Tc < 1.396) {  // 80 degrees
            q0 = make_float4(a.x, a.y, a.z, (float)(cos(Tc) - 1e-7));
            q1 = make_float4((float)(dmin * (1.0 - 1e-6)), (float)(inv * (1.0 + 1e-6)), (float)(dcap * (1.0 - 1e-6)),
                             (float)(sin(Tc) + 1e-7));
        }
    }
    out[2 * c] = q0;
    out[2 * c + 1] = q1;
}

// Camera cluster records in increasing dmin (rank sort, one thread per
// cluster; ties by id), the cluster id in q1.y (unused by camera tests).
__global__ void rt_cluster_sort(const float4* __restrict__ in, int nclu, float4* __restrict__ out)
{
    const int c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= nclu) return;
    const float key = in[2 * c + 1].x;
    int rank = 0;
    for (int j = 0; j < nclu; ++j) {
        const float kj = in[2 * j + 1].x;
        rank += (kj < key) | ((kj == key) & (j < c));
    }
    float4 q1 = in[2 * c + 1];
    q1.y = __int_as_float(c);
    out[2 * rank] = in[2 * c];
    out[2 * rank + 1] = q1;
}

// ------------------------------------------------------------ light buffer
// Haines & Greenberg's light buffer, made exact: a cube map around each
// light.  The direction d from the light to a shading point (d = -L) picks
// the face of its largest |component| and the cell (i, j) of u = a/|m|,
// v = b/|m| on that face (lb_cell).  Every cell has a cone [w, W] (lb_cone,
// in double) containing every float direction the lookup can map to it,
// with the invariants of a wave cone (exact w . d >= cosW + 2e-6 for every
// such d; sinW, chord raised).  So the wave-level predicates cone_overlap and
// edges_open applied to a CELL are the proven wave-level culling with the
// wave's rays replaced by the cell's: a triangle they reject cannot be
// reported by the reference for any ray of the cell whose length is at most
// the distance dcov the angular slack was sized for (lanes beyond it, or
// with a degenerate direction, take the per-lane path).  Cell lists hold the
// kept triangles nearest-first (the per-lane dmin exit); pairs whose cull
// is not valid up to dcov (dcap < dcov, or never culled) are in a separate
// per-light list sorted by dcap, tested by the lanes with dist > dcap — the
// per-lane predicate light_reach, split in two.
constexpr int kLbGroup = 16;  // cells per supercell edge (two-level build)
constexpr int kLbEnt = 3;     // float4 per light-buffer entry (48 B)

__device__ __forceinline__ int lb_cell(const Vec3 d, int R)
{
    const float ax = fabsf(d.x), ay = fabsf(d.y), az = fabsf(d.z);
    int face;
    float m, a, b;
    if ((ax >= ay) & (ax >= az)) {
        face = d.x >= 0.0f ? 0 : 1;
        m = ax; a = d.y; b = d.z;
    } else if (ay >= az) {
        face = d.y >= 0.0f ? 2 : 3;
        m = ay; a = d.z; b = d.x;
    } else {
        face = d.z >= 0.0f ? 4 : 5;
        m = az; a = d.x; b = d.y;
    }
    const float inv = __builtin_amdgcn_rcpf(m);  // ~1 ulp: the cells' 1e-5 margins cover it
    const float h = 0.5f * (float)R;
    int i = (int)floorf((a * inv + 1.0f) * h);
    int j = (int)floorf((b * inv + 1.0f) * h);
    i = min(max(i, 0), R - 1);
    j = min(max(j, 0), R - 1);
    return (face * R + j) * R + i;
}

__device__ __forceinline__ void lb_face_dir(int face, double u, double v, double* o)
{
    switch (face) {
    case 0: o[0] = 1.0; o[1] = u; o[2] = v; break;
    case 1: o[0] = -1.0; o[1] = u; o[2] = v; break;
    case 2: o[0] = v; o[1] = 1.0; o[2] = u; break;
    case 3: o[0] = v; o[1] = -1.0; o[2] = u; break;
    case 4: o[0] = u; o[1] = v; o[2] = 1.0; break;
    default: o[0] = u; o[1] = v; o[2] = -1.0; break;
    }
    const double n = sqrt(o[0] * o[0] + o[1] * o[1] + o[2] * o[2]);
    o[0] /= n; o[1] /= n; o[2] /= n;
}

// Cone of the cells [i0, i1) x [j0, j1) of a face (u range widened by 1e-5
// for the lookup's rounding), its half-angle grown by `widen` (supercells).
// The farthest point of a small geodesically convex cell from its centre
// direction is a corner.  Float |d| = 1 within 1e-6 (sqrt_w/recip_w), float
// w within 1.2e-7 of the unit centre: cosW = cos(W)(1 - 2e-6) - 4e-6 keeps
// exact w.d >= cosW + 2e-6 for every direction of the cells.
__device__ WaveCone lb_cone(int face, int i0, int i1, int j0, int j1, int R, double widen)
{
    const double du = 1e-5;
    const double u0 = 2.0 * i0 / R - 1.0 - du, u1 = 2.0 * i1 / R - 1.0 + du;
    const double v0 = 2.0 * j0 / R - 1.0 - du, v1 = 2.0 * j1 / R - 1.0 + du;
    double w[3];
    lb_face_dir(face, 0.5 * (u0 + u1), 0.5 * (v0 + v1), w);
    double W = 0.0;
    for (int q = 0; q < 4; ++q) {
        double c[3];
        lb_face_dir(face, (q & 1) ? u1 : u0, (q & 2) ? v1 : v0, c);
        const double x = w[1] * c[2] - w[2] * c[1], y = w[2] * c[0] - w[0] * c[2], z = w[0] * c[1] - w[1] * c[0];
        W = fmax(W, atan2(sqrt(x * x + y * y + z * z), w[0] * c[0] + w[1] * c[1] + w[2] * c[2]));
    }
    W = W * (1.0 + 1e-9) + 1e-6 + widen;
    WaveCone k;
    k.w = make3((float)w[0], (float)w[1], (float)w[2]);
    const double cw = cos(W) * (1.0 - 2e-6) - 4e-6;
    float cf = (float)cw;
    if ((double)cf > cw) cf = nextafterf(cf, -INFINITY);
    const double sw = sqrt(fmax(0.0, 1.0 - (double)cf * (double)cf)) + 1e-6;
    float sf = (float)sw;
    if ((double)sf < sw) sf = nextafterf(sf, INFINITY);
    const double ch = sqrt(2.0 * (1.0 - (double)cf)) + 1e-6;
    float chf = (float)ch;
    if ((double)chf < ch) chf = nextafterf(chf, INFINITY);
    k.cosW = cf;
    k.sinW = sf;
    k.chord = chf;
    k.ok = W < 1.0;  // cosW >= 0.54 like every wave cone (>= 0.5)
    return k;
}

// May a ray of cone wc (up to length dcov) need light record k?  The shadow
// wave batch's predicate with dmax = dcov, minus its dcap term (the dcap
// list), with the edge planes always.  Never-culled pairs: the dcap list.
__device__ __forceinline__ bool lb_keep(const WaveCone& wc, const float4 c0, const float4 c1, const float4* e,
                                        float dcov)
{
    if (!(c0.w > 0.0f) || !(c1.x < dcov)) return false;
    if (!wc.ok) return true;
    const float ang = dcov * 1e-6f * c1.y;
    return cone_overlap(wc, c0, c1.w, ang) && edges_open(wc, e, ang);
}

// Build pass 1: per supercell (16 x 16 cells, cone widened by 1e-3 rad so
// that rejecting a triangle for it implies rejecting it for each of its
// cells), the triangles of `perm` (nearest-first) it keeps, in order
// (block-ordered compaction).  lists == nullptr: counts only.
__global__ __launch_bounds__(256) void rt_lb_super(const float4* __restrict__ cone, int n, const int* __restrict__ perm,
                                                   int np, int R, float dcov, const unsigned* __restrict__ offs,
                                                   unsigned* __restrict__ counts, int* __restrict__ lists)
{
    const int G = R / kLbGroup;
    const int s = blockIdx.x;
    const int face = s / (G * G), rem = s % (G * G), sj = rem / G, si = rem % G;
    const WaveCone wc = lb_cone(face, si * kLbGroup, si * kLbGroup + kLbGroup, sj * kLbGroup, sj * kLbGroup + kLbGroup,
                                R, 1e-3);
    __shared__ unsigned wtot[4];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    unsigned total = 0;
    const unsigned base = lists ? offs[s] : 0u;
    for (int q0 = 0; q0 < np; q0 += 256) {
        const int q = q0 + (int)threadIdx.x;
        int k = -1;
        bool keep = false;
        if (q < np) {
            k = perm[q];
            keep = lb_keep(wc, cone[2 * k], cone[2 * k + 1], cone + 2 * (size_t)n + 3 * (size_t)k, dcov);
        }
        const unsigned long long b = __ballot(keep);
        const unsigned pre = (unsigned)__popcll(b & ((1ull << lane) - 1ull));
        if (lane == 0) wtot[wv] = (unsigned)__popcll(b);
        __syncthreads();
        unsigned off = 0;
        for (int w = 0; w < wv; ++w) off += wtot[w];
        const unsigned blk = wtot[0] + wtot[1] + wtot[2] + wtot[3];
        if (lists && keep) lists[base + total + off + pre] = k;
        total += blk;
        __syncthreads();
    }
    if (!lists && threadIdx.x == 0) counts[s] = total;
}

// 48-byte light-buffer entry of triangle k (its tri[] record):
//   [p0, key] [e1, e2.x] [e2.y e2.z, 0, 0]
// key = dmin (cell lists) or dcap (dcap list).  (A per-lane cone test in
// front of the exact test was measured to spare no wave any exact test: a
// cell's list is already what its lanes' cones can reach.)
__device__ __forceinline__ void lb_write(float4* o, const float4* __restrict__ tri, int k, float key)
{
    const float4 a = tri[3 * k], b = tri[3 * k + 1], c = tri[3 * k + 2];
    o[0] = make_float4(a.x, a.y, a.z, key);
    o[1] = make_float4(a.w, b.x, b.y, b.z);
    o[2] = make_float4(b.w, c.x, 0.0f, 0.0f);
}

// Build pass 2: one thread per cell of a supercell, over the supercell's
// list (staged in LDS), in order.  ent == nullptr: counts only.
__global__ __launch_bounds__(256) void rt_lb_cells(const float4* __restrict__ cone, int n, const float4* __restrict__ tri,
                                                   int R, float dcov, const unsigned* __restrict__ soffs,
                                                   const int* __restrict__ slists, const unsigned* __restrict__ coffs,
                                                   unsigned* __restrict__ ccounts, float4* __restrict__ ent)
{
    const int G = R / kLbGroup;
    const int s = blockIdx.x;
    const int face = s / (G * G), rem = s % (G * G), sj = rem / G, si = rem % G;
    const int i = si * kLbGroup + (int)(threadIdx.x & 15), j = sj * kLbGroup + (int)(threadIdx.x >> 4);
    const int cell = (face * R + j) * R + i;
    const WaveCone wc = lb_cone(face, i, i + 1, j, j + 1, R, 0.0);
    __shared__ float4 rec[256 * kConeRec];
    __shared__ int kid[256];
    const unsigned b0 = soffs[s], b1 = soffs[s + 1];
    unsigned cnt = 0, out = ent ? coffs[cell] : 0u;
    for (unsigned q0 = b0; q0 < b1; q0 += 256) {
        __syncthreads();
        const unsigned q = q0 + threadIdx.x;
        if (q < b1) {
            const int k = slists[q];
            kid[threadIdx.x] = k;
            rec[kConeRec * threadIdx.x] = cone[2 * k];
            rec[kConeRec * threadIdx.x + 1] = cone[2 * k + 1];
            for (int e = 0; e < 3; ++e) rec[kConeRec * threadIdx.x + 2 + e] = cone[2 * (size_t)n + 3 * (size_t)k + e];
        }
        __syncthreads();
        const int m = (int)min(256u, b1 - q0);
        for (int x = 0; x < m; ++x) {
            const float4 c0 = rec[kConeRec * x], c1 = rec[kConeRec * x + 1];
            if (!lb_keep(wc, c0, c1, rec + kConeRec * x + 2, dcov)) continue;
            if (ent) lb_write(ent + kLbEnt * (size_t)out++, tri, kid[x], c1.x);
            else ++cnt;
        }
    }
    if (!ent) ccounts[cell] = cnt;
}

// The dcap list of one light: entries of perm (sorted by dcap), key = dcap.
__global__ void rt_lb_dcap(const float4* __restrict__ cone, const float4* __restrict__ tri, const int* __restrict__ perm,
                           int m, float4* __restrict__ out)
{
    const int q = blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= m) return;
    const int k = perm[q];
    const float4 c0 = cone[2 * k], c1 = cone[2 * k + 1];
    lb_write(out + kLbEnt * (size_t)q, tri, k, c1.z == c1.z ? c1.z : -INFINITY);
}

// ---------------------------------------------------------- camera buffer
// One wave per 8x8 tile of the full frame, laid out like rt_trace_kernel
// (256-thread blocks of 2 x 2 tiles): the tile's 64 camera rays (camera_dir
// on the same clamped pixels as the trace kernel, so the same bits), their
// wave cone, and the camera wave test of every cluster / member
// (cone_overlap, and the edge planes) — the culling closest_hit_camera_wave
// runs per frame, done once per camera.  COUNT: cnt[tile] = survivors;
// else the survivors {triangle, dmin} in cluster order from off[tile].
template <bool FILL>
__global__ __launch_bounds__(256) void rt_cb_build(const SceneDev S, const FrameDev F, const unsigned* __restrict__ off,
                                                   unsigned* __restrict__ cnt, unsigned* __restrict__ flag,
                                                   int2* __restrict__ ent)
{
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int tx = blockIdx.x * 2 + (wave & 1), ty = blockIdx.y * 2 + (wave >> 1);
    if (tx * 8 >= F.width || ty * 8 >= F.height) return;
    const int tile = ty * S.cb_tiles_x + tx;
    const int px = tx * 8 + (lane & 7), py = ty * 8 + (lane >> 3);
    const Vec3 D = camera_dir(F, px < F.width ? px : F.width - 1, py < F.height ? py : F.height - 1);
    const WaveCone wc = wave_cone(D, true);
    if (!wc.ok) {  // no list: the trace kernel's per-wave path
        if (!FILL && lane == 0) {
            flag[tile] = 1u;
            cnt[tile] = 0u;
        }
        return;
    }
    unsigned n = 0, base = FILL ? off[tile] : 0u;
    const unsigned long long below = (1ull << lane) - 1ull;
    auto batch = [&](int k0) {
        const int k = k0 + lane;
        bool reach = false;
        float dmin = 0.0f;
        if (k < S.n_tri) {
            const float4 c0 = S.cone_cam[2 * k], c1 = S.cone_cam[2 * k + 1];
            dmin = c1.x;
            reach = cone_overlap(wc, c0, c1.w, 0.0f) && edges_open(wc, S.cone_cam + 2 * (size_t)S.n_tri + 3 * k, 0.0f);
        }
        const unsigned long long m = __ballot(reach);
        if (FILL && reach) ent[base + n + (unsigned)__popcll(m & below)] = make_int2(k, __float_as_int(dmin));
        n += (unsigned)__popcll(m);
    };
    if (S.n_clu > 0) {
        for (int c0i = 0; c0i < S.n_clu; c0i += 64) {
            const int cl = c0i + lane;
            float4 q0 = make_float4(0.f, 0.f, 0.f, 1.f), q1 = make_float4(INFINITY, 0.f, 0.f, 0.f);
            if (cl < S.n_clu) {
                q0 = S.clu_cam[2 * cl];
                q1 = S.clu_cam[2 * cl + 1];
            }
            const int id = __float_as_int(q1.y);
            unsigned long long cm = __ballot(cone_overlap(wc, q0, q1.w, 0.0f, 4e-6f));
            while (cm) {
                const int b = (int)__builtin_ctzll(cm);
                cm &= cm - 1;
                batch(64 * __builtin_amdgcn_readlane(id, b));
            }
        }
    } else {
        for (int k0 = 0; k0 < S.n_tri; k0 += 64) batch(k0);
    }
    if (!FILL && lane == 0) {
        cnt[tile] = n;
        flag[tile] = 0u;
    }
}

// Keys: entry e's key = min dmin over entries [e, end) of its tile (one
// thread per tile), so a wave may stop at the first key beyond its hits.
__global__ void rt_cb_keys(const unsigned* __restrict__ off, int ntiles, int2* __restrict__ ent)
{
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= ntiles) return;
    float m = INFINITY;
    for (unsigned e = off[t + 1]; e > off[t]; --e) {
        const float d = __int_as_float(ent[e - 1].y);
        m = d == d ? fminf(m, d) : -INFINITY;
        ent[e - 1].y = __float_as_int(m);
    }
}

// Shadow-ray cull predicate (L normalised towards the light, dist to it):
// the segment reaches the sphere's distance and the cone, or the lane lies
// beyond the distance the culling argument covers (c1.z).
__device__ __forceinline__ bool light_reach(const float4 c0, const float4 c1, const Vec3 L, float dist, float slack)
{
    return ((c1.x < dist) & (-dot(L, make3(c0.x, c0.y, c0.z)) >= c0.w - slack * c1.y)) | (dist > c1.z);
}

__device__ __forceinline__ Vec3 hit_normal(const SceneDev& S, int idx, const Vec3 O, const Vec3 D, float t)
{
    const float4* rec = S.geom + 4 * idx;
    const float4 a = rec[0], b = rec[1], c = rec[2], d = rec[3];
    const int kind = kind_of(a);
    if (kind == RT_TRIANGLE) return make3(c.z, c.w, d.x);
    if (kind == RT_PLANE) return make3(a.y, a.z, a.w);
    return quadric_normal(a, b, c, O, D, t);
}

struct Mat {
    Color color;
    float ka, kd, ks, shin, kr, kt, ior;
};
__device__ __forceinline__ Mat load_mat(const SceneDev& S, int idx)
{
    const float4 m0 = S.mat[3 * idx], m1 = S.mat[3 * idx + 1], m2 = S.mat[3 * idx + 2];
    return Mat{{m0.x, m0.y, m0.z}, m0.w, m1.x, m1.y, m1.z, m1.w, m2.x, m2.y};
}

// An opaque plane against a shadow ray: Plan.cpp:128-144 and the filter's
// window EPS < t < dist (Scene.cpp:1853).  t = -num / vd is only divided
// out when some lane could pass: never when |vd| <= EPS, when num and vd
// share a sign (t <= 0), or when |num| < 0.0099 |vd| (then |t| < EPS even
// after rounding) — the common cases of points above a ground plane and of
// points on it.
__device__ __forceinline__ bool shadow_plane_hit(const float4 a, const Vec3 P, const Vec3 L, float dist)
{
    const Vec3 n = make3(a.x, a.y, a.z);
    const float vd = dot(n, L);
    const float num = dot(n, P) + a.w;
    const bool maybe = (fabsf(vd) > kEps) & (((num < 0) & (vd > 0)) | ((num > 0) & (vd < 0))) &
                       !(fabsf(num) < 0.0099f * fabsf(vd));
    if (!__any(maybe)) return false;
    const float t = -num / vd;
    return (fabsf(vd) > kEps) & (t > kEps) & (t < dist);
}

// One file-order surface record against a shadow ray (generic path).
__device__ __forceinline__ bool shadow_hit_record(const float4* rec, const Vec3 P, const Vec3 L, float dist,
                                                  Color& fc, Counters& cnt)
{
    const float4 a = rec[0], b = rec[1], c = rec[2], d = rec[3];
    float t;
    bool ok;
    const int kind = kind_of(a);
    if (kind == RT_TRIANGLE) {
        ++cnt.tri;
        ok = hit_triangle(a, b, c, P, L, t);
    } else if (kind == RT_PLANE) {
        ++cnt.pla;
        ok = hit_plane(a, b, P, L, t);
    } else {
        ++cnt.qua;
        ok = hit_quadric(a, b, c, P, L, t);
    }
    fc = Color{d.y, d.z, d.w};
    return ok & (t > kEps) & (t < dist);
}

// Scene.cpp:1842-1861 ObtenirFiltreDeSurface.  L is the UNNORMALISED light
// vector; it is normalised here exactly like the reference (in place).
__device__ __forceinline__ Color shadow_filter(const SceneDev& S, int light, const Vec3 P, Vec3& L,
                                               Counters& cnt)
{
    Color F{1.0f, 1.0f, 1.0f};
    const float dist = norm(L);
    L = div_recip(L, dist);
    if (!S.shadow_split) {
        // General case: the product over every surface in file order.
        for (int i = 0; i < S.n_surf; ++i) {
            Color fc;
            if (shadow_hit_record(S.geom + 4 * i, P, L, dist, fc, cnt)) F *= fc;
        }
        return F;
    }
    // Opaque surfaces: any hit zeroes the filter exactly.  A lane stops
    // counting once occluded; the wave leaves a loop once all lanes are.
    bool occluded = false;
    int done = 0, total = S.n_tri_opaque + S.n_plane_opaque + S.n_quad_opaque;
    const float4* cone = S.cone_light + kConeRec * (size_t)S.n_tri * light;
    // The float ray P + t*L (L normalised, |L - exact| <= ~6 ulp) can stray
    // from the exact segment to the light by <= dist * 1e-6 at distance
    // >= cone.y from the light: widen each lane's cone by that angle.
    const float slack = dist * 1e-6f;
    for (int k = 0; k < S.n_tri_opaque; ++k) {
        if (!__any(!occluded)) break;
        ++done;
        const float4 c0 = cone[2 * k], c1 = cone[2 * k + 1];
        const bool reach = !occluded & light_reach(c0, c1, L, dist, slack);
        if (!__any(reach)) continue;
        const TriRec tr = load_tri(S, k);
        ++cnt.tri;
        const TriU r = tri_u(tr.p0, tr.e1, tr.e2, P, L);
        if (!__any(r.ok && !occluded)) continue;
        float t;
        const bool ok = tri_vt(r, tr.e1, tr.e2, L, t);
        occluded |= ok & (t > kEps) & (t < dist);
    }
    for (int k = 0; k < S.n_plane_opaque; ++k) {
        if (!__any(!occluded)) break;
        ++done;
        const float4 a = S.plane[2 * k];
        float t;
        ++cnt.pla;
        const bool ok = hit_plane(make_float4(0.f, a.x, a.y, a.z), make_float4(a.w, 0.f, 0.f, 0.f), P, L, t);
        occluded |= ok & (t > kEps) & (t < dist);
    }
    for (int k = 0; k < S.n_quad_opaque; ++k) {
        if (!__any(!occluded)) break;
        ++done;
        const float4* r = S.quad + 3 * k;
        const float4 a = r[0], b = r[1], c = r[2];
        float t;
        ++cnt.qua;
        const bool ok = hit_quadric(make_float4(0.f, a.x, a.y, a.z), make_float4(a.w, b.x, b.y, b.z),
                                    make_float4(b.w, c.x, c.y, 0.f), P, L, t);
        occluded |= ok & (t > kEps) & (t < dist);
    }
    cnt.skipped += (unsigned)(total - done);
    if (occluded) return Color{0.0f, 0.0f, 0.0f};
    // Translucent surfaces, file order (the relative order of the factors the
    // reference multiplies is preserved; unhit opaque surfaces contribute none).
    for (int j = 0; j < S.n_translucent; ++j) {
        Color fc;
        if (shadow_hit_record(S.geom + 4 * S.translucent[j], P, L, dist, fc, cnt)) F *= fc;
    }
    return F;
}


// Scene.cpp:1742-1777: ambient + every light (N.L gate on the unnormalised
// light vector, filter, Lambert "Gouraud" term, Phong term).
// Shadow rays of up to LB lights from the same point P, against the OPAQUE
// surfaces, in one pass over the surface list (shadow_split scenes only).
// Each light's any-hit result is exactly the per-light loop's; sharing the
// pass shares the record loads, the loop overhead and the light-independent
// part of the triangle test (S = P - p0, Q = S x e1, e2 . Q — the same
// values Triangle.cpp:143-158 computes for every light's ray from P).
// This is the per-lane-culled form (partial waves, bounce rays); full waves
// of depth-0 kernels use shadow_opaque_wave.
template <int kLightBatch>
__device__ __forceinline__ void shadow_opaque_batch(const SceneDev& S, int l0, int nl, const Vec3 P,
                                                    const Vec3 (&L)[kLightBatch], const float (&dist)[kLightBatch],
                                                    bool (&occ)[kLightBatch], Counters& cnt)
{
    const float4* cone = S.cone_light + kConeRec * (size_t)S.n_tri * l0;
    const size_t cstride = kConeRec * (size_t)S.n_tri;
    float slack[kLightBatch];
#pragma unroll
    for (int j = 0; j < kLightBatch; ++j) slack[j] = dist[j] * 1e-6f;
    for (int k = 0; k < S.n_tri_opaque; ++k) {
        bool live = false;
#pragma unroll
        for (int j = 0; j < kLightBatch; ++j) live |= (j < nl) & !occ[j];
        if (!__any(live)) break;
        bool reach[kLightBatch];
        bool any_reach = false;
#pragma unroll
        for (int j = 0; j < kLightBatch; ++j) {
            reach[j] = false;
            if (j < nl) {
                const float4 c0 = cone[cstride * j + 2 * k], c1 = cone[cstride * j + 2 * k + 1];
                reach[j] = !occ[j] & light_reach(c0, c1, L[j], dist[j], slack[j]);
                any_reach |= reach[j];
            }
        }
        if (__any(any_reach)) {
            const TriRec tr = load_tri(S, k);
            const Vec3 Sv = P - tr.p0;
            const Vec3 Q = cross(Sv, tr.e1);
            const float tq = dot(tr.e2, Q);
#pragma unroll
            for (int j = 0; j < kLightBatch; ++j) {
                if (j < nl && __any(reach[j])) {
                    ++cnt.tri;
                    const Vec3 Pv = cross(L[j], tr.e2);
                    const float det = dot(tr.e1, Pv);
                    const float inv = recip_det(det);
                    const float u = dot(Sv, Pv) * inv;
                    const float v = dot(L[j], Q) * inv;
                    const float t = tq * inv;
                    const bool ok = !(fabsf(det) < kEps) & !((u < 0) | (u > 1)) & !((v < 0) | (u + v > 1));
                    occ[j] |= ok & (t > kEps) & (t < dist[j]);
                }
            }
        }
    }
    for (int k = 0; k < S.n_plane_opaque; ++k) {
        const float4 a = S.plane[2 * k];
#pragma unroll
        for (int j = 0; j < kLightBatch; ++j) {
            if (j < nl && __any(!occ[j])) {
                ++cnt.pla;
                occ[j] |= shadow_plane_hit(a, P, L[j], dist[j]);
            }
        }
    }
    for (int k = 0; k < S.n_quad_opaque; ++k) {
        const float4* r = S.quad + 3 * k;
        const float4 a = r[0], b = r[1], c = r[2];
#pragma unroll
        for (int j = 0; j < kLightBatch; ++j) {
            if (j < nl && __any(!occ[j])) {
                float t;
                ++cnt.qua;
                const bool ok = hit_quadric(make_float4(0.f, a.x, a.y, a.z), make_float4(a.w, b.x, b.y, b.z),
                                            make_float4(b.w, c.x, c.y, 0.f), P, L[j], t);
                occ[j] |= ok & (t > kEps) & (t < dist[j]);
            }
        }
    }
}

// May some gated lane's shadow ray need any triangle of the union record
// u?  Each lane is taken as a wave of one live lane (the cone wave_cone
// builds for it: w = d, cosW = d.d - 1e-6), so the test is the proven
// cluster test of shadow_opaque_wave with dmax = the lane's dist.
__device__ __forceinline__ bool union_reach(const float4* u, const Vec3 L, float dist, bool gate)
{
    const Vec3 d = -L;
    WaveCone c;
    c.w = d;
    c.cosW = dot(d, d) - 1e-6f;
    c.sinW = __builtin_amdgcn_sqrtf(fmaxf(0.0f, 1.0f - c.cosW * c.cosW)) + 1e-6f;
    c.chord = __builtin_amdgcn_sqrtf(2.0f * (1.0f - c.cosW)) + 1e-6f;
    const float dm = dist == dist ? dist : INFINITY;
    const float4 q0 = u[0], q1 = u[1];
    const bool reach = !(c.cosW >= 0.5f) | ((q1.x < dm) & cone_overlap(c, q0, q1.w, dm * 1e-6f * q1.y, 4e-6f)) |
                       (dm > q1.z);
    return __any(gate & reach);
}

// One batch of 64 opaque triangles [k0, k0 + 64) for the lights in the bit
// set `lights`: one lane per triangle against each light's wave cone, then
// exact any-hit tests on the survivors; the light-independent part of the
// test (S = P - p0, Q = S x e1, e2 . Q) is shared by the lights.
template <int kLightBatch>
__device__ __forceinline__ void shadow_wave_batch(const SceneDev& S, const float4* cone, size_t cstride, int k0,
                                                  unsigned lights, const Vec3 P, const Vec3 (&L)[kLightBatch],
                                                  const float (&dist)[kLightBatch], bool (&occ)[kLightBatch],
                                                  const WaveCone (&wc)[kLightBatch],
                                                  const float (&dmax)[kLightBatch], Counters& cnt)
{
    const int k = k0 + (int)(threadIdx.x & 63);
    // every record load of the batch first (one wait), then the tests
    float4 c0[kLightBatch], c1[kLightBatch], ed[kLightBatch][3];
    const bool edges = RT_EDGES && S.use_edges;
#pragma unroll
    for (int j = 0; j < kLightBatch; ++j) {
        c0[j] = make_float4(0.f, 0.f, 0.f, 1.f);
        c1[j] = make_float4(INFINITY, 0.f, INFINITY, 0.f);  // no reach
        for (int q = 0; q < 3; ++q) ed[j][q] = make_float4(0.f, 0.f, 0.f, -4.0f);  // open
        if (((lights >> j) & 1u) && k < S.n_tri_opaque) {
            const float4* rec = cone + cstride * j + 2 * k;
            c0[j] = rec[0];
            c1[j] = rec[1];
            if (edges) {  // with the sphere records: one memory round trip
                const float4* er = cone + cstride * j + 2 * (size_t)S.n_tri + 3 * k;
                ed[j][0] = er[0];
                ed[j][1] = er[1];
                ed[j][2] = er[2];
            }
        }
    }
    RT_EV(cnt, 4);
    unsigned long long mj[kLightBatch], m = 0;
#pragma unroll
    for (int j = 0; j < kLightBatch; ++j) {
        mj[j] = 0;
        if (((lights >> j) & 1u) && wc[j].ok) {
            const float ang = dmax[j] * 1e-6f * c1[j].y;
            bool reach = (c1[j].x < dmax[j]) & cone_overlap(wc[j], c0[j], c1[j].w, ang);
            if (edges) reach &= edges_open(wc[j], ed[j], ang);
            reach |= dmax[j] > c1[j].z;
            mj[j] = __ballot(reach);
            m |= mj[j];
        }
    }
    RT_MARK(cnt, 3);
    while (m) {
        const int b = (int)__builtin_ctzll(m);
        m &= m - 1;
        const TriRec tr = load_tri(S, k0 + b);
        const Vec3 Sv = P - tr.p0;
        const Vec3 Q = cross(Sv, tr.e1);
        const float tq = dot(tr.e2, Q);
#pragma unroll
        for (int j = 0; j < kLightBatch; ++j) {
            if (((mj[j] >> b) & 1ull) && __any(!occ[j])) {
                RT_EV(cnt, 5);
                ++cnt.tri;
                const Vec3 Pv = cross(L[j], tr.e2);
                const float det = dot(tr.e1, Pv);
                const float inv = recip_det(det);
                const float u = dot(Sv, Pv) * inv;
                const float v = dot(L[j], Q) * inv;
                const float t = tq * inv;
                const bool ok = !(fabsf(det) < kEps) & !((u < 0) | (u > 1)) & !((v < 0) | (u + v > 1));
                occ[j] |= ok & (t > kEps) & (t < dist[j]);
            }
        }
    }
    RT_MARK(cnt, 4);
}

// shadow_opaque_batch with wave-level culling (full wave; every light of the
// batch with a live lane must have ok cones — else the caller uses the
// per-lane form).  Same any-hit results: a triangle no lane of the wave can
// reach is skipped, the rest are tested exactly per lane.
template <int kLightBatch, bool CLU>
__device__ __forceinline__ void shadow_opaque_wave(const SceneDev& S, int l0, int nl, unsigned tmask, const Vec3 P,
                                                   const Vec3 (&L)[kLightBatch], const float (&dist)[kLightBatch],
                                                   bool (&occ)[kLightBatch], const WaveCone (&wc)[kLightBatch],
                                                   const float (&dmax)[kLightBatch], Counters& cnt)
{
    const float4* cone = S.cone_light + kConeRec * (size_t)S.n_tri * l0;
    const size_t cstride = kConeRec * (size_t)S.n_tri;
    const int lane = (int)(threadIdx.x & 63);
    if constexpr (CLU) {
        const float4* clu = S.clu_light + 2 * (size_t)S.n_clu * l0;
        const int ncl = (S.n_tri_opaque + 63) / 64;
        for (int c0i = 0; c0i < ncl; c0i += 64) {
            bool live = false;
#pragma unroll
            for (int j = 0; j < kLightBatch; ++j) live |= (j < nl) & !occ[j];
            if (!__any(live)) break;
            const int cl = c0i + lane;
            unsigned long long cj[kLightBatch], cm = 0;
#pragma unroll
            for (int j = 0; j < kLightBatch; ++j) {
                cj[j] = 0;
                if (j < nl && wc[j].ok) {
                    bool reach = false;
                    if (cl < ncl) {
                        const float4 q0 = clu[2 * (size_t)S.n_clu * j + 2 * cl];
                        const float4 q1 = clu[2 * (size_t)S.n_clu * j + 2 * cl + 1];
                        const float ang = dmax[j] * 1e-6f * q1.y;
                        reach = ((q1.x < dmax[j]) & cone_overlap(wc[j], q0, q1.w, ang, 4e-6f)) | (dmax[j] > q1.z);
#ifdef RT_PROF
                        const bool by_cone = (q1.x < dmax[j]) & cone_overlap(wc[j], q0, q1.w, ang, 4e-6f);
                        cnt.ev[6] += (unsigned)__popcll(__ballot(reach & !by_cone));
                        cnt.ev[7] += (unsigned)__popcll(__ballot(by_cone));
#endif
                    }
                    cj[j] = __ballot(reach);
                    RT_EV(cnt, 3);
                    cm |= cj[j];
                }
            }
            while (cm) {
                const int b = (int)__builtin_ctzll(cm);
                cm &= cm - 1;
                unsigned lights = 0;
#pragma unroll
                for (int j = 0; j < kLightBatch; ++j) lights |= (unsigned)((cj[j] >> b) & 1ull) << j;
                shadow_wave_batch<kLightBatch>(S, cone, cstride, 64 * (c0i + b), lights, P, L, dist, occ, wc, dmax,
                                               cnt);
            }
        }
    } else {
        for (int k0 = 0; k0 < S.n_tri_opaque && tmask; k0 += 64) {
            bool live = false;
#pragma unroll
            for (int j = 0; j < kLightBatch; ++j) live |= (j < nl) & ((tmask >> j) & 1u) & !occ[j];
            if (!__any(live)) break;
            shadow_wave_batch<kLightBatch>(S, cone, cstride, k0, tmask, P, L, dist, occ, wc, dmax, cnt);
        }
    }
    RT_MARK(cnt, 3);
#ifndef RT_ABLATE_SHADOW_PLANE  // timing-only build: no plane shadow tests
    for (int k = 0; k < S.n_plane_opaque; ++k) {
#else
    for (int k = 0; k < 0; ++k) {
#endif
        const float4 a = S.plane[2 * k];
#pragma unroll
        for (int j = 0; j < kLightBatch; ++j) {
            if (j < nl && __any(!occ[j])) {
                ++cnt.pla;
                occ[j] |= shadow_plane_hit(a, P, L[j], dist[j]);
            }
        }
    }
    RT_MARK(cnt, 7);
    for (int k = 0; k < S.n_quad_opaque; ++k) {
        const float4* r = S.quad + 3 * k;
        const float4 a = r[0], b = r[1], c = r[2];
#pragma unroll
        for (int j = 0; j < kLightBatch; ++j) {
            if (j < nl && __any(!occ[j])) {
                float t;
                ++cnt.qua;
                const bool ok = hit_quadric(make_float4(0.f, a.x, a.y, a.z), make_float4(a.w, b.x, b.y, b.z),
                                            make_float4(b.w, c.x, c.y, 0.f), P, L[j], t);
                occ[j] |= ok & (t > kEps) & (t < dist[j]);
            }
        }
    }
}

// One light's shadow rays against the OPAQUE surfaces with the light buffer
// (shadow_split scenes).  occ: in = lanes without a shadow ray, out = also
// the occluded ones (any-hit, so the order of the tests is free).  Each lane
// walks its own cell's list (nearest first, leaving at the first entry that
// lies beyond its point) with the per-lane cone test in front of the exact
// test, then the dcap list while its dist exceeds the entries' caps; lanes
// the buffer does not cover take the per-lane loop over every triangle.
__device__ __forceinline__ void shadow_opaque_lb(const SceneDev& S, int l, const Vec3 P, const Vec3 L, float dist,
                                                 bool& occ, Counters& cnt)
{
    for (int k = 0; k < S.n_plane_opaque; ++k) {
        if (!__any(!occ)) return;
        ++cnt.pla;
        occ |= shadow_plane_hit(S.plane[2 * k], P, L, dist);
    }
    {
    const float4 m0 = S.lb_meta[2 * l], m1 = S.lb_meta[2 * l + 1];
    const unsigned obase = __float_as_uint(m0.x), dbase = __float_as_uint(m0.y), ndcap = __float_as_uint(m0.z);
    const int R = __float_as_int(m0.w);
    const float dcov = m1.x;
    const Vec3 d = -L;
    const float mx = fmaxf(fabsf(d.x), fmaxf(fabsf(d.y), fabsf(d.z)));
    const bool use = !occ & (dist <= dcov) & (mx >= 0.5f) & (R > 0);
    unsigned e = 0, end = 0;
    if (use) {
        const unsigned* o = S.lb_off + obase + lb_cell(d, R);
        e = o[0];
        end = o[1];
    }
    const float slack = dist * 1e-6f;
    RT_MARK(cnt, 3);
    // The next entry's loads are issued before the current entry's exact
    // test (software pipelining of the per-lane gathers).
    float4 r0 = make_float4(0.f, 0.f, 0.f, 0.f), r1 = r0, r2 = r0;
#ifdef RT_ABLATE_LBCELL  // timing-only build: no cell walk
    bool have = false;
#else
    bool have = e < end;
#endif
    if (have) {
        const float4* r = S.lb_ent + kLbEnt * (size_t)e;
        r0 = r[0];
        r1 = r[1];
        r2 = r[2];
    }
    for (;;) {
        const bool act = have & !occ;
        if (!__any(act)) break;
        RT_EV(cnt, 3);
        bool go = false;
        const float4 c0 = r0, c1 = r1, c2 = r2;
        if (act) {
            if (!(c0.w < dist)) {
                have = false;  // this and every later entry lie beyond P (dmin)
            } else {
                go = true;
                ++e;
                have = e < end;
                if (have) {
                    const float4* r = S.lb_ent + kLbEnt * (size_t)e;
                    r0 = r[0];
                    r1 = r[1];
                    r2 = r[2];
                }
            }
        }
        if (__any(go)) {
            ++cnt.tri;
            RT_EV(cnt, 4);
            if (go) {
                const Vec3 e1 = make3(c1.x, c1.y, c1.z), e2 = make3(c1.w, c2.x, c2.y);
                const TriU u = tri_u(make3(c0.x, c0.y, c0.z), e1, e2, P, L);
                if (__any(u.ok)) {  // v and t only where some lane's u is in [0, 1]
                    float t;
                    const bool ok = tri_vt(u, e1, e2, L, t);
                    occ |= ok & (t > kEps) & (t < dist);
                }
            }
        }
    }
    RT_MARK(cnt, 4);
    // pairs not culled up to dcov: sorted by dcap, so once no live lane lies
    // beyond an entry's cap none lies beyond a later one
#ifdef RT_ABLATE_LBLIST  // timing-only build: no per-light list
    for (unsigned q = 0; q < 0; ++q) {
#else
    for (unsigned q = 0; q < ndcap; ++q) {
#endif
        const float4* r = S.lb_dcap + kLbEnt * (size_t)(dbase + q);
        const float4 r0 = r[0];
        const bool need = use & !occ & (dist > r0.w);
        if (!__any(need)) break;
        ++cnt.tri;
        RT_EV(cnt, 5);
        const float4 r1 = r[1], r2 = r[2];
        if (need) {
            const Vec3 e1 = make3(r1.x, r1.y, r1.z), e2 = make3(r1.w, r2.x, r2.y);
            const TriU u = tri_u(make3(r0.x, r0.y, r0.z), e1, e2, P, L);
            if (__any(u.ok)) {
                float t;
                const bool ok = tri_vt(u, e1, e2, L, t);
                occ |= ok & (t > kEps) & (t < dist);
            }
        }
    }
    // lanes the buffer does not cover: every opaque triangle, culled per lane
    if (__any(!occ & !use)) {
        RT_EV(cnt, 6);
        bool o2 = occ | use;
        const float4* cone = S.cone_light + kConeRec * (size_t)S.n_tri * l;
        for (int k = 0; k < S.n_tri_opaque; ++k) {
            if (!__any(!o2)) break;
            const float4 c0 = cone[2 * k], c1 = cone[2 * k + 1];
            const bool reach = !o2 & light_reach(c0, c1, L, dist, slack);
            if (!__any(reach)) continue;
            const TriRec tr = load_tri(S, k);
            ++cnt.tri;
            RT_EV(cnt, 7);
            const TriU r = tri_u(tr.p0, tr.e1, tr.e2, P, L);
            if (!__any(r.ok && !o2)) continue;
            float t;
            const bool ok = tri_vt(r, tr.e1, tr.e2, L, t);
            o2 |= ok & (t > kEps) & (t < dist);
        }
        occ = use ? occ : o2;
    }
    }
    RT_MARK(cnt, 7);
    for (int k = 0; k < S.n_quad_opaque; ++k) {
        if (!__any(!occ)) break;
        const float4* r = S.quad + 3 * k;
        const float4 a = r[0], b = r[1], c = r[2];
        float t;
        ++cnt.qua;
        const bool ok = hit_quadric(make_float4(0.f, a.x, a.y, a.z), make_float4(a.w, b.x, b.y, b.z),
                                    make_float4(b.w, c.x, c.y, 0.f), P, L, t);
        occ |= ok & (t > kEps) & (t < dist);
    }
}

// Scene.cpp:1742-1777: ambient + every light (N.L gate on the unnormalised
// light vector, filter, Lambert "Gouraud" term, Phong term).  Lights are
// accumulated strictly in file order; only the filters of a batch of lights
// are computed ahead (they do not depend on the colour being accumulated).
__device__ __forceinline__ void add_light(Color& res, const Mat& m, const float4 l0, const float4 l1, const Vec3 N,
                                          const Vec3 L, const Vec3 D, const Color F)
{
    const Color LC = Color{l1.x, l1.y, l1.z} * F;
    const float g = l0.w * m.kd * dot(N, L);
    // Exact shortcuts: a term that evaluates to +-0 leaves every non-zero
    // component of res bit-identical, so it is skipped when res has none.
    // The Phong term is +-0 when shin == 0 (pw = 1) and I * ks == 0; the
    // Lambert term when the light is filtered to 0 and g is finite
    // (colours are finite by construction: integers / 255).
    const bool zero_phong = (m.shin == 0.0f) & (l0.w * m.ks == 0.0f);
    const bool dark = (F.r == 0.0f) & (F.g == 0.0f) & (F.b == 0.0f);
    if (zero_phong & dark & (fabsf(g) <= 3.4e38f) & (res.r != 0.0f) & (res.g != 0.0f) & (res.b != 0.0f)) return;
    res += (m.color * g) * LC;
    if (zero_phong & (res.r != 0.0f) & (res.g != 0.0f) & (res.b != 0.0f)) return;
    const Vec3 rf = reflect(L, N);
    const float ps = dot(rf, D);
    if (ps > 0) {
        // pow(x, 0) == 1 for every x (C99 F.9.4.4, glibc and ocml alike):
        // materials without a shininess never pay for powf.
        float pw = 1.0f;
        if (m.shin != 0.0f) pw = powf(ps, m.shin);
        const float pf = l0.w * m.ks * pw;
        res += LC * pf;
    }
}

template <int kLightBatch, int WAVE>
__device__ __forceinline__ Color shade_local(const SceneDev& S, const Mat& m, const Vec3 P, const Vec3 N,
                                             const Vec3 D, Counters& cnt, bool active = true)
{
    // active = false: a lane kept in step with its wave (no hit / outside the
    // frame) whose result is discarded; it casts no shadow rays.
    Color res = m.color * m.ka;
    if (!S.shadow_split) {
        for (int li = 0; li < S.n_lights; ++li) {
            const float4 l0 = S.lights[2 * li], l1 = S.lights[2 * li + 1];
            Vec3 L = make3(l0.x, l0.y, l0.z) - P;
            if (active && dot(L, N) > 0) {
                ++cnt.shadow;
                const Color F = shadow_filter(S, li, P, L, cnt);
                add_light(res, m, l0, l1, N, L, D, F);
            }
        }
        return res;
    }
    if constexpr ((WAVE & 4) != 0) {  // light buffer: one light at a time, file order
        for (int li = 0; li < S.n_lights; ++li) {
            const float4 l0 = S.lights[2 * li], l1 = S.lights[2 * li + 1];
            const Vec3 Lr = make3(l0.x, l0.y, l0.z) - P;
            const bool gate = active & (dot(Lr, N) > 0);  // Scene.cpp:1756, unnormalised
            const float dist = sqrt_w(Lr.x * Lr.x + Lr.y * Lr.y + Lr.z * Lr.z);
            const Vec3 L = Lr * recip_w(dist);
            cnt.shadow += gate;
            bool occ = !gate;
            RT_MARK(cnt, 2);
#ifndef RT_ABLATE_SHADOW
            shadow_opaque_lb(S, li, P, L, dist, occ, cnt);
#endif
            RT_MARK(cnt, 7);
            if (gate) {
                Color F{0.0f, 0.0f, 0.0f};
                if (!occ) {  // translucent surfaces, file order
                    F = Color{1.0f, 1.0f, 1.0f};
                    for (int q = 0; q < S.n_translucent; ++q) {
                        Color fc;
                        if (shadow_hit_record(S.geom + 4 * S.translucent[q], P, L, dist, fc, cnt)) F *= fc;
                    }
                }
                add_light(res, m, l0, l1, N, L, D, F);
            }
            RT_MARK(cnt, 5);
        }
        return res;
    }
    for (int lb = 0; lb < S.n_lights; lb += kLightBatch) {
        const int nl = S.n_lights - lb < kLightBatch ? S.n_lights - lb : kLightBatch;
        Vec3 L[kLightBatch];
        float dist[kLightBatch];
        bool gate[kLightBatch], occ[kLightBatch];
#pragma unroll
        for (int j = 0; j < kLightBatch; ++j) {
            gate[j] = false;
            dist[j] = 0.0f;
            L[j] = make3(0.f, 0.f, 0.f);
            if (j < nl) {
                const float4 l0 = S.lights[2 * (lb + j)];
                const Vec3 Lr = make3(l0.x, l0.y, l0.z) - P;
                gate[j] = active & (dot(Lr, N) > 0);  // Scene.cpp:1756, unnormalised
                // Scene.cpp:1847-1848: norm + one reciprocal, by the exact
                // fast sequences (rt_fastmath.h) when the whole wave is in range
                dist[j] = sqrt_w(Lr.x * Lr.x + Lr.y * Lr.y + Lr.z * Lr.z);
                L[j] = Lr * recip_w(dist[j]);
                cnt.shadow += gate[j];
            }
            occ[j] = !gate[j];
        }
        RT_MARK(cnt, 2);
        bool use_wave = (WAVE & 3) > 0 && wave_full();
        WaveCone wc[kLightBatch];
        float dmax[kLightBatch];
        unsigned tmask = (1u << nl) - 1u;  // lights whose triangles the wave must walk
#ifdef RT_ABLATE_SHADOW_TRI  // timing-only build: no triangle shadow tests
        tmask = 0;
#endif
        if (use_wave) {
#pragma unroll
            for (int j = 0; j < kLightBatch; ++j) {
                wc[j].ok = false;
                dmax[j] = 0.0f;
                if (j < nl && ((tmask >> j) & 1u)) {
                    // no lane's ray can need any triangle: skip the wave cone too
                    if ((WAVE & 3) == 1 && S.uni && !union_reach(S.uni + 2 * (1 + lb + j), L[j], dist[j], gate[j])) {
                        tmask &= ~(1u << j);
                        continue;
                    }
                    wc[j] = wave_cone(-L[j], gate[j]);  // directions from the light
                    dmax[j] = wave_max(gate[j] ? (dist[j] == dist[j] ? dist[j] : INFINITY) : 0.0f);
                    use_wave &= wc[j].ok | !__any(gate[j]);
                }
            }
        }
#ifndef RT_ABLATE_SHADOW  // timing-only build: no shadow rays
        RT_MARK(cnt, 3);
        if (use_wave) shadow_opaque_wave<kLightBatch, (WAVE & 3) == 2>(S, lb, nl, tmask, P, L, dist, occ, wc, dmax, cnt);
        else shadow_opaque_batch<kLightBatch>(S, lb, nl, P, L, dist, occ, cnt);
#endif
        RT_MARK(cnt, 4);
#pragma unroll
        for (int j = 0; j < kLightBatch; ++j) {
            if (j < nl && gate[j]) {
                const float4 l0 = S.lights[2 * (lb + j)], l1 = S.lights[2 * (lb + j) + 1];
                Color F{0.0f, 0.0f, 0.0f};
                if (!occ[j]) {  // translucent surfaces, file order
                    F = Color{1.0f, 1.0f, 1.0f};
                    for (int q = 0; q < S.n_translucent; ++q) {
                        Color fc;
                        if (shadow_hit_record(S.geom + 4 * S.translucent[q], P, L[j], dist[j], fc, cnt)) F *= fc;
                    }
                }
                add_light(res, m, l0, l1, N, L[j], D, F);
            }
        }
        RT_MARK(cnt, 5);
    }
    return res;
}

// One pixel's colour.  MAXD = compile-time bounce-stack capacity (0 = no
// bounces: the reference as shipped).
// A pushed node: its colour so far, its surface, and which child runs:
// 0 reflected (no refraction to follow), 2 reflected (the refracted ray is
// waiting in Refr), 1 refracted.  5 dwords; the 8-dword Refr is written only
// by nodes that spawn both children.
struct Frame {
    Color acc;
    int surf, stage;
};
struct Refr {
    Vec3 P, D;
    float rior, energy;
};

template <int MAXD, int LB, int WAVE>
__device__ Color radiance(const SceneDev& S, const FrameDev& F, Vec3 O, Vec3 D, Counters& cnt, bool live, int tile)
{
    const Color bg{F.bg[0], F.bg[1], F.bg[2]};
    if constexpr (MAXD == 0) {
#ifdef RT_ABLATE_ALL  // timing-only build: ray set-up and store only
        return Color{D.x, D.y, D.z};
#endif
        float t;
        RT_MARK(cnt, 0);
        const int idx = closest_hit_primary<(WAVE & 11)>(S, O, D, t, cnt, tile);
        RT_MARK(cnt, 1);
        // Lanes that miss (or lie outside the frame) stay in step through the
        // shading so the wave stays whole for wave-level shadow culling.
        const bool hit = idx >= 0;
        if (!__any(hit & live)) return bg;
#ifdef RT_ABLATE_SHADE  // timing-only build: primary closest hit only
        return Color{t, (float)idx, 0.f};
#endif
        const int sidx = hit ? idx : 0;
        // A tile usually sees one surface: then its normal and material
        // records come by scalar (broadcast) loads instead of a per-lane gather.
        const int s0 = __builtin_amdgcn_readfirstlane(sidx);
        Vec3 N;
        Mat m;
        if (__all(sidx == s0)) {
            N = hit_normal(S, s0, O, D, t);
            m = load_mat(S, s0);
        } else {
            N = hit_normal(S, sidx, O, D, t);
            m = load_mat(S, sidx);
        }
        const Vec3 P = O + t * D;
        const Color c = shade_local<LB, WAVE>(S, m, P, N, D, cnt, hit & live);
        return hit ? c : bg;
    } else {
        Frame stk[MAXD];
        Refr rf[MAXD];
        int sp = 0;
        float rior = 1.0f, energy = 1.0f;
        Color ret{0.f, 0.f, 0.f};
        bool trace = true, camera_ray = true;
        for (;;) {
            if (trace) {
                float t;
                const int idx = camera_ray ? closest_hit_primary<(WAVE & 11)>(S, O, D, t, cnt, tile)
                                           : closest_hit<false>(S, O, D, t, cnt);
                camera_ray = false;
                ret = bg;
                if (idx >= 0) {
                    const Vec3 N = hit_normal(S, idx, O, D, t);
                    const Mat m = load_mat(S, idx);
                    const Vec3 P = O + t * D;
                    const Color acc = shade_local<LB, WAVE>(S, m, P, N, D, cnt);
                    // Scene.cpp:1779-1781 / :1790-1792 gates; bounces == sp
                    const float er = m.kr * energy;
                    const float et = m.kt * energy;
                    const bool can = sp < F.max_bounces && sp < MAXD;
                    const bool doR = er > F.min_energy && can;
                    const bool doT = et > F.min_energy && can;
                    if (doR || doT) {
                        Frame& fr = stk[sp];
                        fr.acc = acc;
                        fr.surf = idx;
                        ++cnt.bounce;
                        // The refracted ray (Scene.cpp:1793-1822), from this
                        // node's incoming ray — the same values whether it
                        // is traced now or after the reflected subtree.
                        Vec3 Dt = D;
                        float rior_t = rior;
                        if (doT) {
                            Vec3 n = N;
                            float ratio;
                            if (rior == m.ior) {  // Scene.cpp:1797-1803 inside -> out
                                rior_t = F.scene_ior;
                                ratio = m.ior / F.scene_ior;
                                n = -n;
                            } else {
                                rior_t = m.ior;
                                ratio = F.scene_ior / m.ior;
                            }
                            Dt = refract(D, n, ratio);
                        }
                        O = P;
                        if (doR) {  // Scene.cpp:1782-1788: IOR left at CRayon's default 0
                            fr.stage = doT ? 2 : 0;
                            if (doT) rf[sp] = Refr{P, Dt, rior_t, et};
                            D = reflect(D, N);
                            rior = 0.0f;
                            energy = er;
                        } else {
                            fr.stage = 1;
                            D = Dt;
                            rior = rior_t;
                            energy = et;
                        }
                        ++sp;
                        continue;
                    }
                    ret = acc;
                }
                trace = false;
            }
            if (sp == 0) return ret;
            Frame& fr = stk[sp - 1];
            const Mat m = load_mat(S, fr.surf);
            if (fr.stage != 1) {
                fr.acc += ret * m.kr;  // Scene.cpp:1787
                if (fr.stage == 2) {   // the refracted child (Scene.cpp:1790)
                    fr.stage = 1;
                    ++cnt.bounce;
                    const Refr r = rf[sp - 1];
                    O = r.P;
                    D = r.D;
                    rior = r.rior;
                    energy = r.energy;
                    trace = true;
                    continue;
                }
                ret = fr.acc;
                --sp;
            } else {
                fr.acc += ret * m.kt;  // Scene.cpp:1822
                ret = fr.acc;
                --sp;
            }
        }
    }
}

// Occupancy floor (waves per SIMD) for the depth-0 kernels: 7 (<= 72
// VGPRs).  It costs 4 VGPR spills (scratch: ~7 MB of HBM writes per C2
// frame, far below any bandwidth limit) and wins C2 by 4% over the
// unconstrained 81 VGPRs / 5 waves; 6 and 8 waves are slower
// (tools/ab_variants.py, MI355X).
#ifndef RT_WAVES_PER_EU
#define RT_WAVES_PER_EU 7
#endif
// COUNT: also tally the exact tests executed (the RT_FLAG_STATS launch); in
// the timed kernels the tallies are dead and compile away.
template <int MAXD, int LB, int WAVE, bool COUNT>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(MAXD == 0 ? RT_WAVES_PER_EU : 1))) void rt_trace_kernel(const SceneDev S, const FrameDev F, unsigned* __restrict__ rgba,
                                                       float* __restrict__ rgbf, StatsDev* __restrict__ stats)
{
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    // XCD-aware block order: the dispatcher deals workgroups round-robin over
    // the 8 XCDs (each with its own L2), so workgroup w runs on XCD w % 8 as
    // that XCD's (w / 8)-th; give every XCD one contiguous run of blocks in
    // row-major order, so neighbouring tiles — which read the same cells,
    // tile lists and records — share an L2.  A bijection for any grid size.
    int bx = (int)blockIdx.x, by = (int)blockIdx.y;
#ifndef RT_NO_XCD_MAP
    {
        // chunks of K = 4 consecutive blocks dealt round-robin to the XCDs
        // (C2 -2.3%, C3 -1.2% in A/B; whole-region runs per XCD were 1.8x
        // slower on C3: the mesh rows then pile onto a few XCDs)
        const unsigned nb = gridDim.x * gridDim.y, w = blockIdx.y * gridDim.x + blockIdx.x;
        const unsigned K = RT_XCD_CHUNK, x = w % kXcds, i = w / kXcds;
        const unsigned lw = ((i / K) * kXcds + x) * K + i % K;
        if (lw < nb && (nb % (kXcds * K)) == 0) {
            bx = (int)(lw % gridDim.x);
            by = (int)(lw / gridDim.x);
        }
    }
#endif
    const int px = bx * 16 + (wave & 1) * 8 + (lane & 7);
    const int ly0 = by * 16 + (wave >> 1) * 8;  // the wave's first output row
    const int ly = ly0 + (lane >> 3);
    // frame row of output row r: the slab, or band (r / band_rows) of this
    // rank's cyclic set (a wave's 8 rows never straddle a band: 16 | band_rows)
    int py0 = F.row_begin + ly0, rend = F.row_end;
    if (F.band_rows > 0) {
        py0 = ((ly0 / F.band_rows) * F.band_count + F.band_index) * F.band_rows + ly0 % F.band_rows;
        rend = F.height;
    }
    if (py0 >= rend) return;  // the whole wave lies past the frame (wave-uniform)
    const int py = py0 + (lane >> 3);
    const bool valid = px < F.width && py < rend;

    Counters cnt;
#ifdef RT_PROF
    cnt.last = __builtin_amdgcn_s_memtime();
#endif
    Color c{0.f, 0.f, 0.f};
    // Without bounces every lane runs (lanes outside the frame on a clamped
    // pixel, result dropped) so edge waves stay whole for wave-level culling.
    if (MAXD == 0 || valid) {
        const int pxc = px < F.width ? px : F.width - 1;
        const int pyc = py < rend ? py : rend - 1;
        const Vec3 D = camera_dir(F, pxc, pyc);
        const Vec3 O = make3(F.cam[0], F.cam[1], F.cam[2]);
        cnt.primary = valid ? 1u : 0u;
        // camera-buffer tile: this wave's 8 rows must be one tile row of the
        // full frame (the buffer's lists hold for its lanes' clamped pixels)
        int tile = -1;
        if ((WAVE & 8) && S.cb_tiles_x > 0 && (py0 & 7) == 0) {
            tile = (py0 >> 3) * S.cb_tiles_x + bx * 2 + (wave & 1);
            if (S.cb_flag[tile]) tile = -1;
        }
        c = radiance<MAXD, LB, WAVE>(S, F, O, D, cnt, valid, tile);
        if (valid) {
            const size_t o = (size_t)ly * F.width + px;
            if (rgbf) {
                rgbf[3 * o] = c.r;
                rgbf[3 * o + 1] = c.g;
                rgbf[3 * o + 2] = c.b;
            }
            if (rgba) rgba[o] = unorm8(c.r) | (unorm8(c.g) << 8) | (unorm8(c.b) << 16) | 0xFF000000u;
        }
    }
#ifdef RT_PROF
    RT_MARK(cnt, 6);
    if ((threadIdx.x & 63) == 0) {
        unsigned long long tot = 0;
        for (int i = 0; i < 8; ++i) {
            atomicAdd(&rt_prof_acc[i], cnt.pt[i]);
            atomicAdd(&rt_prof_ev[i], (unsigned long long)cnt.ev[i]);
            tot += cnt.pt[i];
        }
        const int tile = (int)((blockIdx.y * 2 + (wave >> 1)) * (gridDim.x * 2) + blockIdx.x * 2 + (wave & 1));
        if (rt_prof_tiles && tile < rt_prof_ntiles) {
            unsigned* o = rt_prof_tiles + 16 * (size_t)tile;
            o[0] = (unsigned)tot;
            o[1] = (unsigned)(tot >> 32);
            for (int i = 0; i < 8; ++i) o[2 + i] = (unsigned)(cnt.pt[i] >> 8);
            const int evi[6] = {1, 2, 4, 5, 6, 7};  // cam member batches, cam exact, shadow member
            for (int i = 0; i < 6; ++i) o[10 + i] = cnt.ev[evi[i]];  // batches, exact, by dcap, by cone
        }
    }
#endif
    if (F.flags & RT_FLAG_STATS) {
        unsigned long long v[7] = {cnt.primary, cnt.bounce, cnt.shadow, cnt.skipped, cnt.tri, cnt.pla, cnt.qua};
        StatsDev* sl = stats + ((blockIdx.x + blockIdx.y * gridDim.x) % kStatSlots);
        unsigned long long* dst[7] = {&sl->primary, &sl->bounce, &sl->shadow, &sl->skipped,
                                      &sl->tri, &sl->pla, &sl->qua};
        const int nv = COUNT ? 7 : 4;
        if (wave_full()) {  // one atomic per counter per wave
#pragma unroll
            for (int i = 0; i < 7; ++i)
                if (i < nv) {
                    const unsigned long long w = wave_sum_u64(v[i]);
                    if ((threadIdx.x & 63) == 0) atomicAdd(dst[i], w);
                }
        } else {
#pragma unroll
            for (int i = 0; i < 7; ++i)
                if (i < nv) atomicAdd(dst[i], v[i]);
        }
    }
}

// Compiled bounce-stack capacities.  The host picks the smallest one that
// covers the bounce depth the scene can actually reach.
#define RT_STACK_DEPTHS(X) X(0) X(1) X(2) X(3) X(4) X(5) X(8) X(12) X(16) X(20) X(32)

// Self-test of the wave primitives the culling relies on (rt_debug_selftest):
// wave_min / wave_max / wave_sum_u64 against plain loops over the same lane
// values, and wave_cone's cos W as a lower bound of every live lane's cosine.
__global__ void rt_selftest_kernel(unsigned seed, unsigned* __restrict__ fails)
{
    const int lane = (int)(threadIdx.x & 63);
    __shared__ float vals[256];
    __shared__ unsigned long long uv[256];
    unsigned h = (seed * 0x9E3779B9u) ^ (blockIdx.x * 0x85EBCA6Bu) ^ (threadIdx.x * 0xC2B2AE35u);
    h ^= h >> 16;
    h *= 0x7FEB352Du;
    h ^= h >> 15;
    const float x = (float)(h & 0xFFFFFF) / 16777216.0f * 2.0f - 1.0f;
    const unsigned long long u = (unsigned long long)(h >> 8) * 977ull;
    vals[threadIdx.x] = x;
    uv[threadIdx.x] = u;
    __syncthreads();
    const float mn = wave_min(x), mx = wave_max(x);
    const unsigned long long su = wave_sum_u64(u);
    const int base = (int)(threadIdx.x & ~63u);
    float rmn = vals[base], rmx = vals[base];
    unsigned long long rsu = 0;
    for (int i = 0; i < 64; ++i) {
        rmn = fminf(rmn, vals[base + i]);
        rmx = fmaxf(rmx, vals[base + i]);
        rsu += uv[base + i];
    }
    // a random cone of directions: every live lane's cosine to the axis >= cos W
    const float th = 0.05f * (float)((h >> 4) & 255) / 255.0f;
    const float ph = 6.2831853f * (float)((h >> 12) & 1023) / 1024.0f;
    const Vec3 d = make3(sinf(th) * cosf(ph), sinf(th) * sinf(ph), cosf(th));
    const bool live = ((h >> 20) & 3) != 0;
    const WaveCone wc = wave_cone(d, live);
    bool bad = (mn != rmn) | (mx != rmx) | (su != rsu);
    if (wc.ok && live) bad |= dot(d, wc.w) < wc.cosW;
    if (bad) atomicAdd(fails, 1u);
    (void)lane;
}

}  // namespace rt

// ===================================================================== host
using namespace rt;

struct rt_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    float4* d_geom = nullptr;
    float4* d_mat = nullptr;
    float4* d_lights = nullptr;
    float4* d_tri = nullptr;
    float4* d_plane = nullptr;
    float4* d_quad = nullptr;
    int* d_translucent = nullptr;
    float4* d_tricam = nullptr;
    float4* d_trisph = nullptr;
    float4* d_cone_cam = nullptr;
    float4* d_cone_light = nullptr;
    float4* d_trinrm = nullptr;
    float4* d_tricoef = nullptr;
    float4* d_clu_cam = nullptr;
    float4* d_clu_light = nullptr;
    int n_clu = 0;
    float4* d_uni = nullptr;  // union records (small lists): camera, then one per light
    // camera buffer (rt_cb_build): per-tile lists for the camera of cb_key
    unsigned* d_cb_off = nullptr;
    unsigned* d_cb_flag = nullptr;
    int2* d_cb_ent = nullptr;
    size_t cb_cap = 0;          // entries allocated
    int cb_tiles_x = 0, cb_ntiles = 0;
    float cb_key[25] = {};      // cam_pos, orient, half_w, half_h, inv_w, inv_h, width, height (as float bits)
    bool cb_valid = false;
    double cb_build_ms = 0.0;
    size_t cb_entries = 0;
    // light buffer (shadow cells), rt_lb_build
    unsigned* d_lb_off = nullptr;
    float4* d_lb_ent = nullptr;
    float4* d_lb_dcap = nullptr;
    float4* d_lb_meta = nullptr;
    bool lb_ready = false;
    size_t lb_entries = 0;
    double lb_build_ms = 0.0;
    float cam_key[3] = {0.f, 0.f, 0.f};
    bool cam_valid = false;
    StatsDev* d_stats = nullptr;
    void* d_scratch = nullptr;  // staging for host outputs
    size_t scratch_bytes = 0;
    int n_surf = 0, n_lights = 0;
    int n_tri = 0, n_plane = 0, n_quad = 0;
    int n_tri_opaque = 0, n_plane_opaque = 0, n_quad_opaque = 0, n_translucent = 0;
    int shadow_split = 0;
    float k_max = 0.0f;         // max(Kr, Kt) over surfaces (NaN ignored)
    bool uploaded = false;
    rt_stats last{};
    std::string err;
};

#define RT_EXPORT extern "C" __attribute__((visibility("default")))

static int hip_fail(rt_ctx* c, hipError_t e, const char* what)
{
    c->err = std::string(what) + ": " + hipGetErrorString(e);
    return RT_E_HIP;
}
#define HIP_TRY(c, call)                                   \
    do {                                                   \
        hipError_t e_ = (call);                            \
        if (e_ != hipSuccess) return hip_fail(c, e_, #call); \
    } while (0)

RT_EXPORT const char* rt_last_error(rt_ctx* c) { return c ? c->err.c_str() : "null context"; }

RT_EXPORT int rt_create(int32_t dev, rt_ctx** out)
{
    if (!out) return RT_E_ARG;
    *out = nullptr;
    rt_ctx* c = new rt_ctx();
    c->device = dev;
    int ndev = 0;
    hipError_t e = hipGetDeviceCount(&ndev);
    if (e != hipSuccess || ndev <= 0 || dev < 0 || dev >= ndev) {
        *out = c;
        c->err = "no usable HIP device";
        return RT_E_HIP;
    }
    *out = c;
    HIP_TRY(c, hipSetDevice(dev));
    HIP_TRY(c, hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
    HIP_TRY(c, hipEventCreate(&c->ev0));
    HIP_TRY(c, hipEventCreate(&c->ev1));
    HIP_TRY(c, hipMalloc(&c->d_stats, kStatSlots * sizeof(StatsDev)));
    return RT_OK;
}

RT_EXPORT void rt_destroy(rt_ctx* c)
{
    if (!c) return;
    if (c->stream) {
        (void)hipSetDevice(c->device);
        (void)hipStreamSynchronize(c->stream);
    }
    hipFree(c->d_geom);
    hipFree(c->d_mat);
    hipFree(c->d_lights);
    hipFree(c->d_tri);
    hipFree(c->d_plane);
    hipFree(c->d_quad);
    hipFree(c->d_translucent);
    hipFree(c->d_tricam);
    hipFree(c->d_trisph);
    hipFree(c->d_cone_cam);
    hipFree(c->d_cone_light);
    hipFree(c->d_trinrm);
    hipFree(c->d_tricoef);
    hipFree(c->d_clu_cam);
    hipFree(c->d_clu_light);
    hipFree(c->d_lb_off);
    hipFree(c->d_lb_ent);
    hipFree(c->d_lb_dcap);
    hipFree(c->d_lb_meta);
    hipFree(c->d_uni);
    hipFree(c->d_cb_off);
    hipFree(c->d_cb_flag);
    hipFree(c->d_cb_ent);
    hipFree(c->d_stats);
    hipFree(c->d_scratch);
    if (c->ev0) hipEventDestroy(c->ev0);
    if (c->ev1) hipEventDestroy(c->ev1);
    if (c->stream) hipStreamDestroy(c->stream);
    delete c;
}

static bool nonneg_finite(float v) { return std::isfinite(v) && !std::signbit(v); }

// 256 camera records = 16 KB, the scalar data cache.
static constexpr int kTricamMaxTriangles = 256;
static constexpr int kEdgeMaxTriangles = 1024;
// two-level (clustered) culling above this many triangles
static constexpr int kClusterMinTriangles = 1024;

// Cluster order for the two-level culling: a top-down median split of the
// centroids on the longest axis of their bounds, at multiples of 64, so
// every run of 64 consecutive triangles is a compact leaf (a Morton order
// scatters clusters of meshes with a thin, noisy axis: C3 cluster cones
// 34 mrad median, 94 at the 90th percentile vs the members' 7.6).
static void kd_order(std::vector<size_t>& ord, const std::vector<double>& cen, size_t b, size_t e)
{
    while (e - b > 64) {
        double lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
        for (size_t i = b; i < e; ++i)
            for (int a = 0; a < 3; ++a) {
                lo[a] = std::min(lo[a], cen[3 * ord[i] + a]);
                hi[a] = std::max(hi[a], cen[3 * ord[i] + a]);
            }
        int ax = 0;
        for (int a = 1; a < 3; ++a)
            if (hi[a] - lo[a] > hi[ax] - lo[ax]) ax = a;
        const size_t n = e - b;
        const size_t mid = b + std::max<size_t>(64, ((n / 2 + 32) / 64) * 64);
        std::nth_element(ord.begin() + b, ord.begin() + mid, ord.begin() + e, [&](size_t x, size_t y) {
            return cen[3 * x + ax] < cen[3 * y + ax] || (cen[3 * x + ax] == cen[3 * y + ax] && x < y);
        });
        kd_order(ord, cen, b, mid);
        b = mid;
    }
}
// Reorder 12-float triangle records into clusters, the ranges [0, n_opaque)
// and [n_opaque, n) separately.
static void cluster_order(std::vector<float>& tri, int n_opaque)
{
    const size_t n = tri.size() / 12;
    std::vector<double> cen(3 * n);
    for (size_t k = 0; k < n; ++k)
        for (int a = 0; a < 3; ++a) {
            const double v = tri[12 * k + a] + (tri[12 * k + 3 + a] + (double)tri[12 * k + 6 + a]) / 3.0;
            cen[3 * k + a] = std::isfinite(v) ? v : 0.0;
        }
    std::vector<size_t> ord(n);
    for (size_t k = 0; k < n; ++k) ord[k] = k;
    kd_order(ord, cen, 0, (size_t)n_opaque);
    kd_order(ord, cen, (size_t)n_opaque, n);
    std::vector<float> out(tri.size());
    for (size_t k = 0; k < n; ++k) std::memcpy(&out[12 * k], &tri[12 * ord[k]], 12 * sizeof(float));
    tri.swap(out);
}

// RT_AMD_LIGHTBUF (diagnostic/A-B switch): 0 = never build or use the light
// buffer (wave-level shadow culling), 2 = only for lists above
// kClusterMinTriangles; unset/1 = every depth-0 scene with opaque
// triangles (same-box A/B since the exact dmin and the camera buffer: C1
// -8%, C2 -6%, C4 -6% against the wave path).  RT_AMD_LB_SCALE scales the
// cell count.
static int lb_mode()
{
    const char* v = getenv("RT_AMD_LIGHTBUF");
    if (!v || !*v) return 1;
    return atoi(v);
}

// Light buffer of every light (shadow_opaque_lb, lb_cone): resolution from
// the median angular radius of the light's triangle cones (cell half-width
// ~ that radius), nearest-first cell lists built on the device in two
// levels (supercells of 16 x 16 cells, then cells), offsets by host scans.
static int lb_build(rt_ctx* c, int ntr, int n_opaque, int nl, const std::vector<double>& dcov)
{
    const auto t0 = std::chrono::steady_clock::now();
    const char* sc = getenv("RT_AMD_LB_SCALE");
    // cells of ~1/4 the median cone radius: best of 0.5-6 on C3 and C5
    const double scale = sc && *sc ? atof(sc) : 4.0;
    struct Build {
        int R = 16;
        std::vector<int> dperm;
        std::vector<unsigned> soff, ccount;
        int* d_slists = nullptr;
        unsigned* d_soff = nullptr;
    };
    std::vector<Build> B((size_t)nl);
    std::vector<float4> h((size_t)ntr * 2);
    int* d_perm = nullptr;
    unsigned* d_cnt = nullptr;
    int rc = RT_OK;
    auto fail = [&](hipError_t e, const char* what) {
        if (rc == RT_OK) rc = hip_fail(c, e, what);
    };
#define LB_TRY(call)                              \
    do {                                          \
        hipError_t e_ = (call);                   \
        if (e_ != hipSuccess) { fail(e_, #call); goto done; } \
    } while (0)
    {
        size_t total = 0, off_words = 0, dcap_total = 0;
        LB_TRY(hipMalloc(&d_perm, std::max<size_t>(ntr, 1) * sizeof(int)));
        for (int j = 0; j < nl; ++j) {
            Build& b = B[j];
            const float4* cone = c->d_cone_light + kConeRec * (size_t)ntr * j;
            LB_TRY(hipMemcpy(h.data(), cone, h.size() * sizeof(float4), hipMemcpyDeviceToHost));
            std::vector<double> T;
            std::vector<int> perm;
            for (int k = 0; k < n_opaque; ++k) {
                const float4 c0 = h[2 * k], c1 = h[2 * k + 1];
                if (c0.w > 0.0f && c0.w <= 1.0f) T.push_back(std::acos((double)c0.w));
                if (c0.w > 0.0f && c1.x < (float)dcov[j]) perm.push_back(k);
                if (!(c1.z >= (float)dcov[j])) b.dperm.push_back(k);
            }
            if (!T.empty()) {
                std::nth_element(T.begin(), T.begin() + T.size() / 2, T.end());
                const double med = std::max(T[T.size() / 2], 1e-4);
                b.R = (int)std::lround(scale / (kLbGroup * med)) * kLbGroup;
                b.R = std::min(1024, std::max(kLbGroup, b.R));
            }
            std::sort(perm.begin(), perm.end(), [&](int x, int y) {
                return h[2 * x + 1].x < h[2 * y + 1].x || (h[2 * x + 1].x == h[2 * y + 1].x && x < y);
            });
            auto key = [&](int k) { const float z = h[2 * k + 1].z; return z == z ? z : -INFINITY; };
            std::sort(b.dperm.begin(), b.dperm.end(),
                      [&](int x, int y) { return key(x) < key(y) || (key(x) == key(y) && x < y); });
            const int G = b.R / kLbGroup;
            const unsigned nsup = 6u * G * G, ncell = 6u * b.R * b.R;
            if (!perm.empty()) LB_TRY(hipMemcpy(d_perm, perm.data(), perm.size() * sizeof(int), hipMemcpyHostToDevice));
            hipFree(d_cnt);
            d_cnt = nullptr;
            LB_TRY(hipMalloc(&d_cnt, std::max(nsup, ncell) * sizeof(unsigned)));
            hipLaunchKernelGGL(rt_lb_super, dim3(nsup), dim3(256), 0, 0, cone, ntr, d_perm, (int)perm.size(), b.R,
                               (float)dcov[j], nullptr, d_cnt, nullptr);
            LB_TRY(hipGetLastError());
            b.soff.assign(nsup + 1, 0u);
            LB_TRY(hipMemcpy(b.soff.data() + 1, d_cnt, nsup * sizeof(unsigned), hipMemcpyDeviceToHost));
            for (unsigned q = 0; q < nsup; ++q) b.soff[q + 1] += b.soff[q];
            LB_TRY(hipMalloc(&b.d_soff, (nsup + 1) * sizeof(unsigned)));
            LB_TRY(hipMemcpy(b.d_soff, b.soff.data(), (nsup + 1) * sizeof(unsigned), hipMemcpyHostToDevice));
            LB_TRY(hipMalloc(&b.d_slists, std::max(b.soff[nsup], 1u) * sizeof(int)));
            hipLaunchKernelGGL(rt_lb_super, dim3(nsup), dim3(256), 0, 0, cone, ntr, d_perm, (int)perm.size(), b.R,
                               (float)dcov[j], b.d_soff, nullptr, b.d_slists);
            LB_TRY(hipGetLastError());
            hipLaunchKernelGGL(rt_lb_cells, dim3(nsup), dim3(256), 0, 0, cone, ntr, c->d_tri, b.R, (float)dcov[j],
                               b.d_soff, b.d_slists, nullptr, d_cnt, nullptr);
            LB_TRY(hipGetLastError());
            b.ccount.resize(ncell);
            LB_TRY(hipMemcpy(b.ccount.data(), d_cnt, ncell * sizeof(unsigned), hipMemcpyDeviceToHost));
            for (unsigned q = 0; q < ncell; ++q) total += b.ccount[q];
            off_words += ncell + 1;
            dcap_total += b.dperm.size();
        }
        if (total >= 0xFFFFFFF0ull / 4) {  // entry indices are 32-bit
            c->err = "light buffer too large";
            goto done;
        }
        LB_TRY(hipMalloc(&c->d_lb_off, off_words * sizeof(unsigned)));
        LB_TRY(hipMalloc(&c->d_lb_ent, std::max<size_t>(total, 1) * kLbEnt * sizeof(float4)));
        LB_TRY(hipMalloc(&c->d_lb_dcap, std::max<size_t>(dcap_total, 1) * kLbEnt * sizeof(float4)));
        LB_TRY(hipMalloc(&c->d_lb_meta, std::max(nl, 1) * 2 * sizeof(float4)));
        std::vector<float4> meta((size_t)std::max(nl, 1) * 2);
        size_t obase = 0, ebase = 0, dbase = 0;
        for (int j = 0; j < nl; ++j) {
            Build& b = B[j];
            const float4* cone = c->d_cone_light + kConeRec * (size_t)ntr * j;
            const unsigned G = b.R / kLbGroup, nsup = 6u * G * G, ncell = 6u * b.R * b.R;
            std::vector<unsigned> off(ncell + 1);
            size_t run = ebase;
            for (unsigned q = 0; q < ncell; ++q) {
                off[q] = (unsigned)run;
                run += b.ccount[q];
            }
            off[ncell] = (unsigned)run;
            LB_TRY(hipMemcpy(c->d_lb_off + obase, off.data(), off.size() * sizeof(unsigned), hipMemcpyHostToDevice));
            hipLaunchKernelGGL(rt_lb_cells, dim3(nsup), dim3(256), 0, 0, cone, ntr, c->d_tri, b.R, (float)dcov[j],
                               b.d_soff, b.d_slists, c->d_lb_off + obase, nullptr, c->d_lb_ent);
            LB_TRY(hipGetLastError());
            if (!b.dperm.empty()) {
                LB_TRY(hipMemcpy(d_perm, b.dperm.data(), b.dperm.size() * sizeof(int), hipMemcpyHostToDevice));
                hipLaunchKernelGGL(rt_lb_dcap, dim3((unsigned)((b.dperm.size() + 255) / 256)), dim3(256), 0, 0, cone,
                                   c->d_tri, d_perm, (int)b.dperm.size(), c->d_lb_dcap + kLbEnt * dbase);
                LB_TRY(hipGetLastError());
                LB_TRY(hipDeviceSynchronize());  // d_perm is reused by the next light
            }
            unsigned ob = (unsigned)obase, db = (unsigned)dbase, nd = (unsigned)b.dperm.size();
            float4 m0, m1 = make_float4((float)dcov[j], 0.f, 0.f, 0.f);
            std::memcpy(&m0.x, &ob, 4);
            std::memcpy(&m0.y, &db, 4);
            std::memcpy(&m0.z, &nd, 4);
            std::memcpy(&m0.w, &b.R, 4);
            meta[2 * j] = m0;
            meta[2 * j + 1] = m1;
            obase += ncell + 1;
            ebase = run;
            dbase += b.dperm.size();
        }
        LB_TRY(hipMemcpy(c->d_lb_meta, meta.data(), meta.size() * sizeof(float4), hipMemcpyHostToDevice));
        LB_TRY(hipDeviceSynchronize());
        c->lb_ready = true;
        c->lb_entries = total;
    }
done:
#undef LB_TRY
    for (Build& b : B) {
        hipFree(b.d_slists);
        hipFree(b.d_soff);
    }
    hipFree(d_perm);
    hipFree(d_cnt);
    c->lb_build_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    if (rc == RT_OK && !c->lb_ready) {  // too large: run without it
        hipFree(c->d_lb_off);
        hipFree(c->d_lb_ent);
        hipFree(c->d_lb_dcap);
        hipFree(c->d_lb_meta);
        c->d_lb_off = nullptr;
        c->d_lb_ent = c->d_lb_dcap = c->d_lb_meta = nullptr;
        c->err.clear();
    }
    return rc;
}

RT_EXPORT int rt_upload_scene(rt_ctx* c, const rt_scene_flat* s)
{
    if (!c || !s || s->n_surfaces < 0 || s->n_lights < 0) return RT_E_ARG;
    if (s->n_surfaces > 0 && (!s->type || !s->geom || !s->material)) return RT_E_ARG;
    if (s->n_lights > 0 && !s->lights) return RT_E_ARG;
    if (!c->stream) return RT_E_STATE;
    HIP_TRY(c, hipSetDevice(c->device));
    const int n = s->n_surfaces, nl = s->n_lights;
    std::vector<float> geom((size_t)std::max(n, 1) * 16, 0.0f), mat((size_t)std::max(n, 1) * 12, 0.0f),
        lig((size_t)std::max(nl, 1) * 8, 0.0f);
    bool opaque = true;
    float kmax = 0.0f;
    for (int i = 0; i < n; ++i) {
        const float* g = s->geom + 12 * (size_t)i;
        const float* m = s->material + 10 * (size_t)i;
        float* o = &geom[16 * (size_t)i];
        int kind = s->type[i];
        if (kind < RT_TRIANGLE || kind > RT_QUADRIC) {
            c->err = "unknown surface type";
            return RT_E_ARG;
        }
        std::memcpy(&o[0], &kind, sizeof(int));
        if (kind == RT_TRIANGLE) {
            const Vec3 p0 = make3(g[0], g[1], g[2]), p1 = make3(g[3], g[4], g[5]), p2 = make3(g[6], g[7], g[8]);
            const Vec3 e1 = p1 - p0, e2 = p2 - p0;  // Triangle.cpp:135-136
            o[1] = p0.x; o[2] = p0.y; o[3] = p0.z;
            o[4] = e1.x; o[5] = e1.y; o[6] = e1.z;
            o[7] = e2.x; o[8] = e2.y; o[9] = e2.z;
            o[10] = g[9]; o[11] = g[10]; o[12] = g[11];
        } else if (kind == RT_PLANE) {
            o[1] = g[0]; o[2] = g[1]; o[3] = g[2]; o[4] = g[3];
        } else {
            o[1] = g[0]; o[2] = g[1]; o[3] = g[2];  // quad
            o[4] = g[6]; o[5] = g[7]; o[6] = g[8];  // mix
            o[7] = g[3]; o[8] = g[4]; o[9] = g[5];  // lin
            o[10] = g[9];
        }
        const Color fc = Color{m[0], m[1], m[2]} * m[8];  // colour * Kt
        o[13] = fc.r; o[14] = fc.g; o[15] = fc.b;
        opaque = opaque && nonneg_finite(fc.r) && nonneg_finite(fc.g) && nonneg_finite(fc.b);
        float* q = &mat[12 * (size_t)i];
        for (int k = 0; k < 10; ++k) q[k] = m[k];
        if (m[7] > kmax) kmax = m[7];
        if (m[8] > kmax) kmax = m[8];
    }
    // Per-kind arrays, opaque surfaces first (file order kept inside each class).
    auto opaque_at = [&](int i) {
        const float* o = &geom[16 * (size_t)i];
        return o[13] == 0.0f && o[14] == 0.0f && o[15] == 0.0f;
    };
    std::vector<float> tri, pla, qua;
    std::vector<int> translucent;
    int n_tri_o = 0, n_pla_o = 0, n_qua_o = 0;
    for (int pass = 0; pass < 2; ++pass) {
        for (int i = 0; i < n; ++i) {
            if (opaque_at(i) != (pass == 0)) continue;
            const float* o = &geom[16 * (size_t)i];
            float idx;
            std::memcpy(&idx, &i, sizeof(int));
            const int kind = s->type[i];
            if (kind == RT_TRIANGLE) {
                const float r[12] = {o[1], o[2], o[3], o[4], o[5], o[6], o[7], o[8], o[9], idx, 0.f, 0.f};
                tri.insert(tri.end(), r, r + 12);
                n_tri_o += pass == 0;
            } else if (kind == RT_PLANE) {
                const float r[8] = {o[1], o[2], o[3], o[4], idx, 0.f, 0.f, 0.f};
                pla.insert(pla.end(), r, r + 8);
                n_pla_o += pass == 0;
            } else {
                const float r[12] = {o[1], o[2], o[3], o[4], o[5], o[6], o[7], o[8], o[9], o[10], idx, 0.f};
                qua.insert(qua.end(), r, r + 12);
                n_qua_o += pass == 0;
            }
        }
    }
    for (int i = 0; i < n; ++i)
        if (!opaque_at(i)) translucent.push_back(i);
    // Big lists: cluster order (kd_order) inside the opaque and the
    // translucent ranges, so 64 consecutive triangles form a compact cluster
    // for the two-level culling.  The order is free: closest hit is the
    // lexicographic (t, file index) minimum and opaque shadow tests are any-hit.
    if (tri.size() / 12 > (size_t)kClusterMinTriangles) cluster_order(tri, n_tri_o);
    const int cnt_tri = (int)(tri.size() / 12), cnt_pla = (int)(pla.size() / 8), cnt_qua = (int)(qua.size() / 12);
    const int cnt_translucent = (int)translucent.size();
    tri.resize(std::max<size_t>(tri.size(), 12));
    pla.resize(std::max<size_t>(pla.size(), 8));
    qua.resize(std::max<size_t>(qua.size(), 12));
    translucent.resize(std::max<size_t>(translucent.size(), 1));
    for (int j = 0; j < nl; ++j) {
        const float* l = s->lights + 7 * (size_t)j;
        float* o = &lig[8 * (size_t)j];
        o[0] = l[0]; o[1] = l[1]; o[2] = l[2]; o[3] = l[6];
        o[4] = l[3]; o[5] = l[4]; o[6] = l[5]; o[7] = 0.0f;
    }
    hipFree(c->d_geom);
    hipFree(c->d_mat);
    hipFree(c->d_lights);
    hipFree(c->d_tri);
    hipFree(c->d_plane);
    hipFree(c->d_quad);
    hipFree(c->d_translucent);
    hipFree(c->d_tricam);
    hipFree(c->d_trisph);
    hipFree(c->d_cone_cam);
    hipFree(c->d_cone_light);
    hipFree(c->d_trinrm);
    hipFree(c->d_tricoef);
    hipFree(c->d_clu_cam);
    hipFree(c->d_clu_light);
    c->d_tricam = c->d_trisph = c->d_cone_cam = c->d_cone_light = c->d_trinrm = c->d_tricoef = nullptr;
    c->d_clu_cam = c->d_clu_light = nullptr;
    c->n_clu = 0;
    hipFree(c->d_lb_off);
    hipFree(c->d_lb_ent);
    hipFree(c->d_lb_dcap);
    hipFree(c->d_lb_meta);
    c->d_lb_off = nullptr;
    c->d_lb_ent = c->d_lb_dcap = c->d_lb_meta = nullptr;
    c->lb_ready = false;
    c->lb_entries = 0;
    hipFree(c->d_uni);
    c->d_uni = nullptr;
    c->cb_valid = false;  // buffers are kept (reallocated on demand)
    c->cam_valid = false;
    c->d_geom = c->d_mat = c->d_lights = c->d_tri = c->d_plane = c->d_quad = nullptr;
    c->d_translucent = nullptr;
    c->uploaded = false;
    auto up = [&](void** dst, const void* src, size_t bytes) -> hipError_t {
        hipError_t e = hipMalloc(dst, bytes);
        if (e != hipSuccess) return e;
        return hipMemcpy(*dst, src, bytes, hipMemcpyHostToDevice);
    };
    HIP_TRY(c, up((void**)&c->d_tri, tri.data(), tri.size() * sizeof(float)));
    HIP_TRY(c, up((void**)&c->d_plane, pla.data(), pla.size() * sizeof(float)));
    HIP_TRY(c, up((void**)&c->d_quad, qua.data(), qua.size() * sizeof(float)));
    HIP_TRY(c, up((void**)&c->d_translucent, translucent.data(), translucent.size() * sizeof(int)));
    HIP_TRY(c, hipMalloc((void**)&c->d_tricam, (tri.size() / 12) * 16 * sizeof(float)));
    // Per triangle (tri[] order), for rt_cone_prepass: the bounding sphere of
    // the triangle the reference tests (p0, p0 + e1, p0 + e2 with the float
    // edges; radius measured from the float-rounded centre), the unit normal
    // and longest edge, and the rounding-bound coefficients gS, gL, rho_cap.
    // rho_cap = -1: det can be too inexact at the reference's 0.01 gate
    // (longest edge >~ 110) — never culled.
    const size_t ntr = tri.size() / 12;
    std::vector<float> sph(ntr * 4), nrm(ntr * 4), coef(ntr * 4);
    const double eps = 0x1p-24;
    for (size_t k = 0; k < ntr; ++k) {
        const float* r = &tri[12 * k];
        double p[3][3];
        for (int a = 0; a < 3; ++a) {
            p[0][a] = r[a];
            p[1][a] = (double)r[a] + (double)r[3 + a];
            p[2][a] = (double)r[a] + (double)r[6 + a];
        }
        float ctr[3];
        for (int a = 0; a < 3; ++a) ctr[a] = (float)((p[0][a] + p[1][a] + p[2][a]) / 3.0);
        double rad = 0, L2 = 0;
        for (int q = 0; q < 3; ++q) {
            double d2 = 0;
            for (int a = 0; a < 3; ++a) d2 += (p[q][a] - ctr[a]) * (p[q][a] - ctr[a]);
            rad = std::max(rad, std::sqrt(d2));
            for (int w = q + 1; w < 3; ++w) {
                double l2 = 0;
                for (int a = 0; a < 3; ++a) l2 += (p[q][a] - p[w][a]) * (p[q][a] - p[w][a]);
                L2 = std::max(L2, l2);
            }
        }
        rad = rad * (1.0 + 1e-9);
        for (int a = 0; a < 3; ++a) sph[4 * k + a] = ctr[a];
        sph[4 * k + 3] = std::nextafter((float)rad, INFINITY);
        const double e1[3] = {r[3], r[4], r[5]}, e2[3] = {r[6], r[7], r[8]};
        const double nx = e1[1] * e2[2] - e1[2] * e2[1], ny = e1[2] * e2[0] - e1[0] * e2[2],
                     nz = e1[0] * e2[1] - e1[1] * e2[0];
        const double nn = std::sqrt(nx * nx + ny * ny + nz * nz);
        const double L = std::sqrt(L2) * (1.0 + 1e-9);
        const double dl = 7.0 * eps * L * L;
        const double rho_cap = dl < 0.01 ? dl / (0.01 - dl) + 3.0 * eps : INFINITY;
        const bool fine = nn > 0 && std::isfinite(nn) && rho_cap <= 0.5;
        const double kk = fine ? 1.0 / (1.0 - rho_cap) : 2.0;
        nrm[4 * k] = fine ? (float)(nx / nn) : 0.f;
        nrm[4 * k + 1] = fine ? (float)(ny / nn) : 0.f;
        nrm[4 * k + 2] = fine ? (float)(nz / nn) : 0.f;
        nrm[4 * k + 3] = std::nextafter((float)L, INFINITY);
        coef[4 * k] = fine ? (float)(54.0 * kk * eps * L * L / nn * 1.01) : 0.f;
        coef[4 * k + 1] = fine ? (float)(21.0 * kk * eps * L * L * L / nn * 1.01) : 0.f;
        coef[4 * k + 2] = fine ? (float)(rho_cap * 1.01) : -1.0f;
        coef[4 * k + 3] = fine ? (float)nn : 0.0f;  // |N| = |e1 x e2| (never-hit bound)
    }
    sph.resize(std::max<size_t>(sph.size(), 4));
    nrm.resize(std::max<size_t>(nrm.size(), 4));
    coef.resize(std::max<size_t>(coef.size(), 4));
    HIP_TRY(c, up((void**)&c->d_trisph, sph.data(), sph.size() * sizeof(float)));
    HIP_TRY(c, up((void**)&c->d_trinrm, nrm.data(), nrm.size() * sizeof(float)));
    HIP_TRY(c, up((void**)&c->d_tricoef, coef.data(), coef.size() * sizeof(float)));
    HIP_TRY(c, hipMalloc((void**)&c->d_cone_cam, std::max<size_t>(ntr, 1) * kConeRec * sizeof(float4)));
    HIP_TRY(c, hipMalloc((void**)&c->d_cone_light, std::max<size_t>(ntr * nl, 1) * kConeRec * sizeof(float4)));
    std::vector<double> lb_dcov((size_t)std::max(nl, 0), 0.0);
    for (int j = 0; j < nl && ntr > 0; ++j) {
        const float* l = s->lights + 7 * (size_t)j;
        // shadow rays are culled up to 4x the light's farthest triangle
        double far = 0;
        for (size_t k = 0; k < ntr; ++k) {
            double d2 = 0;
            for (int a = 0; a < 3; ++a) d2 += ((double)sph[4 * k + a] - l[a]) * ((double)sph[4 * k + a] - l[a]);
            far = std::max(far, std::sqrt(d2) + sph[4 * k + 3]);
        }
        hipLaunchKernelGGL(rt_cone_prepass, dim3((unsigned)((ntr + 255) / 256)), dim3(256), 0, 0, c->d_tri, c->d_trisph,
                           c->d_trinrm, c->d_tricoef, (int)ntr, l[0], l[1], l[2], 0, (float)(4.0 * far),
                           c->d_cone_light + kConeRec * ntr * j);
        HIP_TRY(c, hipGetLastError());
        lb_dcov[j] = (double)(float)(4.0 * far);
    }
    if (ntr > (size_t)kClusterMinTriangles) {
        c->n_clu = (int)((ntr + 63) / 64);
        HIP_TRY(c, hipMalloc((void**)&c->d_clu_cam, (size_t)c->n_clu * 4 * sizeof(float4)));
        HIP_TRY(c, hipMalloc((void**)&c->d_clu_light, std::max<size_t>((size_t)c->n_clu * nl, 1) * 2 * sizeof(float4)));
        for (int j = 0; j < nl; ++j) {
            hipLaunchKernelGGL(rt_cluster_prepass, dim3((unsigned)((c->n_clu + 63) / 64)), dim3(64), 0, 0,
                               c->d_cone_light + kConeRec * ntr * j, (int)ntr, c->n_clu,
                               c->d_clu_light + 2 * (size_t)c->n_clu * j);
            HIP_TRY(c, hipGetLastError());
        }
    }
    if (ntr > 0 && ntr <= (size_t)kClusterMinTriangles) {
        // union records: [camera (filled when the camera is set)] [light 0] ...
        HIP_TRY(c, hipMalloc((void**)&c->d_uni, (size_t)(nl + 1) * 2 * sizeof(float4)));
        for (int j = 0; j < nl && n_tri_o > 0; ++j) {
            hipLaunchKernelGGL(rt_cluster_prepass, dim3(1), dim3(64), 0, 0, c->d_cone_light + kConeRec * ntr * j,
                               n_tri_o, 1, c->d_uni + 2 * (1 + (size_t)j), n_tri_o);
            HIP_TRY(c, hipGetLastError());
        }
        if (n_tri_o == 0) {  // no opaque triangle: nothing for shadow rays to walk ("never" record)
            std::vector<float4> nev((size_t)nl * 2);
            for (int j = 0; j < nl; ++j) {
                nev[2 * j] = make_float4(0.f, 0.f, 0.f, 2.0f);
                nev[2 * j + 1] = make_float4(INFINITY, 0.f, INFINITY, 0.f);
            }
            if (nl) HIP_TRY(c, hipMemcpy(c->d_uni + 2, nev.data(), nev.size() * sizeof(float4), hipMemcpyHostToDevice));
        }
    }
    HIP_TRY(c, hipDeviceSynchronize());
    const int lbm = lb_mode();  // built only where launch() will use it
    if (ntr > 0 && nl > 0 && n_tri_o > 0 && opaque && (lbm == 1 || (lbm == 2 && ntr > (size_t)kClusterMinTriangles))) {
        const int rc = lb_build(c, (int)ntr, n_tri_o, nl, lb_dcov);
        if (rc) return rc;
    }
    HIP_TRY(c, hipMalloc(&c->d_geom, geom.size() * sizeof(float)));
    HIP_TRY(c, hipMalloc(&c->d_mat, mat.size() * sizeof(float)));
    HIP_TRY(c, hipMalloc(&c->d_lights, lig.size() * sizeof(float)));
    HIP_TRY(c, hipMemcpy(c->d_geom, geom.data(), geom.size() * sizeof(float), hipMemcpyHostToDevice));
    HIP_TRY(c, hipMemcpy(c->d_mat, mat.data(), mat.size() * sizeof(float), hipMemcpyHostToDevice));
    HIP_TRY(c, hipMemcpy(c->d_lights, lig.data(), lig.size() * sizeof(float), hipMemcpyHostToDevice));
    c->n_surf = n;
    c->n_lights = nl;
    c->n_tri = cnt_tri;
    c->n_plane = cnt_pla;
    c->n_quad = cnt_qua;
    c->n_tri_opaque = n_tri_o;
    c->n_plane_opaque = n_pla_o;
    c->n_quad_opaque = n_qua_o;
    c->n_translucent = cnt_translucent;
    c->shadow_split = opaque ? 1 : 0;
    c->k_max = kmax;
    c->uploaded = true;
    return RT_OK;
}

// Deepest bounce level any pixel can reach: a child exists only while
// K * energy > min_energy (Scene.cpp:1780,1791); energies are products of
// factors <= k_max and float rounding is monotone, so iterating with k_max
// bounds every path.
static int reachable_depth(const rt_ctx* c, const rt_frame* f)
{
    // With a negative threshold the energy argument below does not hold.
    if (!(f->min_energy >= 0.0f)) return f->max_bounces;
    int levels = 0;
    float e = 1.0f;
    while (levels < f->max_bounces) {
        const float child = c->k_max * e;
        if (!(child > f->min_energy)) break;
        e = child;
        ++levels;
        if (levels > 4096) break;
    }
    return levels;
}

typedef void (*kernel_fn)(const SceneDev, const FrameDev, unsigned*, float*, StatsDev*);

// Kernel variants (tools/ab_variants.py, MI355X).  Without bounces and with
// triangles: wave-level culling (two-level above kClusterMinTriangles),
// RT_WAVE_LB lights per shadow pass (1: with the camera buffer and the union
// pre-test, C2 -5.3% and C4 -6.9% against 2; 3 is 50% slower).  Without
// triangles nothing is culled: light batches of 3.  Bounce kernels:
// per-lane culling, one light per pass (LB 3 regressed scene7 by 4%).
#ifndef RT_WAVE_LB
#define RT_WAVE_LB 1
#endif
template <bool COUNT>
static kernel_fn pick_kernel(int depth, int n_tri, int n_lights, bool lbuf, bool cbuf, int& cap, int& lb)
{
    lb = 1;
    if (depth == 0 && n_tri > 0 && lbuf) {  // light-buffer shadows, one light per pass
        cap = 0;
        if (n_tri > kClusterMinTriangles)
            return cbuf ? (kernel_fn)&rt_trace_kernel<0, 1, 14, COUNT> : (kernel_fn)&rt_trace_kernel<0, 1, 6, COUNT>;
        return cbuf ? (kernel_fn)&rt_trace_kernel<0, 1, 13, COUNT> : (kernel_fn)&rt_trace_kernel<0, 1, 5, COUNT>;
    }
    if (depth == 0 && n_tri > kClusterMinTriangles) {
        cap = 0;
        lb = RT_WAVE_LB;
        return cbuf ? (kernel_fn)&rt_trace_kernel<0, RT_WAVE_LB, 10, COUNT>
                    : (kernel_fn)&rt_trace_kernel<0, RT_WAVE_LB, 2, COUNT>;
    }
    if (depth == 0 && n_tri > 0) {
        cap = 0;
        lb = RT_WAVE_LB;
        return cbuf ? (kernel_fn)&rt_trace_kernel<0, RT_WAVE_LB, 9, COUNT>
                    : (kernel_fn)&rt_trace_kernel<0, RT_WAVE_LB, 1, COUNT>;
    }
    if (depth == 0 && n_lights > 1) {
        cap = 0;
        lb = 3;
        return (kernel_fn)&rt_trace_kernel<0, 3, 0, COUNT>;
    }
#define RT_PICK(N)                                                        \
    if (depth <= N) {                                                     \
        cap = N;                                                          \
        return (kernel_fn)&rt_trace_kernel<N, 1, 0, COUNT>;        \
    }
    RT_STACK_DEPTHS(RT_PICK)
#undef RT_PICK
    cap = -1;
    return nullptr;
}

// Output rows of a launch: the slab, or this rank's band set.
static int frame_rows(const rt_frame* f)
{
    if (f->band_rows != 0) return std::max(0, (int)rt_band_rows(f->height, f->band_rows, f->band_count, f->band_index));
    return f->row_end - f->row_begin;
}

// RT_AMD_CAMBUF (A/B switch): 0 = no camera buffer; unset/1 = for depth-0
// scenes with triangles.
static bool cb_mode()
{
    const char* v = getenv("RT_AMD_CAMBUF");
    return !(v && *v == '0');
}

static void cb_key_of(const rt_frame* f, float* key)
{
    std::memcpy(key, f->cam_pos, 3 * sizeof(float));
    std::memcpy(key + 3, f->orient, 16 * sizeof(float));
    key[19] = f->half_w;
    key[20] = f->half_h;
    key[21] = f->inv_w;
    key[22] = f->inv_h;
    std::memcpy(key + 23, &f->width, sizeof(int));
    std::memcpy(key + 24, &f->height, sizeof(int));
}

static void frame_dev(const rt_frame* f, FrameDev& F)
{
    std::memcpy(F.cam, f->cam_pos, sizeof F.cam);
    std::memcpy(F.orient, f->orient, sizeof F.orient);
    F.half_w = f->half_w;
    F.half_h = f->half_h;
    F.inv_w = f->inv_w;
    F.inv_h = f->inv_h;
    std::memcpy(F.bg, f->background, sizeof F.bg);
    F.width = f->width;
    F.height = f->height;
    F.row_begin = f->row_begin;
    F.row_end = f->row_end;
    F.max_bounces = f->max_bounces;
    F.min_energy = f->min_energy;
    F.scene_ior = f->scene_ior;
    F.flags = f->flags;
    F.band_rows = f->band_rows;
    F.band_count = f->band_count;
    F.band_index = f->band_index;
}

// Per-camera prepasses (when the camera position moved): camera-ray
// triangle values, camera cone records, union / cluster records.
static int camera_prepass(rt_ctx* c, const rt_frame* f, hipStream_t st, bool all_tricam)
{
    if (c->n_tri <= 0 || (c->cam_valid && std::memcmp(c->cam_key, f->cam_pos, sizeof c->cam_key) == 0)) return RT_OK;
    const float* cp = f->cam_pos;
    if (all_tricam || c->n_tri <= kTricamMaxTriangles) {
        hipLaunchKernelGGL(rt_camera_prepass, dim3((c->n_tri + 255) / 256), dim3(256), 0, st, c->d_tri, c->n_tri,
                           cp[0], cp[1], cp[2], c->d_tricam);
        HIP_TRY(c, hipGetLastError());
    }
    hipLaunchKernelGGL(rt_cone_prepass, dim3((c->n_tri + 255) / 256), dim3(256), 0, st, c->d_tri, c->d_trisph,
                       c->d_trinrm, c->d_tricoef, c->n_tri, cp[0], cp[1], cp[2], 1, 0.0f, c->d_cone_cam);
    HIP_TRY(c, hipGetLastError());
    if (c->d_uni) {
        hipLaunchKernelGGL(rt_cluster_prepass, dim3(1), dim3(64), 0, st, c->d_cone_cam, c->n_tri, 1, c->d_uni,
                           c->n_tri);
        HIP_TRY(c, hipGetLastError());
    }
    if (c->n_clu > 0) {
        float4* tmp = c->d_clu_cam + 2 * (size_t)c->n_clu;  // second half: unsorted
        hipLaunchKernelGGL(rt_cluster_prepass, dim3((unsigned)((c->n_clu + 63) / 64)), dim3(64), 0, st,
                           c->d_cone_cam, c->n_tri, c->n_clu, tmp);
        HIP_TRY(c, hipGetLastError());
        hipLaunchKernelGGL(rt_cluster_sort, dim3((unsigned)((c->n_clu + 255) / 256)), dim3(256), 0, st, tmp,
                           c->n_clu, c->d_clu_cam);
        HIP_TRY(c, hipGetLastError());
    }
    std::memcpy(c->cam_key, f->cam_pos, sizeof c->cam_key);
    c->cam_valid = true;
    c->cb_valid = false;
    return RT_OK;
}

static SceneDev scene_dev(rt_ctx* c, bool lbuf, bool cbuf)
{
    const int use_tricam = c->n_tri > 0 && c->n_tri <= kTricamMaxTriangles;
    return SceneDev{c->d_geom, c->d_mat, c->d_lights, c->d_tri, c->d_plane, c->d_quad, c->d_translucent, c->d_tricam,
                    use_tricam, c->n_tri <= kEdgeMaxTriangles, c->d_cone_cam, c->d_cone_light, c->d_clu_cam,
                    c->d_clu_light, c->n_clu, c->n_surf, c->n_lights, c->n_tri, c->n_plane, c->n_quad,
                    c->n_tri_opaque, c->n_plane_opaque, c->n_quad_opaque, c->n_translucent, c->shadow_split,
                    lbuf ? 1 : 0, c->d_lb_off, c->d_lb_ent, c->d_lb_dcap, c->d_lb_meta,
                    (c->d_uni && !getenv("RT_AMD_NO_UNION")) ? c->d_uni : nullptr,
                    c->d_cb_off, c->d_cb_ent, c->d_cb_flag, cbuf ? c->cb_tiles_x : 0};
}

// Camera buffer for the frame's camera (synchronous: the list sizes come
// back to the host for the offsets).  Needs the camera prepass done.
static int cb_build(rt_ctx* c, const rt_frame* f, hipStream_t st)
{
    const auto t0 = std::chrono::steady_clock::now();
    const int tx = (f->width + 7) / 8, ty = (f->height + 7) / 8, nt = tx * ty;
    if (nt > c->cb_ntiles || !c->d_cb_off) {
        hipFree(c->d_cb_off);
        hipFree(c->d_cb_flag);
        c->d_cb_off = nullptr;
        c->d_cb_flag = nullptr;
        HIP_TRY(c, hipMalloc(&c->d_cb_off, (size_t)(nt + 1) * sizeof(unsigned)));
        HIP_TRY(c, hipMalloc(&c->d_cb_flag, (size_t)std::max(nt, 1) * sizeof(unsigned)));
        c->cb_ntiles = nt;
    }
    c->cb_tiles_x = tx;
    SceneDev S = scene_dev(c, false, true);
    FrameDev F;
    frame_dev(f, F);
    dim3 grid((tx + 1) / 2, (ty + 1) / 2);
    unsigned* cnt = c->d_cb_off + 1;  // counts land one slot up, scanned in place on the host
    hipLaunchKernelGGL(rt_cb_build<false>, grid, dim3(256), 0, st, S, F, (const unsigned*)nullptr, cnt, c->d_cb_flag,
                       (int2*)nullptr);
    HIP_TRY(c, hipGetLastError());
    std::vector<unsigned> off((size_t)nt + 1, 0u);
    HIP_TRY(c, hipMemcpyAsync(off.data() + 1, cnt, (size_t)nt * sizeof(unsigned), hipMemcpyDeviceToHost, st));
    HIP_TRY(c, hipStreamSynchronize(st));
    size_t run = 0;
    for (int t = 0; t < nt; ++t) {
        run += off[t + 1];
        if (run > 0xFFFFFFF0ull) {
            c->err = "camera buffer too large";
            return RT_E_UNSUPPORTED;
        }
        off[t + 1] = (unsigned)run;
    }
    if (run > c->cb_cap || !c->d_cb_ent) {
        hipFree(c->d_cb_ent);
        c->d_cb_ent = nullptr;
        HIP_TRY(c, hipMalloc(&c->d_cb_ent, std::max<size_t>(run, 1) * sizeof(int2)));
        c->cb_cap = std::max<size_t>(run, 1);
    }
    HIP_TRY(c, hipMemcpyAsync(c->d_cb_off, off.data(), off.size() * sizeof(unsigned), hipMemcpyHostToDevice, st));
    hipLaunchKernelGGL(rt_cb_build<true>, grid, dim3(256), 0, st, S, F, (const unsigned*)c->d_cb_off, (unsigned*)nullptr,
                       c->d_cb_flag, c->d_cb_ent);
    HIP_TRY(c, hipGetLastError());
    hipLaunchKernelGGL(rt_cb_keys, dim3((nt + 255) / 256), dim3(256), 0, st, (const unsigned*)c->d_cb_off, nt,
                       c->d_cb_ent);
    HIP_TRY(c, hipGetLastError());
    HIP_TRY(c, hipStreamSynchronize(st));  // off[] (host) must outlive the copy
    cb_key_of(f, c->cb_key);
    c->cb_valid = true;
    c->cb_entries = run;
    c->cb_build_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    return RT_OK;
}

static bool cb_matches(const rt_ctx* c, const rt_frame* f)
{
    if (!c->cb_valid) return false;
    float key[25];
    cb_key_of(f, key);
    return std::memcmp(key, c->cb_key, sizeof key) == 0;
}

// allow_build: synchronous renders may (re)build the camera buffer; the
// async path (no host sync, capturable) uses it only when it is current.
static int launch(rt_ctx* c, const rt_frame* f, unsigned* rgba_dev, float* rgb_dev, hipStream_t st, bool timed,
                  bool allow_build = false)
{
    if (!c || !f) return RT_E_ARG;
    if (!c->uploaded) {
        c->err = "render before rt_upload_scene";
        return RT_E_STATE;
    }
    if (f->width <= 0 || f->height <= 0 || f->row_begin < 0 || f->row_end > f->height ||
        f->row_begin > f->row_end || f->max_bounces < 0 ||
        (f->band_rows != 0 && rt_band_rows(f->height, f->band_rows, f->band_count, f->band_index) < 0)) {
        c->err = "bad rt_frame geometry";
        return RT_E_ARG;
    }
    const int depth = reachable_depth(c, f);
    int cap = 0, lb = 1;
    const int mode = lb_mode();
    const bool lbuf = c->lb_ready && (mode == 1 || (mode == 2 && c->n_tri > kClusterMinTriangles));
    const bool cb_want = depth == 0 && c->n_tri > 0 && cb_mode();
    const int rows = frame_rows(f);
    if (rows > 0) {
        const int rc = camera_prepass(c, f, st, cb_want);
        if (rc) return rc;
        if (cb_want && allow_build && !cb_matches(c, f)) {
            const int rc2 = cb_build(c, f, st);
            if (rc2) return rc2;
        }
    }
    const bool cbuf = cb_want && cb_matches(c, f);
    kernel_fn k = (f->flags & RT_FLAG_STATS) ? pick_kernel<true>(depth, c->n_tri, c->n_lights, lbuf, cbuf, cap, lb)
                                              : pick_kernel<false>(depth, c->n_tri, c->n_lights, lbuf, cbuf, cap, lb);
    if (!k) {
        c->err = "reachable bounce depth " + std::to_string(depth) + " exceeds the compiled stack (32)";
        return RT_E_UNSUPPORTED;
    }
    SceneDev S = scene_dev(c, lbuf, cbuf);
    FrameDev F;
    frame_dev(f, F);
    c->last = rt_stats{};
    c->last.stack_depth = cap;
    c->last.light_batch = lb;
    if (rows == 0) return RT_OK;
    if (f->flags & RT_FLAG_STATS) HIP_TRY(c, hipMemsetAsync(c->d_stats, 0, kStatSlots * sizeof(StatsDev), st));
    dim3 grid((f->width + 15) / 16, (rows + 15) / 16);
    if (timed) HIP_TRY(c, hipEventRecord(c->ev0, st));
    StatsDev* stats = c->d_stats;
    void* args[] = {&S, &F, &rgba_dev, &rgb_dev, &stats};
    HIP_TRY(c, hipLaunchKernel((const void*)k, grid, dim3(256), args, 0, st));
    if (timed) HIP_TRY(c, hipEventRecord(c->ev1, st));
    return RT_OK;
}

static int finish_sync(rt_ctx* c, const rt_frame* f, hipStream_t st, bool timed)
{
    HIP_TRY(c, hipStreamSynchronize(st));
    if (timed) {
        float ms = 0.f;
        HIP_TRY(c, hipEventElapsedTime(&ms, c->ev0, c->ev1));
        c->last.kernel_ms = ms;
    }
    if (f->flags & RT_FLAG_STATS) {
        std::vector<StatsDev> slots(kStatSlots);
        HIP_TRY(c, hipMemcpy(slots.data(), c->d_stats, kStatSlots * sizeof(StatsDev), hipMemcpyDeviceToHost));
        StatsDev h{};
        for (const StatsDev& q : slots) {
            h.primary += q.primary;
            h.bounce += q.bounce;
            h.shadow += q.shadow;
            h.skipped += q.skipped;
            h.tri += q.tri;
            h.pla += q.pla;
            h.qua += q.qua;
        }
        c->last.primary_rays = h.primary;
        c->last.bounce_rays = h.bounce;
        c->last.shadow_rays = h.shadow;
        c->last.shadow_tests_skipped = h.skipped;
        c->last.triangle_tests = h.tri;
        c->last.plane_tests = h.pla;
        c->last.quadric_tests = h.qua;
    }
    return RT_OK;
}

static bool is_device_ptr(const void* p)
{
    hipPointerAttribute_t a;
    if (hipPointerGetAttributes(&a, p) != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    return a.type == hipMemoryTypeDevice || a.type == hipMemoryTypeManaged;
}

static int ensure_scratch(rt_ctx* c, size_t bytes)
{
    if (c->scratch_bytes >= bytes) return RT_OK;
    hipFree(c->d_scratch);
    c->d_scratch = nullptr;
    c->scratch_bytes = 0;
    HIP_TRY(c, hipMalloc(&c->d_scratch, bytes));
    c->scratch_bytes = bytes;
    return RT_OK;
}

static int render_sync(rt_ctx* c, const rt_frame* f, void* out, bool as_float)
{
    if (!c || !f || !out) return RT_E_ARG;
    HIP_TRY(c, hipSetDevice(c->device));
    const size_t px = (size_t)f->width * (size_t)std::max(0, frame_rows(f));
    const size_t bytes = px * (as_float ? 12 : 4);
    const bool dev = is_device_ptr(out);
    void* target = out;
    if (!dev) {
        int rc = ensure_scratch(c, std::max<size_t>(bytes, 16));
        if (rc) return rc;
        target = c->d_scratch;
    }
    int rc = launch(c, f, as_float ? nullptr : (unsigned*)target, as_float ? (float*)target : nullptr, c->stream, true,
                    true);
    if (rc) return rc;
    if (!dev && bytes) HIP_TRY(c, hipMemcpyAsync(out, target, bytes, hipMemcpyDeviceToHost, c->stream));
    return finish_sync(c, f, c->stream, true);
}

RT_EXPORT int rt_render(rt_ctx* c, const rt_frame* f, uint8_t* rgba8_out) { return render_sync(c, f, rgba8_out, false); }

RT_EXPORT int rt_render_float(rt_ctx* c, const rt_frame* f, float* rgb_out) { return render_sync(c, f, rgb_out, true); }

RT_EXPORT int rt_render_async(rt_ctx* c, const rt_frame* f, uint8_t* rgba8_dev, float* rgb_dev, void* stream)
{
    if (!c || !f) return RT_E_ARG;
    return launch(c, f, (unsigned*)rgba8_dev, rgb_dev, (hipStream_t)stream, false);
}

RT_EXPORT int rt_last_stats(rt_ctx* c, rt_stats* out)
{
    if (!c || !out) return RT_E_ARG;
    *out = c->last;
    return RT_OK;
}

#ifdef RT_PROF
// Diagnostic builds only (not in include/rt.h): read and clear the per-section
// shader-clock totals (summed over waves).
extern "C" __attribute__((visibility("default"))) int rt_debug_prof(unsigned long long* out8)
{
    if (hipMemcpyFromSymbol(out8, HIP_SYMBOL(rt::rt_prof_acc), 8 * sizeof(unsigned long long)) != hipSuccess)
        return RT_E_HIP;
    unsigned long long z[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    if (hipMemcpyToSymbol(HIP_SYMBOL(rt::rt_prof_acc), z, sizeof z) != hipSuccess) return RT_E_HIP;
    return RT_OK;
}
// Per-tile records of the next renders (device buffer of 16 x u32 per 8x8
// tile, tile = tile_row * (2 * grid.x) + tile_col); NULL turns it off.
extern "C" __attribute__((visibility("default"))) int rt_debug_prof_tiles(unsigned* dev, int ntiles)
{
    if (hipMemcpyToSymbol(HIP_SYMBOL(rt::rt_prof_tiles), &dev, sizeof dev) != hipSuccess) return RT_E_HIP;
    if (hipMemcpyToSymbol(HIP_SYMBOL(rt::rt_prof_ntiles), &ntiles, sizeof ntiles) != hipSuccess) return RT_E_HIP;
    return RT_OK;
}
// Same for the wave-uniform event counts (summed over waves).
extern "C" __attribute__((visibility("default"))) int rt_debug_prof_events(unsigned long long* out8)
{
    if (hipMemcpyFromSymbol(out8, HIP_SYMBOL(rt::rt_prof_ev), 8 * sizeof(unsigned long long)) != hipSuccess)
        return RT_E_HIP;
    unsigned long long z[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    if (hipMemcpyToSymbol(HIP_SYMBOL(rt::rt_prof_ev), z, sizeof z) != hipSuccess) return RT_E_HIP;
    return RT_OK;
}
#endif

// Diagnostic (not in include/rt.h): light-buffer summary of the uploaded
// scene: out[0] = built (0/1), out[1] = entries, out[2] = build ms,
// then per light (up to (n - 3) / 3): R, dcap-list length, dcov.
RT_EXPORT int rt_debug_lb_info(rt_ctx* c, double* out, int n)
{
    if (!c || !out || n < 3) return RT_E_ARG;
    out[0] = c->lb_ready ? 1.0 : 0.0;
    out[1] = (double)c->lb_entries;
    out[2] = c->lb_build_ms;
    if (!c->lb_ready) return RT_OK;
    std::vector<float4> meta((size_t)c->n_lights * 2);
    HIP_TRY(c, hipMemcpy(meta.data(), c->d_lb_meta, meta.size() * sizeof(float4), hipMemcpyDeviceToHost));
    for (int j = 0; j < c->n_lights && 3 + 3 * j + 2 < n; ++j) {
        int R;
        unsigned nd;
        std::memcpy(&R, &meta[2 * j].w, 4);
        std::memcpy(&nd, &meta[2 * j].z, 4);
        out[3 + 3 * j] = R;
        out[4 + 3 * j] = nd;
        out[5 + 3 * j] = meta[2 * j + 1].x;
    }
    return RT_OK;
}

// Diagnostic (not in include/rt.h): camera-buffer summary: out[0] = current
// (0/1), out[1] = entries, out[2] = last build ms, out[3] = tiles.
RT_EXPORT int rt_debug_cb_info(rt_ctx* c, double* out, int n)
{
    if (!c || !out || n < 4) return RT_E_ARG;
    out[0] = c->cb_valid ? 1.0 : 0.0;
    out[1] = (double)c->cb_entries;
    out[2] = c->cb_build_ms;
    out[3] = (double)c->cb_ntiles;
    return RT_OK;
}

// Diagnostic (not in include/rt.h): run rt_selftest_kernel over `blocks`
// workgroups; *failures = lanes whose wave reduction or wave cone was wrong.
RT_EXPORT int rt_debug_selftest(int device, int blocks, unsigned* failures)
{
    if (!failures || blocks <= 0) return RT_E_ARG;
    if (hipSetDevice(device) != hipSuccess) return RT_E_HIP;
    unsigned* d = nullptr;
    if (hipMalloc(&d, sizeof(unsigned)) != hipSuccess) return RT_E_HIP;
    int rc = RT_OK;
    if (hipMemset(d, 0, sizeof(unsigned)) != hipSuccess) rc = RT_E_HIP;
    if (rc == RT_OK) {
        hipLaunchKernelGGL(rt_selftest_kernel, dim3((unsigned)blocks), dim3(256), 0, 0, 12345u, d);
        if (hipGetLastError() != hipSuccess || hipDeviceSynchronize() != hipSuccess ||
            hipMemcpy(failures, d, sizeof(unsigned), hipMemcpyDeviceToHost) != hipSuccess)
            rc = RT_E_HIP;
    }
    hipFree(d);
    return rc;
}

