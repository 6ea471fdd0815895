// rt_primitives.h — the exact ray-primitive tests (Triangle / Plan / Quadrique) and the
// camera-ray / closest-hit building blocks.
// Part of the device code of rt_kernels.hip (one translation unit: the
// kernels are templates instantiated by its host half); built with the
// same exactness flags (no FMA contraction, IEEE div/sqrt).
#ifndef RT_AMD_RT_PRIMITIVES_H
#define RT_AMD_RT_PRIMITIVES_H

#include "rt_layout.h"

#pragma clang fp contract(off)

namespace rt {

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
        if constexpr (!CAMERA) ++cnt.btri;  // bounce rays: every triangle
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

}  // namespace rt
#endif  // RT_AMD_RT_PRIMITIVES_H
