// rt_shade.h — shading: shadow rays (per-lane, wave-culled, light-buffer forms),
// the shadow filter and the local Phong colour.
// Part of the device code of rt_kernels.hip (one translation unit: the
// kernels are templates instantiated by its host half); built with the
// same exactness flags (no FMA contraction, IEEE div/sqrt).
#ifndef RT_AMD_RT_SHADE_H
#define RT_AMD_RT_SHADE_H

#include "rt_lightbuf.h"
#include "rt_cambuf.h"

#pragma clang fp contract(off)

namespace rt {

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
    const bool edges = S.use_edges;
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

// LDS-staged per-lane walk (the big-list kernel: C5 -11%, C3 -6.5%; the
// small-list kernel measured slower with it): when
// the wave's lanes fall in a few cells, every still-active lane of one cell is
// at the same entry of its list (each active lane consumes one entry per
// iteration), so the wave stages the next W entries of every cell's list in
// its own LDS window with ONE batch of coalesced loads, and the lanes read
// their entries from LDS — one load latency per W entries instead of a
// dependent gather per entry.  Same tests, same order per lane: the any-hit
// result is the global walk's.  Returns false (nothing done) for more cells
// than it stages (kLbLdsG).
constexpr int kLbLdsG = 4;  // most cells a wave stages
__device__ __forceinline__ bool lb_walk_lds(const SceneDev& S, bool use, int cell, unsigned e, unsigned end,
                                            const Vec3 P, const Vec3 L, float dist, bool& occ, Counters& cnt)
{
    unsigned long long rem = __ballot(use);
    unsigned gp[kLbLdsG], ge[kLbLdsG];
    unsigned long long gm[kLbLdsG];
    int ng = 0, grp = 0;
#pragma unroll
    for (int i = 0; i < kLbLdsG; ++i) {
        gp[i] = ge[i] = 0u;
        gm[i] = 0ull;
        if (rem) {
            const int lead = (int)__builtin_ctzll(rem);
            const int c = __builtin_amdgcn_readlane(cell, lead);
            const unsigned long long m = __ballot(use & (cell == c));
            gp[i] = (unsigned)__builtin_amdgcn_readlane((int)e, lead);
            ge[i] = (unsigned)__builtin_amdgcn_readlane((int)end, lead);
            gm[i] = m;
            if (use & (cell == c)) grp = i;
            rem &= ~m;
            ng = i + 1;
        }
    }
    if (rem) return false;
    // window per cell: the capacity over the cell count rounded up to a power of 2
    const int lg = ng <= 1 ? 0 : 32 - __builtin_clz((unsigned)(ng - 1));
    const int sh = __builtin_ctz((unsigned)kLbLdsCap) - lg;
    const unsigned wmask = (1u << sh) - 1u;
    const LdsWin win = lds_window();
    const unsigned long long ex = __ballot(true);
    const int nact = __popcll(ex);
    const int rk = (int)__builtin_amdgcn_mbcnt_hi((unsigned)(ex >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)ex, 0u));
    bool have = use & (e < end);
    unsigned k = 0;  // entries each active lane has consumed (wave-uniform)
    const int nslots = ng << sh;
    for (;;) {
        const bool act = have & !occ;
        const unsigned long long ba = __ballot(act);
        if (!ba) break;
        if ((k & wmask) == 0) {  // stage entries k .. k + W - 1 of every cell with an active lane
            unsigned gact = 0;
#pragma unroll
            for (int i = 0; i < kLbLdsG; ++i) gact |= (ba & gm[i]) ? (1u << i) : 0u;
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            for (int s = rk; s < nslots; s += nact) {
                const int gi = s >> sh;
                unsigned q0 = gp[0], q1 = ge[0];
#pragma unroll
                for (int i = 1; i < kLbLdsG; ++i) {
                    q0 = gi == i ? gp[i] : q0;
                    q1 = gi == i ? ge[i] : q1;
                }
                const unsigned q = q0 + k + ((unsigned)s & wmask);
                if (((gact >> gi) & 1u) && q < q1) {
                    float4 a, b;
                    float2 c;
                    lb_cell_entry(S.lb_ent, q, a, b, c);
                    win.a[s] = a;
                    win.b[s] = b;
                    win.c[s] = c;
                }
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        }
        RT_EV(cnt, 3);
        const int slot = (grp << sh) + (int)(k & wmask);
        bool go = false;
        float4 c0 = make_float4(0.f, 0.f, 0.f, 0.f), c1 = c0;
        float2 c2 = make_float2(0.f, 0.f);
        if (act) {
            c0 = win.a[slot];
            if (!(c0.w < dist)) {
                have = false;  // this and every later entry lie beyond P (dmin)
            } else {
                go = true;
                c1 = win.b[slot];
                c2 = win.c[slot];
            }
        }
        ++k;
        have = have & (e + k < end);
        if (__any(go)) {
            ++cnt.tri;
            RT_EV(cnt, 4);
            RT_EVN(cnt, 7, (unsigned)__popcll(__ballot(go)));
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
    return true;
}

// One buffer slot's walk for the lanes in `cand` (slot = a light, or
// n_lights + the light for its far buffer): the lanes whose dist the slot
// covers (dist <= its dcov) look their cell up, walk its list, then the
// slot's dcap list while their dist exceeds the entries' caps.  Returns
// those lanes (the covered ones).
// BIG (the big-list kernel): multi-cell waves walk staged in LDS, and lanes
// beyond a level's dcov take the next level of the ladder.
template <bool BIG, bool UNROLL = false>
__device__ __forceinline__ bool lb_slot(const SceneDev& S, int slot, const Vec3 P, const Vec3 L, float dist, bool cand,
                                        bool& occ, Counters& cnt)
{
    const float4 m0 = S.lb_meta[2 * slot], m1 = S.lb_meta[2 * slot + 1];
    const unsigned obase = __float_as_uint(m0.x), dbase = __float_as_uint(m0.y), ndcap = __float_as_uint(m0.z);
    const int R = __float_as_int(m0.w);
    const float dcov = m1.x;
    const Vec3 d = -L;
    const bool use = cand & !occ & (dist <= dcov) & (R > 0);
    const int cell = use ? lb_cell(d, R) : 0;
    RT_MARK(cnt, 3);
    // Every lane that uses the buffer in ONE cell (a tile's points seen from
    // the light usually are, at coarse resolutions): the wave walks that list
    // once, its entries by wave-uniform scalar loads into SGPRs — no per-lane
    // gathers.  A lane takes an entry while it lies nearer than the lane's
    // point (the list is nearest-first, so the first entry no live lane
    // takes ends the walk for all); the any-hit result is the per-lane walk's.
    const unsigned long long bu = __ballot(use);
    const int cf = bu ? __builtin_amdgcn_readlane(cell, (int)__builtin_ctzll(bu)) : 0;
    const bool one_cell = bu != 0 && __all(!use | (cell == cf));
    unsigned e = 0, end = 0;
    if (bu) {
        if (one_cell) RT_EV(cnt, 0);
        else RT_EV(cnt, 1);
    }
    if (one_cell) {
        const unsigned* o = S.lb_off + obase + cf;
        const unsigned q0 = o[0], q1 = o[1];
        for (unsigned q = q0; q < q1; ++q) {
            const float* r = lb_rec(S.lb_ent, q);
            const float4 c0 = lb_a(r);
            if (!__any(use & !occ & (c0.w < dist))) break;
            const float4 c1 = lb_b(r);
            const float2 c2 = lb_tail(r);
            const bool act = use & !occ & (c0.w < dist);
            ++cnt.tri;
            RT_EV(cnt, 4);
            if (act) {
                const Vec3 e1 = make3(c1.x, c1.y, c1.z), e2 = make3(c1.w, c2.x, c2.y);
                const TriU u = tri_u(make3(c0.x, c0.y, c0.z), e1, e2, P, L);
                if (__any(u.ok)) {
                    float t;
                    const bool ok = tri_vt(u, e1, e2, L, t);
                    occ |= ok & (t > kEps) & (t < dist);
                }
            }
        }
    } else if (use) {
        const unsigned* o = S.lb_off + obase + cell;
        e = o[0];
        end = o[1];
    }
    // big lists: waves over 2-4 cells walk their lists staged in LDS
    if (BIG && !one_cell && bu && lb_walk_lds(S, use, cell, e, end, P, L, dist, occ, cnt))
        end = e;  // walked: skip the global walk below
    bool have = e < end;
    if constexpr (UNROLL) {
        // The per-lane walk two entries per round (WAVE bit 2048: the
        // big-list depth-0 kernel on frames under 4 Mpx, whose 8 x 8 tiles
        // see more cells than the LDS-staged walk takes): the two loads
        // issue together, so a lit point's long list (every entry nearer
        // than the light) waits one load latency per two entries.  Entries
        // are taken in list order while nearer than P (dmin < dist), as one
        // at a time; an entry past an occluding one is not tested.
        // (profiles/r06/lbwalk/: C3 -6%; on other kernels the extra
        // registers cost occupancy, so only there.)
        for (;;) {
            const bool act = have & !occ;
            if (!__any(act)) break;
            RT_EV(cnt, 3);
            constexpr int K = 2;
            float4 c0[K], c1[K];
            float2 c2[K];
            bool go[K];
#pragma unroll
            for (int k = 0; k < K; ++k) {
                c0[k] = c1[k] = make_float4(0.f, 0.f, 0.f, 0.f);
                c2[k] = make_float2(0.f, 0.f);
                go[k] = false;
                if (act & (e + (unsigned)k < end)) lb_cell_entry(S.lb_ent, e + (unsigned)k, c0[k], c1[k], c2[k]);
            }
            if (act) {
                bool open = true;
#pragma unroll
                for (int k = 0; k < K; ++k) {
                    go[k] = open & (e < end) & (c0[k].w < dist);
                    e += go[k] ? 1u : 0u;
                    open = go[k];
                }
                have = open & (e < end);
            }
#pragma unroll
            for (int k = 0; k < K; ++k) {
                const bool g = go[k] & !occ;
                if (__any(g)) {
                    ++cnt.tri;
                    RT_EV(cnt, 4);
                    if (g) {
                        const Vec3 e1 = make3(c1[k].x, c1[k].y, c1[k].z), e2 = make3(c1[k].w, c2[k].x, c2[k].y);
                        const TriU u = tri_u(make3(c0[k].x, c0[k].y, c0[k].z), e1, e2, P, L);
                        if (__any(u.ok)) {
                            float t;
                            const bool ok = tri_vt(u, e1, e2, L, t);
                            occ |= ok & (t > kEps) & (t < dist);
                        }
                    }
                }
            }
        }
    } else {
        for (;;) {
            const bool act = have & !occ;
            if (!__any(act)) break;
            RT_EV(cnt, 3);
            bool go = false;
            float4 c0 = make_float4(0.f, 0.f, 0.f, 0.f), c1 = c0;
            float2 c2 = make_float2(0.f, 0.f);
            if (act) {
                lb_cell_entry(S.lb_ent, e, c0, c1, c2);
                if (!(c0.w < dist)) {
                    have = false;  // this and every later entry lie beyond P (dmin)
                } else {
                    go = true;
                    ++e;
                    have = e < end;
                }
            }
            if (__any(go)) {
                ++cnt.tri;
                RT_EV(cnt, 4);
                RT_EVN(cnt, 7, (unsigned)__popcll(__ballot(go)));  // lanes doing a test (RT_PROF)
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
    }
    RT_MARK(cnt, 4);
    // pairs not culled up to dcov: sorted by dcap, so once no live lane lies
    // beyond an entry's cap none lies beyond a later one
    for (unsigned q = 0; q < ndcap; ++q) {
        const float* r = lb_rec(S.lb_dcap, dbase + q);
        const float4 r0 = lb_a(r);
        const bool need = use & !occ & (dist > r0.w);
        if (!__any(need)) break;
        ++cnt.tri;
        RT_EV(cnt, 5);
        const float4 r1 = lb_b(r);
        const float2 r2 = lb_tail(r);
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
    return use;
}

// One light's shadow rays against the OPAQUE surfaces with the light buffer
// (shadow_split scenes).  occ: in = lanes without a shadow ray, out = also
// the occluded ones (any-hit, so the order of the tests is free).  Lanes
// within the light's buffer distance walk it (lb_slot); with far buffers
// (big lists, S.lb_R levels) the lanes beyond walk the next level's; lanes
// no buffer covers take the per-lane loop over every triangle.
template <bool BIG, bool UNROLL = false>
__device__ __forceinline__ void shadow_opaque_lb(const SceneDev& S, int l, const Vec3 P, const Vec3 L, float dist,
                                                 bool& occ, Counters& cnt)
{
    for (int k = 0; k < S.n_plane_opaque; ++k) {
        if (!__any(!occ)) return;
        ++cnt.pla;
        occ |= shadow_plane_hit(S.plane[2 * k], P, L, dist);
    }
    {
    const float mx = fmaxf(fabsf(L.x), fmaxf(fabsf(L.y), fabsf(L.z)));
    const bool cand = !occ & (mx >= 0.5f);  // a direction the lookup takes
    bool use = lb_slot<BIG, UNROLL>(S, l, P, L, dist, cand, occ, cnt);
    if constexpr (BIG) {  // big lists: lanes beyond a buffer take the next
        for (int lv = 1; lv < S.lb_R; ++lv) {
            if (!__any(cand & !use & !occ)) break;
            use |= lb_slot<BIG, UNROLL>(S, lv * S.n_lights + l, P, L, dist, cand & !use, occ, cnt);
        }
    }
    const float slack = dist * 1e-6f;
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
            shadow_opaque_lb<((WAVE) & 2) != 0, ((WAVE) & 2048) != 0>(S, li, P, L, dist, occ, cnt);
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
        RT_MARK(cnt, 3);
        if (use_wave) shadow_opaque_wave<kLightBatch, (WAVE & 3) == 2>(S, lb, nl, tmask, P, L, dist, occ, wc, dmax, cnt);
        else shadow_opaque_batch<kLightBatch>(S, lb, nl, P, L, dist, occ, cnt);
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

}  // namespace rt
#endif  // RT_AMD_RT_SHADE_H
