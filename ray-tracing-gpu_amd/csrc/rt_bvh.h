// rt_bvh.h — exact bounding-volume hierarchy for bounce rays (reflected and
// refracted rays of depth > 0 frames: arbitrary origins, so none of the
// apex-based cones of rt_cull.h applies).
// Part of the device code of rt_kernels.hip (one translation unit: the
// kernels are templates instantiated by its host half); built with the
// same exactness flags (no FMA contraction, IEEE div/sqrt).
//
// The reference traces every bounce ray through the all-surface loop of
// ObtenirCouleur (Scene.cpp:1705-1715, called from the commented block
// :1779-1823).  Here the triangles are walked through a BVH2 whose boxes are
// grown by a margin that provably holds every hit the reference's f32 test
// (Triangle.cpp:127-172) can REPORT, so skipping a box never changes the
// winner of the lexicographic (t, file index) minimum:
//
//   a reported hit (|det~| >= 0.01, u~ in [0,1], v~ >= 0, fl(u~+v~) <= 1)
//   puts the exact point O + t~ D within
//       mu = eps (40 K + 4) |S| + 16 eps L
//   of the triangle, K = |D||e1||e2| / |det| <= 1.01 |e1||e2| / (0.01 -
//   6.1 eps 1.01 |e1||e2|), S = O - p0, L = max(|e1|, |e2|), eps = 2^-24
//
// (forward error analysis of Moller-Trumbore: with exact P = D x e2,
// det = e1.P, u = S.P/det, Q = S x e1, v = D.Q/det, t = e2.Q/det the exact
// identity O + tD = p0 + u e1 + v e2 holds, so O + t~D - (p0 + u~e1 + v~e2)
// = (t~-t)D - (u~-u)e1 - (v~-v)e2.  det~'s relative error r (|det~ - det|
// <= 5.83 eps |D||e1||e2|) divides u~, v~ and t~ alike, which moves the
// point by r (tD - u e1 - v e2) = -r S: 5.83 eps K |S|; the numerators err
// by <= 6.83 eps |S| |.||.| each: 20.5 eps K |S|; the reciprocal and the
// products round by 2 eps: 2 eps (|S| + 4 L); fl(u~+v~) <= 1 leaves Y =
// p0 + u~e1 + v~e2 within eps L of the triangle — 26.3 eps K |S| + 2 eps |S|
// + 9 eps L to first order; 40, 4 and 16 carry a 1.5x safety factor.
// tools/bvh_bound_probe.py samples adversarial near-grazing pairs: the
// largest dist / mu seen is 0.06.)
//
// Per box the host stores alpha = max over its triangles of eps (40 K + 4)
// + 32 eps (raised by 1e-5 relative and 1e-6 absolute for the rounding of
// the box test itself); the device bounds |S| by sb, the L1 distance from O
// to the box's farthest corner, and grows the box by alpha sb (16 eps L <=
// 32 eps sb: sb >= half the box's L1 extent >= half any edge inside it),
// then runs a slab test whose interval is widened by 1e-6 relative.  A box is skipped when that interval ends before EPS or
// starts after the best reported t (strictly: a tie at t == best still
// needs the file-index compare).
// Rays that are not finite or not unit length (|D|^2 outside [0.98, 1.02]:
// the reference's Normaliser returns (0,0,0) for short vectors) walk every
// triangle instead.
#ifndef RT_AMD_RT_BVH_H
#define RT_AMD_RT_BVH_H

#include "rt_cull.h"

#pragma clang fp contract(off)

namespace rt {

// Per-lane traversal stack in LDS, after the wave's staging window (the
// kernel's `win` bytes: kLdsWaveBytes where the shading stages light-buffer
// entries, 0 in the wavefront's trace kernel): entry i of lane l at word
// 64 i + l (lane-contiguous rows, no bank conflicts).  A path of d inner
// nodes pushes at most d entries: the launch gives depth x 256 bytes, and
// the host enables the BVH only for depth <= kBvhStack.
constexpr int kBvhStack = 24;
constexpr size_t kBvhLdsBytes = (size_t)kBvhStack * 64 * sizeof(int);

template <size_t WIN>
__device__ __forceinline__ int* bvh_stack()
{
    extern __shared__ float4 rt_lds_dyn[];
    return reinterpret_cast<int*>(rt_lds_dyn + WIN / sizeof(float4)) + (threadIdx.x & 63);
}

// Inner node (4 float4 = 64 bytes, two per 128-byte line): child c's box
// [lo.xyz alpha] [hi.xyz ref] for c = 0, 1: ref >= 0 an inner node, ref < 0
// the leaf ~(first << 4 | (count - 1)) of bvh_tri (3 float4 per triangle,
// tri[]'s layout).
//
// One child box against the ray (inv = per-component reciprocals of D;
// a zero component gives +-inf, see the NaN note below).  tn = the entry
// distance (lower bound), for the near-first order.
__device__ __forceinline__ bool bvh_box(const float4 lo, const float4 hi, const Vec3 O, const Vec3 inv, bool have,
                                        float bt, float& tn)
{
    const float dlx = lo.x - O.x, dly = lo.y - O.y, dlz = lo.z - O.z;
    const float dhx = hi.x - O.x, dhy = hi.y - O.y, dhz = hi.z - O.z;
    // |S| <= the L1 distance from O to the box's farthest corner
    const float sb = fmaxf(fabsf(dlx), fabsf(dhx)) + fmaxf(fabsf(dly), fabsf(dhy)) + fmaxf(fabsf(dlz), fabsf(dhz));
    const float mu = lo.w * sb;
    const float ax = (dlx - mu) * inv.x, bx = (dhx + mu) * inv.x;
    const float ay = (dly - mu) * inv.y, by = (dhy + mu) * inv.y;
    const float az = (dlz - mu) * inv.z, bz = (dhz + mu) * inv.z;
    // A NaN (0 * inf: a zero direction component with O exactly on a grown
    // face) is dropped by min/max — the ray then lies in that face, at
    // distance >= mu from every triangle of the box, so dropping the box is
    // exact; were it propagated, no comparison below would hold and the box
    // would be kept.
    const float tmin = fmaxf(fmaxf(fminf(ax, bx), fminf(ay, by)), fminf(az, bz));
    const float tmax = fminf(fminf(fmaxf(ax, bx), fmaxf(ay, by)), fmaxf(az, bz));
    // widened by 1e-6 relative (a product, so +-inf stays +-inf)
    const float t0 = tmin * (tmin > 0.0f ? 1.0f - 1e-6f : 1.0f + 1e-6f);
    const float t1 = tmax * (tmax > 0.0f ? 1.0f + 1e-6f : 1.0f - 1e-6f);
    tn = t0;
    return !(t0 > t1) & !(t1 < kEps) & !(have & (t0 > bt));
}

__device__ __forceinline__ unsigned lane_rank_u(unsigned long long m)
{
    return __builtin_amdgcn_mbcnt_hi((unsigned)(m >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)m, 0u));
}

__device__ __forceinline__ bool finite3(const Vec3 v)
{
    return (fabsf(v.x) <= 3.4e38f) & (fabsf(v.y) <= 3.4e38f) & (fabsf(v.z) <= 3.4e38f);
}

// Scene.cpp:1705-1715 for a bounce ray: planes and quadrics one by one, the
// triangles through the BVH.  Same winner as closest_hit<false>: the file
// order's first minimum is the lexicographic (t, file index) minimum, which
// does not depend on the order the candidates are tested in.
// BUDGET > 0 (the wavefront's trace kernel): a walk still running after that
// many steps (inner nodes + leaves) stops with *straggled set and its
// partial minimum in best_t / the return value — a valid starting bound for
// bvh_walk_wave, which finishes it with the whole wave.
template <size_t WIN = kLdsWaveBytes, int BUDGET = 0>
__device__ __forceinline__ int closest_hit_bvh(const SceneDev& S, const Vec3 O, const Vec3 D, float& best_t,
                                               Counters& cnt, bool* straggled = nullptr)
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
    const float dd = dot(D, D);
    const bool walk = finite3(O) & finite3(D) & (dd >= 0.98f) & (dd <= 1.02f);
    if (!walk) {  // every triangle (the bound assumes a finite, unit-length ray)
        for (int k = 0; k < S.n_tri; ++k) {
            const TriRec tr = load_tri(S, k);
            ++cnt.tri;
            ++cnt.btri;
            float t;
            const bool ok = hit_triangle(make_float4(0.f, tr.p0.x, tr.p0.y, tr.p0.z),
                                         make_float4(tr.e1.x, tr.e1.y, tr.e1.z, tr.e2.x),
                                         make_float4(tr.e2.y, tr.e2.z, 0.f, 0.f), O, D, t);
            take_min(ok, t, tr.idx, bt, bi);
        }
    } else {
        const Vec3 inv = make3(__builtin_amdgcn_rcpf(D.x), __builtin_amdgcn_rcpf(D.y), __builtin_amdgcn_rcpf(D.z));
        int* const stk = bvh_stack<WIN>();
        // "while-while" (Aila & Laine): a lane walks inner nodes until it
        // holds a leaf, postponing the first leaf it meets, and the wave
        // leaves the inner loop once every lane still in it holds one; then
        // the lanes test their leaves together — the inner steps (2 box
        // tests) and the leaf steps (up to 4 exact triangle tests) no longer
        // both run in every iteration of a wave with lanes of both kinds.
        constexpr int kDone = 0x7fffffff;  // (never an inner node index)
        int node = 0, leaf = 0, sp = 0, steps = 0;  // leaf: 0 = none, else a leaf reference (< 0)
        for (;;) {
            while ((node >= 0) & (node != kDone)) {
                if constexpr (BUDGET > 0) {
                    if (++steps > BUDGET) break;
                }
                const float4* n = S.bvh_node + 4 * (size_t)node;
                const float4 a0 = n[0], a1 = n[1], b0 = n[2], b1 = n[3];
                ++cnt.bnode;
                const int r0 = __float_as_int(a1.w), r1 = __float_as_int(b1.w);
                float t0, t1;
                const bool have = bi >= 0;
                const bool h0 = bvh_box(a0, a1, O, inv, have, bt, t0);
                const bool h1 = bvh_box(b0, b1, O, inv, have, bt, t1);
                if (h0 & h1) {
                    const bool near0 = !(t1 < t0);
                    stk[64 * sp] = near0 ? r1 : r0;
                    ++sp;
                    node = near0 ? r0 : r1;
                } else if (h0 | h1) {
                    node = h0 ? r0 : r1;
                } else {
                    node = sp > 0 ? stk[64 * --sp] : kDone;
                }
                if ((node < 0) & (leaf == 0)) {  // postpone the first leaf, walk on
                    leaf = node;
                    node = sp > 0 ? stk[64 * --sp] : kDone;
                }
                if (__all(leaf != 0)) break;
            }
            if constexpr (BUDGET > 0) {
                if (steps > BUDGET) {
                    *straggled = true;
                    break;
                }
            }
            while (leaf != 0) {
                const unsigned enc = ~(unsigned)leaf;
                const int first = (int)(enc >> 4), count = (int)(enc & 15u) + 1;
                for (int k = first; k < first + count; ++k) {
                    const float4* r = S.bvh_tri + 3 * (size_t)k;
                    const float4 a = r[0], b = r[1], c = r[2];
                    ++cnt.tri;
                    ++cnt.btri;
                    float t;
                    const bool ok = hit_triangle(make_float4(0.f, a.x, a.y, a.z), make_float4(a.w, b.x, b.y, b.z),
                                                 make_float4(b.w, c.x, 0.f, 0.f), O, D, t);
                    take_min(ok, t, __float_as_int(c.y), bt, bi);
                }
                leaf = 0;
                if ((node < 0) & (node != kDone)) {  // the leaf that ended the inner loop
                    leaf = node;
                    node = sp > 0 ? stk[64 * --sp] : kDone;
                }
                if constexpr (BUDGET > 0) ++steps;
            }
            if (node == kDone) break;
        }
    }
    best_t = bt;
    return bi;
}

// Lexicographic (t, file index) minimum of the wave's lanes' candidates
// (bi < 0: none), combined with the running (bt, bi): every lane gets it.
__device__ __forceinline__ void wave_take_min(float lt, int li, float& bt, int& bi)
{
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
        const float ot = __shfl_xor(lt, off, 64);
        const int oi = __shfl_xor(li, off, 64);
        if ((oi >= 0) & ((li < 0) | (ot < lt) | ((ot == lt) & (oi < li)))) {
            lt = ot;
            li = oi;
        }
    }
    if ((li >= 0) & ((bi < 0) | (lt < bt) | ((lt == bt) & (li < bi)))) {
        bt = lt;
        bi = li;
    }
}

// One ray's BVH walk by the whole wave (the stragglers of the budgeted
// walk: a ray skimming the mesh whose walk would hold its wave for
// thousands of dependent steps).  A shared stack of node references in LDS
// (cap entries at stk): each round the lanes take up to 64 references off
// its top — an inner node's two child boxes are tested (against the
// wave's current minimum), the ones that pass are pushed; a leaf's
// triangles are tested exactly — then one wave reduction updates the
// minimum.  The same boxes, the same exact tests and the same lexicographic
// minimum as the serial walk: only the order differs, which the minimum
// does not see.  The rounds take at most cap - 32 - sp references, so the
// stack never overflows (with one reference per round it grows by at most
// the tree's depth, <= kBvhStack).  Wave-uniform: every lane calls it with
// the same ray; (bt, bi) in: the partial minimum (planes, quadrics and the
// triangles tested so far), out: the ray's minimum.
__device__ __forceinline__ void bvh_walk_wave(const SceneDev& S, const Vec3 O, const Vec3 D, float& bt, int& bi,
                                              int* __restrict__ stk, int cap, Counters& cnt)
{
    const int lane = (int)(threadIdx.x & 63);
    const Vec3 inv = make3(__builtin_amdgcn_rcpf(D.x), __builtin_amdgcn_rcpf(D.y), __builtin_amdgcn_rcpf(D.z));
    int sp = 1;
    if (lane == 0) stk[0] = 0;
    for (;;) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        if (sp == 0) break;
        int take = min(64, min(sp, cap - 32 - sp));
        if (take < 1) take = 1;
        const int ref = lane < take ? stk[sp - take + lane] : 0;
        const bool mine = lane < take;
        sp -= take;
        float lt = -1.0f;
        int li = -1;
        bool p0 = false, p1 = false;
        int r0 = 0, r1 = 0;
        const bool have = bi >= 0;
        if (mine && ref >= 0) {
            const float4* n = S.bvh_node + 4 * (size_t)ref;
            const float4 a0 = n[0], a1 = n[1], b0 = n[2], b1 = n[3];
            ++cnt.bnode;
            r0 = __float_as_int(a1.w);
            r1 = __float_as_int(b1.w);
            float t0, t1;
            p0 = bvh_box(a0, a1, O, inv, have, bt, t0);
            p1 = bvh_box(b0, b1, O, inv, have, bt, t1);
        } else if (mine) {
            const unsigned enc = ~(unsigned)ref;
            const int first = (int)(enc >> 4), count = (int)(enc & 15u) + 1;
            for (int k = first; k < first + count; ++k) {
                const float4* r = S.bvh_tri + 3 * (size_t)k;
                const float4 a = r[0], b = r[1], c = r[2];
                ++cnt.tri;
                ++cnt.btri;
                float t;
                const bool ok = hit_triangle(make_float4(0.f, a.x, a.y, a.z), make_float4(a.w, b.x, b.y, b.z),
                                             make_float4(b.w, c.x, 0.f, 0.f), O, D, t);
                take_min(ok, t, __float_as_int(c.y), lt, li);
            }
        }
        // every lane has read its reference before the pushes overwrite them
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        const unsigned long long m0 = __ballot(p0), m1 = __ballot(p1);
        if (p0) stk[sp + (int)lane_rank_u(m0)] = r0;
        if (p1) stk[sp + __popcll(m0) + (int)lane_rank_u(m1)] = r1;
        sp += __popcll(m0) + __popcll(m1);
        wave_take_min(lt, li, bt, bi);
    }
}

}  // namespace rt
#endif  // RT_AMD_RT_BVH_H
