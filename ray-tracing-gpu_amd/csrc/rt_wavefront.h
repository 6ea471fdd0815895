// rt_wavefront.h — wavefront bounce levels for the BVH scenes: the
// commented reflect/refract recursion (Scene.cpp:1779-1823) unrolled level
// by level through queues in HBM instead of a per-lane DFS stack, so each
// bounce level runs as its own launch over a COMPACTED queue of live rays
// (ballot + prefix per wave, one atomic per wave) — full waves for the
// BVH walk and the shading, whatever fraction of the pixels still bounces.
// Part of the device code of rt_kernels.hip (one translation unit: the
// kernels are templates instantiated by its host half); built with the
// same exactness flags (no FMA contraction, IEEE div/sqrt).
//
// Level 0 is the depth-0 kernel (camera rays, camera buffer, light buffer)
// with WAVE bit 512: a pixel whose hit spawns children writes a node record
// instead of its colour.  Level L >= 1 (rt_wf_level): each queued ray is
// traced through the BVH, shaded, and either spawns children into level
// L + 1 (a node record) or writes its colour.  Then the levels fold from the
// deepest up (rt_wf_fold): a node's colour is ((acc + C_refl * Kr) + C_refr
// * Kt) — the reference's order, Scene.cpp:1787 then :1822 — from its
// children's colours, and level 0's parents write their pixels.  Every ray
// is the same ray the DFS traces (same origin P = O + t D, Reflect /
// Refract of the same operands, same gates), and every fold one thread's
// fixed-order sums, so the image is the DFS's bit for bit; the queue order
// (atomic per wave) changes nothing but where records live.
#ifndef RT_AMD_RT_WAVEFRONT_H
#define RT_AMD_RT_WAVEFRONT_H

#include "rt_bvh.h"

#pragma clang fp contract(off)


namespace rt {

__device__ __forceinline__ unsigned lane_rank(unsigned long long m)
{
    return __builtin_amdgcn_mbcnt_hi((unsigned)(m >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)m, 0u));
}

__device__ __forceinline__ void wave_bins_count(bool on, unsigned key, unsigned* __restrict__ hist)
{
    const int lane = (int)(threadIdx.x & 63);
    unsigned cnt = 0u;
    unsigned long long left = __ballot(on);
    while (left) {
        const int lead = (int)__builtin_ctzll(left);
        const unsigned k0 = (unsigned)__builtin_amdgcn_readlane((int)key, lead);
        const unsigned long long same = __ballot(on & (key == k0)) & left;
        if (lane == lead) cnt = (unsigned)__popcll(same);
        left &= ~same;
    }
    if (cnt > 0u) atomicAdd(&hist[key], cnt);  // every bin's first lane, one instruction
}
// The wave's bins are found first (each lane: its bin's first lane and its
// rank there; the first lane: the bin's count), then every bin's first lane
// claims the bin's positions in ONE atomic instruction, and every lane
// takes its first lane's.
__device__ __forceinline__ unsigned wave_bins_place(bool on, unsigned key, unsigned* __restrict__ next)
{
    const int lane = (int)(threadIdx.x & 63);
    unsigned cnt = 0u, rank = 0u;
    int lead_of = lane;
    unsigned long long left = __ballot(on);
    while (left) {
        const int lead = (int)__builtin_ctzll(left);
        const unsigned k0 = (unsigned)__builtin_amdgcn_readlane((int)key, lead);
        const unsigned long long same = __ballot(on & (key == k0)) & left;
        if (lane == lead) cnt = (unsigned)__popcll(same);
        if ((same >> lane) & 1ull) {
            lead_of = lead;
            rank = lane_rank(same);
        }
        left &= ~same;
    }
    unsigned mine = 0u;
    if (cnt > 0u) mine = atomicAdd(&next[key], cnt);
    return (unsigned)__shfl((int)mine, lead_of) + rank;
}

// A segmented queue as the consumer sees it: the prefix sums of its
// kWfSeg segment counts (wave-uniform: scalar loads of the counters the
// previous launch left) and the slot of compacted index x.
struct WfQueue {
    unsigned pre[kWfSeg + 1];
    unsigned seg;
};
__device__ __forceinline__ WfQueue wf_queue(const unsigned* count, int first_word, unsigned seg)
{
    WfQueue q;
    q.seg = seg;
    q.pre[0] = 0u;
#pragma unroll
    for (int k = 0; k < kWfSeg; ++k) q.pre[k + 1] = q.pre[k] + count[first_word + k * kWfCntStride];
    return q;
}
__device__ __forceinline__ unsigned wf_slot(const WfQueue& q, unsigned x)
{
    unsigned p = 0u, s = 0u;
#pragma unroll
    for (int k = 1; k < kWfSeg; ++k) {
        const bool ge = x >= q.pre[k];
        p = ge ? q.pre[k] : p;
        s = ge ? (unsigned)k : s;
    }
    return s * q.seg + (x - p);
}

// The children of a level-L node (act: a ray of level L that hit a surface
// of material m at P with normal N, coming along D with ray IOR rior and
// energy; acc its local colour; self its index — the pixel for level 0, the
// ray for level L >= 1).  Gates of Scene.cpp:1780 / :1791 (bounces = L);
// reflected rays keep CRayon's default IOR 0 (:1782-1788), refracted ones
// Scene.cpp:1793-1822.  Returns true when the node spawned a child (its
// colour then comes from rt_wf_fold).  chunk: the wave's 64-ray chunk (or
// tile) index, which picks its segments.
__device__ __forceinline__ bool wf_children(const FrameDev& F, int L, bool act, const Mat& m, const Vec3 P,
                                            const Vec3 N, const Vec3 D, float rior, float energy, const Color acc,
                                            unsigned self, unsigned chunk, int surf)
{
    const float er = m.kr * energy;
    const float et = m.kt * energy;
    const bool can = act & (L < F.max_bounces) & (L < F.wf.levels);
    const bool doR = can & (er > F.min_energy);
    const bool doT = can & (et > F.min_energy);
    const unsigned long long bR = __ballot(doR), bT = __ballot(doT), bP = __ballot(doR | doT);
    if (bP == 0ull) return false;
    // one atomic per wave for the rays, one for the parents; slots in lane
    // order, reflected children first
    const int lead = (int)__builtin_ctzll(__ballot(true));
    const int lane = (int)(threadIdx.x & 63);
    const int sg = (int)(chunk % (unsigned)kWfSeg);
    unsigned base = 0u, pbase = 0u;
    if (lane == lead) {
        base = atomicAdd(&F.wf.count[wf_rays(L + 1, sg)], (unsigned)(__popcll(bR) + __popcll(bT)));
        pbase = atomicAdd(&F.wf.count[wf_pars(L, sg)], (unsigned)__popcll(bP));
    }
    base = (unsigned)__builtin_amdgcn_readlane((int)base, lead) + (unsigned)sg * F.wf.seg[L + 1];
    pbase = (unsigned)__builtin_amdgcn_readlane((int)pbase, lead) + (unsigned)sg * F.wf.pseg[L];
    int cR = -1, cT = -1;
    float4* const q = F.wf.ray[L + 1];
    if (doR) {
        cR = (int)(base + lane_rank(bR));
        const Vec3 Dr = reflect(D, N);
        q[2 * (size_t)cR] = make_float4(P.x, P.y, P.z, 0.0f);
        q[2 * (size_t)cR + 1] = make_float4(Dr.x, Dr.y, Dr.z, er);
        if (F.wf.kin) F.wf.kin[cR] = F.wf.skey[surf];
    }
    if (doT) {
        cT = (int)(base + (unsigned)__popcll(bR) + lane_rank(bT));
        Vec3 n = N;
        float ratio, rior_t;
        if (rior == m.ior) {  // Scene.cpp:1797-1803 inside -> out
            rior_t = F.scene_ior;
            ratio = m.ior / F.scene_ior;
            n = -n;
        } else {
            rior_t = m.ior;
            ratio = F.scene_ior / m.ior;
        }
        const Vec3 Dt = refract(D, n, ratio);
        q[2 * (size_t)cT] = make_float4(P.x, P.y, P.z, rior_t);
        q[2 * (size_t)cT + 1] = make_float4(Dt.x, Dt.y, Dt.z, et);
        if (F.wf.kin) F.wf.kin[cT] = F.wf.skey[surf] + F.wf.nbin_half;
    }
    if (F.wf.kin) {  // the coherence sort's bin counts (rt_wf_sort_place)
        const unsigned kb = (doR | doT) ? F.wf.skey[surf] : 0u;
        if (bR) wave_bins_count(doR, kb, F.wf.hist);
        if (bT) wave_bins_count(doT, kb + F.wf.nbin_half, F.wf.hist);
    }
    if (doR | doT) {
        float4* nd = F.wf.node[L] + 2 * (size_t)self;
        nd[0] = make_float4(acc.r, acc.g, acc.b, m.kr);
        nd[1] = make_float4(m.kt, __int_as_float(cR), __int_as_float(cT), 0.0f);
        F.wf.plist[L][pbase + lane_rank(bP)] = self;
    }
    return doR | doT;
}

// The coherence sort of a level's live rays by bin (WfDev::kin), a counting
// sort whose work follows the rays, not the queue's capacity: the producers
// (the level-0 kernel, the shade launches) count each appended ray into
// hist[bin] as they write its bin (wf_children); before the level's trace
// the host scans the counts into each bin's first position (zeroing them
// for the next level), and rt_wf_sort_place claims positions and writes the
// level's slots to kout in bin order.  Both use one atomic per distinct bin
// of a wave (wave_bins_*: rays of one parent triangle sit together in a
// wave).  The order inside a bin is the atomics' — every ray is
// independent, so the image does not depend on it.
// KEY 0: the ray's parent bin (kin, counted by its producer); KEY 1 (the
// hit sort before a level's shade, RT_OPT_WF_SORT 2 / 3): its hit surface's
// bin — so the shading, its light-buffer cells, and the children it appends
// (whose parent is that surface) stay together — and for a miss one of
// kWfMissBins bins by its 64-ray chunk of the trace's order (one bin for
// every miss serialised all waves' atomics on one address).
// order: the level's slots in the trace's order (null: queue order).
constexpr unsigned kWfMissBins = 256;
constexpr int kWfPending = -2;  // hit[slot] of a straggler whose minimum goes to hit2 (WfDev::hit2)
// KEY 2 (RT_OPT_WF_SORT bit 2 with bit 1): the light-buffer cell of the hit
// point seen from light 0 (lb_cell of P - light, the direction the shading's
// lookup takes, at light 0's first buffer's resolution), so a wave's lanes
// share one cell and walk its list once (lb_slot's one-cell path); misses in
// kWfMissBins bins after the 6 R^2 cells.  Only the order: the key may be
// any function of the ray.
template <int KEY>
__device__ __forceinline__ unsigned wf_sort_key(const SceneDev& S, const FrameDev& F, int L, unsigned slot,
                                                unsigned x)
{
    if constexpr (KEY == 0) return F.wf.kin[slot];
    const float2 h = F.wf.hit[slot];
    const int idx = __float_as_int(h.x);
    if constexpr (KEY == 2) {
        const int R = __float_as_int(S.lb_meta[0].w);
        const unsigned ncell = 6u * (unsigned)R * (unsigned)R;
        if (idx < 0) return ncell + ((x >> 6) & (kWfMissBins - 1u));
        const float4 r0 = F.wf.ray[L][2 * (size_t)slot], r1 = F.wf.ray[L][2 * (size_t)slot + 1];
        const Vec3 P = make3(r0.x, r0.y, r0.z) + h.y * make3(r1.x, r1.y, r1.z);
        const float4 l0 = S.lights[0];
        return (unsigned)lb_cell(P - make3(l0.x, l0.y, l0.z), R);
    }
    return idx >= 0 ? F.wf.skey[idx] : F.wf.nbin_half + ((x >> 6) & (kWfMissBins - 1u));
}

template <int KEY>
__global__ __launch_bounds__(64) void rt_wf_hit_count(const SceneDev S, const FrameDev F, int L,
                                                      const unsigned* __restrict__ order, unsigned* __restrict__ hist)
{
    const WfQueue Q = wf_queue(F.wf.count, wf_rays(L, 0), F.wf.seg[L]);
    const unsigned n = Q.pre[kWfSeg];
    for (unsigned base = blockIdx.x * 64u; base < n; base += gridDim.x * 64u) {
        const unsigned x = base + (threadIdx.x & 63u);
        const bool valid = x < n;
        const unsigned slot = valid ? (order ? order[x] : wf_slot(Q, x)) : 0u;
        wave_bins_count(valid, valid ? wf_sort_key<KEY>(S, F, L, slot, x) : 0u, hist);
    }
}

template <int KEY>
__global__ __launch_bounds__(64) void rt_wf_sort_place(const SceneDev S, const FrameDev F, int L,
                                                       const unsigned* __restrict__ order, unsigned* __restrict__ next,
                                                       unsigned* __restrict__ kout)
{
    const WfQueue Q = wf_queue(F.wf.count, wf_rays(L, 0), F.wf.seg[L]);
    const unsigned n = Q.pre[kWfSeg];
    for (unsigned base = blockIdx.x * 64u; base < n; base += gridDim.x * 64u) {
        const unsigned x = base + (threadIdx.x & 63u);
        const bool valid = x < n;
        const unsigned slot = valid ? (order ? order[x] : wf_slot(Q, x)) : 0u;
        const unsigned k = valid ? wf_sort_key<KEY>(S, F, L, slot, x) : 0u;
        const unsigned pos = wave_bins_place(valid, k, next);
        if (valid) kout[pos] = slot;
    }
}

// Bounce level L >= 1 runs as two launches over the level's queue (a
// grid-stride loop over the count the previous launch left, 64 rays per
// wave; every wave leaves when the queue is exhausted):
//  * rt_wf_trace: each ray's closest hit, through the BVH (rt_bvh.h) —
//    alone, so the walk's node and triangle records keep the L2 to
//    themselves and its small register and LDS footprint (the stack only,
//    depth x 256 bytes) keeps many waves in flight for its dependent loads;
//  * rt_wf_shade: the hit's shading (light buffer) and its children.
template <bool COUNT>
__device__ __forceinline__ void wf_tally(const Counters& cnt, StatsDev* __restrict__ stats)
{
    unsigned long long v[9] = {cnt.primary, cnt.bounce, cnt.shadow, cnt.skipped, cnt.tri,
                               cnt.pla,     cnt.qua,    cnt.btri,   cnt.bnode};
    StatsDev* sl = stats + (blockIdx.x % kStatSlots);
    unsigned long long* dst[9] = {&sl->primary, &sl->bounce, &sl->shadow, &sl->skipped, &sl->tri,
                                  &sl->pla,     &sl->qua,    &sl->btri,   &sl->bnode};
#pragma unroll
    for (int k = 0; k < 9; ++k) {
        const unsigned long long w = wave_sum_u64(v[k]);
        if ((threadIdx.x & 63) == 0) atomicAdd(dst[k], w);
    }
}

// Persistent lanes (round 5): a lane whose walk ends takes the queue's next
// ray instead of idling until its wave's longest walk ends (the level's rays
// skim a rough mesh: walks of 10 to 200+ steps side by side, VALU lane
// utilisation 0.28 with one ray per lane per wave round).  Each round the
// free lanes refill from the level's fetch cursor — one atomic per wave,
// only once at least kWfRefill lanes are free (or none is busy), so the
// cursor sees a few atomics per 64 rays — then every busy lane takes one
// while-while round of its walk (closest_hit_bvh's, step for step: inner
// nodes until every busy lane holds a leaf, then the leaves).  A lane's
// ray, its stack (its own LDS column), bounds and order are its walk alone,
// so each ray's minimum is closest_hit_bvh's; the budget and the straggler
// hand-off are unchanged.
// (refill at 16 / 32 / 48 free lanes, with the launch shapes of
// profiles/r05/sorder/: c3r 3.110 / 2.945 / 2.933 ms, c5r 23.06 / 19.00 /
// 18.32 — ab_knobs.log)
#ifndef RT_WF_REFILL
#define RT_WF_REFILL 48
#endif
constexpr int kWfRefill = RT_WF_REFILL;

template <bool COUNT>
__global__ __launch_bounds__(64) void rt_wf_trace(const SceneDev S, const FrameDev F, int L,
                                                  StatsDev* __restrict__ stats)
{
    const WfQueue Q = wf_queue(F.wf.count, wf_rays(L, 0), F.wf.seg[L]);
    const unsigned n = Q.pre[kWfSeg];
    const float4* __restrict__ q = F.wf.ray[L];
    unsigned* const cursor = F.wf.count + wf_fetch(L);
    int* const stk = bvh_stack<0>();
    const int lane = (int)(threadIdx.x & 63);
    constexpr int kDone = 0x7fffffff;
    Counters cnt;
    bool busy = false, more = true;  // more: the cursor has not passed n (wave-uniform)
    unsigned slot = 0u;
    Vec3 O = make3(0.f, 0.f, 0.f), D = O, inv = O;
    float bt = -1.0f;
    int bi = -1, node = kDone, leaf = 0, sp = 0, steps = 0;
#define WF_PUSH(x)            \
    do {                      \
        stk[64 * sp] = (x);   \
        ++sp;                 \
    } while (0)
#define WF_POP(dst) (dst) = sp > 0 ? stk[64 * --sp] : kDone
    for (;;) {
        const unsigned long long fm = __ballot(!busy);
        if (more && fm && (__popcll(fm) >= kWfRefill || !__any(busy))) {
            const int lead = (int)__builtin_ctzll(fm);
            unsigned b = 0u;
            if (lane == lead) b = atomicAdd(cursor, (unsigned)__popcll(fm));
            b = (unsigned)__builtin_amdgcn_readlane((int)b, lead);
            more = b + (unsigned)__popcll(fm) < n;
            const unsigned x = b + lane_rank(fm);
            if (!busy && x < n) {
                slot = F.wf.kout ? F.wf.kout[x] : wf_slot(Q, x);
                const float4 r0 = q[2 * (size_t)slot], r1 = q[2 * (size_t)slot + 1];
                O = make3(r0.x, r0.y, r0.z);
                D = make3(r1.x, r1.y, r1.z);
                ++cnt.bounce;
                // closest_hit_bvh's prologue: planes, quadrics, the walk test
                bt = -1.0f;
                bi = -1;
                for (int k = 0; k < S.n_plane; ++k) {
                    const float4 a = S.plane[2 * k], c = S.plane[2 * k + 1];
                    float t;
                    ++cnt.pla;
                    const bool ok = hit_plane(make_float4(0.f, a.x, a.y, a.z), make_float4(a.w, 0.f, 0.f, 0.f), O, D, t);
                    take_min(ok, t, __float_as_int(c.x), bt, bi);
                }
                for (int k = 0; k < S.n_quad; ++k) {
                    const float4* r = S.quad + 3 * k;
                    const float4 a = r[0], c = r[1], e = r[2];
                    float t;
                    ++cnt.qua;
                    const bool ok = hit_quadric(make_float4(0.f, a.x, a.y, a.z), make_float4(a.w, c.x, c.y, c.z),
                                                make_float4(c.w, e.x, e.y, 0.f), O, D, t);
                    take_min(ok, t, __float_as_int(e.z), bt, bi);
                }
                const float dd = dot(D, D);
                if (finite3(O) & finite3(D) & (dd >= 0.98f) & (dd <= 1.02f)) {
                    inv = make3(__builtin_amdgcn_rcpf(D.x), __builtin_amdgcn_rcpf(D.y), __builtin_amdgcn_rcpf(D.z));
                    node = 0;
                    leaf = 0;
                    sp = 0;
                    steps = 0;
                    busy = true;
                } else {  // every triangle (closest_hit_bvh's non-walk branch)
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
                    F.wf.hit[slot] = make_float2(__int_as_float(bi), bt);
                }
            }
        }
        if (!__any(busy)) {
            if (!more) break;
            continue;
        }
        // one while-while round of every busy lane's walk
        bool fin = false, str = false;
        if (busy) {
            while ((node >= 0) & (node != kDone)) {
                if (++steps > F.wf.budget) break;
                const float4* nd = S.bvh_node + 4 * (size_t)node;
                const float4 a0 = nd[0], a1 = nd[1], b0 = nd[2], b1 = nd[3];
                ++cnt.bnode;
                const int r0 = __float_as_int(a1.w), r1 = __float_as_int(b1.w);
                float t0, t1;
                const bool have = bi >= 0;
                const bool h0 = bvh_box(a0, a1, O, inv, have, bt, t0);
                const bool h1 = bvh_box(b0, b1, O, inv, have, bt, t1);
                if (h0 & h1) {
                    const bool near0 = !(t1 < t0);
                    WF_PUSH(near0 ? r1 : r0);
                    node = near0 ? r0 : r1;
                } else if (h0 | h1) {
                    node = h0 ? r0 : r1;
                } else {
                    WF_POP(node);
                }
                if ((node < 0) & (leaf == 0)) {  // postpone the first leaf, walk on
                    leaf = node;
                    WF_POP(node);
                }
                if (__all(leaf != 0)) break;
            }
            if (steps > F.wf.budget) {
                str = true;
            } else {
                while (leaf != 0) {
                    const unsigned enc = ~(unsigned)leaf;
                    const int first = (int)(enc >> 4), count = (int)(enc & 15u) + 1;
                    for (int k = first; k < first + count; ++k) {
                        const float4* r = S.bvh_tri + 3 * (size_t)k;
                        const float4 a = r[0], c = r[1], e = r[2];
                        ++cnt.tri;
                        ++cnt.btri;
                        float t;
                        const bool ok = hit_triangle(make_float4(0.f, a.x, a.y, a.z), make_float4(a.w, c.x, c.y, c.z),
                                                     make_float4(c.w, e.x, 0.f, 0.f), O, D, t);
                        take_min(ok, t, __float_as_int(e.y), bt, bi);
                    }
                    leaf = 0;
                    if ((node < 0) & (node != kDone)) {  // the leaf that ended the inner loop
                        leaf = node;
                        WF_POP(node);
                    }
                    ++steps;
                }
                fin = node == kDone;
            }
        }
        // a walk past the budget goes to the straggler queue with its partial
        // minimum (rt_wf_straggle finishes it with a whole wave)
        const unsigned long long bs = __ballot(str);
        if (bs) {
            const int lead = (int)__builtin_ctzll(bs);
            unsigned sb = 0u;
            if (lane == lead) sb = atomicAdd(&F.wf.count[wf_strag(L)], (unsigned)__popcll(bs));
            sb = (unsigned)__builtin_amdgcn_readlane((int)sb, lead);
            if (str) F.wf.strag[sb + lane_rank(bs)] = make_int4((int)slot, __float_as_int(bt), bi, 0);
            if (str && F.wf.hit2) F.wf.hit[slot] = make_float2(__int_as_float(kWfPending), bt);
        }
        if (fin) F.wf.hit[slot] = make_float2(__int_as_float(bi), bt);
        if (fin | str) busy = false;
    }
    if (COUNT && (F.flags & RT_FLAG_STATS)) wf_tally<COUNT>(cnt, stats);
#undef WF_PUSH
#undef WF_POP
}

// The straggling walks of level L, one ray per wave (bvh_walk_wave: the
// wave's LDS stack of kWfStragCap references).
#ifndef RT_WF_STRAG_CAP
#define RT_WF_STRAG_CAP 1024
#endif
constexpr int kWfStragCap = RT_WF_STRAG_CAP;
template <bool COUNT>
__global__ __launch_bounds__(64) void rt_wf_straggle(const SceneDev S, const FrameDev F, int L,
                                                     StatsDev* __restrict__ stats)
{
    extern __shared__ float4 rt_lds_dyn[];
    int* const stk = reinterpret_cast<int*>(rt_lds_dyn);
    const unsigned n = F.wf.count[wf_strag(L)];
    const float4* __restrict__ q = F.wf.ray[L];
    Counters cnt;
    for (unsigned j = blockIdx.x; j < n; j += gridDim.x) {
        const int4 rec = F.wf.strag[j];
        const unsigned i = (unsigned)rec.x;
        const float4 r0 = q[2 * (size_t)i], r1 = q[2 * (size_t)i + 1];
        float bt = __int_as_float(rec.y);
        int bi = rec.z;
        bvh_walk_wave(S, make3(r0.x, r0.y, r0.z), make3(r1.x, r1.y, r1.z), bt, bi, stk, kWfStragCap, cnt);
        if ((threadIdx.x & 63) == 0) (F.wf.hit2 ? F.wf.hit2 : F.wf.hit)[i] = make_float2(__int_as_float(bi), bt);
    }
    if (COUNT && (F.flags & RT_FLAG_STATS)) {
        // the lanes tally the work they did; the wave's one ray counts once
        cnt.bounce = 0;
        wf_tally<COUNT>(cnt, stats);
    }
}

// Occupancy: at the compiler's free choice the shade kernel takes 87 VGPRs
// (5 waves per SIMD) and its light-buffer walks are latency-bound (L2 hit
// rate 0.29 on scattered hit points); bounded to 6 waves per SIMD it fits
// 80 VGPRs without spilling: c3r -5.8%, c5r -6.3% with a grid of 24 waves
// per CU (profiles/r05/sorder/ab_shade_occupancy*.log).
#ifndef RT_WF_SHADE_EU
#define RT_WF_SHADE_EU 6
#endif
// STRAG (RT_OPT_WF_OVERLAP, on the second stream after rt_wf_straggle):
// only the stragglers (hit = kWfPending), with their minima from hit2, in
// the same order and 64-ray chunks as the main launch — which skips them —
// so every chunk's children still go to its own queue segment.
template <int WAVE, bool COUNT, bool STRAG = false>
__global__ __launch_bounds__(64, RT_WF_SHADE_EU) void rt_wf_shade(const SceneDev S, const FrameDev F, int L,
                                                  StatsDev* __restrict__ stats)
{
    const WfQueue Q = wf_queue(F.wf.count, wf_rays(L, 0), F.wf.seg[L]);
    const unsigned n = Q.pre[kWfSeg];
    const Color bg{F.bg[0], F.bg[1], F.bg[2]};
    Counters cnt;
    const float4* __restrict__ q = F.wf.ray[L];
    for (unsigned base = blockIdx.x * 64u; base < n; base += gridDim.x * 64u) {
        const unsigned x = base + (threadIdx.x & 63u);
        if (x < n) {
            const unsigned i = F.wf.kout ? F.wf.kout[x] : wf_slot(Q, x);
            float2 h = F.wf.hit[i];
            const bool pending = __float_as_int(h.x) == kWfPending;
            if constexpr (STRAG) {
                if (!pending) continue;
                h = F.wf.hit2[i];
            } else {
                if (pending) continue;
            }
            const int idx = __float_as_int(h.x);
            Color res = bg;
            bool parent = false;
            if (idx >= 0) {
                const float4 r0 = q[2 * (size_t)i], r1 = q[2 * (size_t)i + 1];
                const Vec3 O = make3(r0.x, r0.y, r0.z), D = make3(r1.x, r1.y, r1.z);
                const float t = h.y;
                const Vec3 N = hit_normal(S, idx, O, D, t);
                const Mat m = load_mat(S, idx);
                const Vec3 P = O + t * D;
#ifdef RT_WF_NO_SHADE  // timing experiment only (wrong images)
                res = m.color;
#else
                res = shade_local<1, WAVE>(S, m, P, N, D, cnt);
#endif
                parent = wf_children(F, L, true, m, P, N, D, r0.w, r1.w, res, i, base / 64u, idx);
            }
            if (!parent) F.wf.res[L][i] = make_float4(res.r, res.g, res.b, 0.0f);
        }
    }
    if (COUNT && (F.flags & RT_FLAG_STATS)) wf_tally<COUNT>(cnt, stats);
}

// Fold level L (deepest first): each parent's colour from its children's,
// in the reference's order; level 0 writes the parents' pixels.
__global__ __launch_bounds__(256) void rt_wf_fold(const FrameDev F, int L, unsigned* __restrict__ rgba,
                                                  float* __restrict__ rgbf)
{
    const WfQueue Q = wf_queue(F.wf.count, wf_pars(L, 0), F.wf.pseg[L]);
    const unsigned n = Q.pre[kWfSeg];
    const float4* __restrict__ child = F.wf.res[L + 1];
    for (unsigned j = blockIdx.x * blockDim.x + threadIdx.x; j < n; j += gridDim.x * blockDim.x) {
        const unsigned i = F.wf.plist[L][wf_slot(Q, j)];
        const float4 a = F.wf.node[L][2 * (size_t)i], b = F.wf.node[L][2 * (size_t)i + 1];
        Color c{a.x, a.y, a.z};
        const int cR = __float_as_int(b.y), cT = __float_as_int(b.z);
        if (cR >= 0) {
            const float4 r = child[cR];
            c += Color{r.x, r.y, r.z} * a.w;  // Scene.cpp:1787
        }
        if (cT >= 0) {
            const float4 r = child[cT];
            c += Color{r.x, r.y, r.z} * b.x;  // Scene.cpp:1822
        }
        if (L > 0) {
            F.wf.res[L][i] = make_float4(c.r, c.g, c.b, 0.0f);
        } else {
            if (rgbf) {
                rgbf[3 * (size_t)i] = c.r;
                rgbf[3 * (size_t)i + 1] = c.g;
                rgbf[3 * (size_t)i + 2] = c.b;
            }
            if (rgba) rgba[i] = unorm8(c.r) | (unorm8(c.g) << 8) | (unorm8(c.b) << 16) | 0xFF000000u;
        }
    }
}

}  // namespace rt
#endif  // RT_AMD_RT_WAVEFRONT_H
