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
//  * one wave64 = one 8x8 pixel tile, lane l -> (l&7, l>>3); one wave per
//    workgroup;
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
#include <thread>
#include <vector>

#include "../../include/rt.h"
#include "../../include/rt_debug.h"
#include "rt_cpu.hpp"
#include "rt_scan.h"
#include "rt_shade.h"
#include "rt_bvh.h"
#include "rt_wavefront.h"

#pragma clang fp contract(off)

namespace rt {

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

// WAVE bit 512 (MAXD 0, the wavefront's level 0, rt_wavefront.h): a hit
// that spawns children writes a node record and its child rays instead of
// its colour (deferred: rt_wf_fold writes the pixel).
template <int MAXD, int LB, int WAVE>
__device__ Color radiance(const SceneDev& S, const FrameDev& F, Vec3 O, Vec3 D, Counters& cnt, bool live, int tile,
                          const TinyCam* T, unsigned tmask, unsigned pix, bool& deferred, unsigned chunk)
{
    const Color bg{F.bg[0], F.bg[1], F.bg[2]};
    if constexpr (MAXD == 0) {
        float t;
        RT_MARK(cnt, 0);
        const int idx = closest_hit_primary<(WAVE & 107)>(S, O, D, t, cnt, tile, T, tmask);
        RT_MARK(cnt, 1);
        // Lanes that miss (or lie outside the frame) stay in step through the
        // shading so the wave stays whole for wave-level shadow culling.
        const bool hit = idx >= 0;
        if (!__any(hit & live)) return bg;
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
        if constexpr ((WAVE & 512) != 0)
            deferred = wf_children(F, 0, hit & live, m, P, N, D, 1.0f, 1.0f, c, pix, chunk, sidx);
        return hit ? c : bg;
    } else if constexpr ((WAVE & 1024) != 0) {
        // Reflect-only scenes (no Kt can pass the gate: the host's kt_max <= 0
        // with min_energy >= 0): every node has at most one child, the
        // reflected ray, and its colour is acc + C_child * Kr (Scene.cpp:1787).
        // The chain's (acc, Kr) pairs live in registers — a shift stack with
        // compile-time indices, top at [0] — instead of the DFS's scratch
        // frames; the fold runs bottom-up in the same order.
        Color accs[MAXD];
        float krs[MAXD];
#pragma unroll
        for (int k = 0; k < MAXD; ++k) {
            accs[k] = Color{0.f, 0.f, 0.f};
            krs[k] = 0.f;
        }
        int d = 0;  // nodes on the chain (pushed)
        float energy = 1.0f;
        Color ret = bg;
        for (int lv = 0;; ++lv) {
            float t;
            int idx;
            if (lv == 0)
                idx = closest_hit_primary<(WAVE & 107)>(S, O, D, t, cnt, tile, T);
            else if constexpr ((WAVE & 256) != 0)  // bounce rays through the BVH (rt_bvh.h)
                idx = closest_hit_bvh(S, O, D, t, cnt);
            else
                idx = closest_hit<false>(S, O, D, t, cnt);
            ret = bg;
            if (idx < 0) break;
            const Vec3 N = hit_normal(S, idx, O, D, t);
            const Mat m = load_mat(S, idx);
            const Vec3 P = O + t * D;
            const Color acc = shade_local<LB, WAVE>(S, m, P, N, D, cnt);
            // Scene.cpp:1779-1781 gate; bounces == lv
            const float er = m.kr * energy;
            const bool doR = er > F.min_energy && lv < F.max_bounces && lv < MAXD;
            if (!doR) {
                ret = acc;
                break;
            }
#pragma unroll
            for (int k = MAXD - 1; k > 0; --k) {
                accs[k] = accs[k - 1];
                krs[k] = krs[k - 1];
            }
            accs[0] = acc;
            krs[0] = m.kr;
            ++d;
            ++cnt.bounce;
            O = P;
            D = reflect(D, N);  // Scene.cpp:1782-1788
            energy = er;
        }
#pragma unroll
        for (int k = 0; k < MAXD; ++k) {
            if (k < d) {
                Color a = accs[k];
                a += ret * krs[k];  // Scene.cpp:1787
                ret = a;
            }
        }
        return ret;
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
                int idx;
                if (camera_ray)
                    idx = closest_hit_primary<(WAVE & 107)>(S, O, D, t, cnt, tile, T);
                else if constexpr ((WAVE & 256) != 0)  // bounce rays through the BVH (rt_bvh.h)
                    idx = closest_hit_bvh(S, O, D, t, cnt);
                else
                    idx = closest_hit<false>(S, O, D, t, cnt);
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
// VGPRs, no spills) — C2 -4% against the unconstrained 5 waves, 6 waves
// +1-3% and 8 waves +40% (spills) at C2/C4.  The big-list kernels (WAVE 14:
// C3, C5) ran at 8 in round 1 (-3/-4% against 7) while spilling 9-10 VGPRs
// (44 B/lane of scratch: 1.4 GB of writes per C5 frame, tools/calib); with
// the LDS walks and an unpipelined global walk they fit 72 VGPRs with no
// scratch at 7 waves, as fast as 8 waves with spills (C3 -0.4%, C5 +0.5%)
// and 0.57 GB fewer bytes written per C5 frame.
#ifndef RT_WAVES_PER_EU
#define RT_WAVES_PER_EU 7
#endif
#ifndef RT_WAVES_PER_EU_BIG
#define RT_WAVES_PER_EU_BIG 7
#endif
// The launch-camera kernel that computes its tile masks (WAVE bit 64) is
// held to 64 VGPRs, 8 waves/SIMD (A/B, moving C2 camera: -2.3% against 7;
// the mask-reading kernel fits 58 VGPRs anyway, and asked for 8 measured
// +2.4% static).  RT_TINY_HOIST: its mask planes are loaded at the top of
// the kernel (A/B: -2.7% against loading them where the mask is computed).
#ifndef RT_WAVES_PER_EU_TINY
#define RT_WAVES_PER_EU_TINY 8
#endif
#ifndef RT_TINY_HOIST
#define RT_TINY_HOIST 1
#endif
constexpr int waves_per_eu(int maxd, int wave)
{
    return maxd != 0 ? 1
                     : ((wave & 64) ? RT_WAVES_PER_EU_TINY
                                    : ((wave & 15) == 14 ? RT_WAVES_PER_EU_BIG : RT_WAVES_PER_EU));
}
// One 8 x 8 tile (the body of both trace kernels below).
// COUNT: also tally the exact tests executed (the RT_FLAG_STATS launch); in
// the timed kernels the tallies are dead and compile away.
// T: the launch's camera records (WAVE bit 32, rt_trace_tiny), else nullptr.
template <int MAXD, int LB, int WAVE, bool COUNT>
__device__ __forceinline__ void trace_tile(const SceneDev& S, const FrameDev& F, unsigned* __restrict__ rgba,
                                           float* __restrict__ rgbf, StatsDev* __restrict__ stats, const TinyCam* T,
                                           int bx, int by)
{
    const int lane = threadIdx.x & 63;
    // XCD-aware block order: the dispatcher deals workgroups round-robin over
    // the 8 XCDs (each with its own L2), so workgroup w runs on XCD w % 8 as
    // that XCD's (w / 8)-th; give every XCD one contiguous run of blocks in
    // row-major order, so neighbouring tiles — which read the same cells,
    // tile lists and records — share an L2.  A bijection for any grid size.
    const int tile_x = bx;  // 8-pixel column of the wave's tile
    const int px = tile_x * 8 + (lane & 7);
    const int ly0 = by * 8;  // the wave's first output row
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
    TinyLane tl;
    if constexpr ((WAVE & 64) != 0 && RT_TINY_HOIST) tl = tiny_lane_load(*T);  // the mask's records, in flight under the set-up
    // Without bounces every lane runs (lanes outside the frame on a clamped
    // pixel, result dropped) so edge waves stay whole for wave-level culling.
    if (MAXD == 0 || valid) {
        const int pxc = px < F.width ? px : F.width - 1;
        const int pyc = py < rend ? py : rend - 1;
        const Vec3 D = camera_dir(F, pxc, pyc);
        const Vec3 O = make3(F.cam[0], F.cam[1], F.cam[2]);
        cnt.primary = valid ? 1u : 0u;
        // camera-buffer tile (or the launch records' tile): this wave's 8
        // rows must be one tile row of the full frame (the lists and boxes
        // hold for its lanes' clamped pixels, a superset of the wave's)
        int tile = -1;
        if ((WAVE & 8) && S.cb_tiles_x > 0 && (py0 & 7) == 0) {
            tile = (py0 >> 3) * S.cb_tiles_x + tile_x;
            if (S.cb_flag[tile]) tile = -1;
        }
        unsigned tmask = 0;
        if ((WAVE & 32) && (py0 & 7) == 0) tile = (py0 >> 3) * T->tiles_x + tile_x;
        if constexpr ((WAVE & 64) != 0 && !RT_TINY_HOIST) tl = tiny_lane_load(*T);
        if constexpr ((WAVE & 64) != 0) tmask = tiny_tile_mask(*T, tl, D);
        const size_t o = (size_t)ly * F.width + px;
        bool deferred = false;
        c = radiance<MAXD, LB, WAVE>(S, F, O, D, cnt, valid, tile, T, tmask, (unsigned)o, deferred,
                                     (unsigned)(by * F.tiles_x + bx));
        if (valid & !deferred) {
            if (rgbf) {
                rgbf[3 * o] = c.r;
                rgbf[3 * o + 1] = c.g;
                rgbf[3 * o + 2] = c.b;
            }
            // Nontemporal (streaming) stores in the small-list kernels: the
            // frame's lines leave each XCD's L2 during the kernel instead of
            // in the release at its end (A/B, same images: C2 -1 to -2%, C4
            // -2%, C1 +1%).  Not in the big-list kernels: at C5 they write
            // each 128-B line out twice (WRITE_SIZE 134 -> 268 MB per frame:
            // 32-B tile rows evicted before the neighbouring tiles fill the
            // line) for -0.5%.
            if (rgba) {
                const unsigned px8 = unorm8(c.r) | (unorm8(c.g) << 8) | (unorm8(c.b) << 16) | 0xFF000000u;
                if constexpr (!(WAVE & 2)) __builtin_nontemporal_store(px8, rgba + o);
                else rgba[o] = px8;
            }
        }
        // the tile's mask for its camera's later frames on this stream (WAVE
        // bit 128), stored last: at the top of the kernel the store's
        // completion held up the loads behind it (A/B: C2 -2.8%, C4 -2.5%)
        if constexpr ((WAVE & 128) != 0)
            if (lane == 0 && T->masked && tile >= 0) T->mask[tile] = tmask;
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
        const int tile = (int)(blockIdx.y * gridDim.x + blockIdx.x);
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
    // Only the COUNT variant (the RT_FLAG_STATS launch, pick_kernel) tallies:
    // in the timed kernels every counter is dead code.
    if (COUNT && (F.flags & RT_FLAG_STATS)) {
        unsigned long long v[9] = {cnt.primary, cnt.bounce, cnt.shadow, cnt.skipped, cnt.tri,
                                   cnt.pla,     cnt.qua,    cnt.btri,   cnt.bnode};
        StatsDev* sl = stats + ((blockIdx.x + blockIdx.y * gridDim.x) % kStatSlots);
        unsigned long long* dst[9] = {&sl->primary, &sl->bounce, &sl->shadow, &sl->skipped, &sl->tri,
                                      &sl->pla,     &sl->qua,    &sl->btri,   &sl->bnode};
        if (wave_full()) {  // one atomic per counter per wave
#pragma unroll
            for (int i = 0; i < 9; ++i) {
                const unsigned long long w = wave_sum_u64(v[i]);
                if ((threadIdx.x & 63) == 0) atomicAdd(dst[i], w);
            }
        } else {
#pragma unroll
            for (int i = 0; i < 9; ++i) atomicAdd(dst[i], v[i]);
        }
    }
}

// One wave per workgroup: one 8 x 8 tile each, so a CU takes a new tile as
// soon as any wave slot frees instead of four at once (A/B against 2 x 2
// tiles per workgroup: C3 -3.1%, C5 -4.5%, C4 -3.7%, scene7 -3.4%, scene9
// -1.4%, C2 -0.8%; declaring 64 threads: C5 -1.1%).
// XCD-aware block order: the dispatcher deals workgroups round-robin over
// the 8 XCDs (each with its own L2), so workgroup w runs on XCD w % 8 as
// that XCD's (w / 8)-th.  Big-list kernels (RT_OPT_XCD_DEAL, F.xcd_mode):
//  1: chunks of K consecutive blocks of a tile row go to one XCD, when the
//     grid divides evenly (C5 -1.4% against K = 4; C3's 240 x 135 tiles do
//     not divide: hardware order) — horizontal neighbours share an L2;
//  2: column stripes of xcd_w tiles, stripe s on XCD s % 8 (one stripe per
//     XCD by default, RT_OPT_XCD_STRIPE): XCD x walks its stripes' tiles row
//     by row, so a tile's horizontal AND vertical neighbours — which read
//     the same light-buffer cells, tile lists and records — share its L2,
//     while at any moment all XCDs work on the same frame rows (whole-region
//     runs per XCD were 1.8x slower on C3: the mesh rows piled onto a few
//     XCDs);
//  3: 4 x 2 super-tiles dealt round-robin over the XCDs;
//  0: hardware order.
// Modes 2 and 3 launch a padded grid (xcd_grid); its blocks past the frame's
// tiles return at once.  The small-list kernels: hardware order (C2 -2.5%
// against K = 4; the remap's code alone costs it).
template <int WAVE>
__device__ __forceinline__ bool tile_of_block(const FrameDev& F, int& bx, int& by)
{
    bx = (int)blockIdx.x;
    by = (int)blockIdx.y;
    constexpr unsigned K = (WAVE & 2) ? RT_XCD_CHUNK_BIG : RT_XCD_CHUNK_SMALL;
    if constexpr ((WAVE & 2) != 0) {
        const unsigned w = blockIdx.y * gridDim.x + blockIdx.x;
        const unsigned x = w % kXcds, i = w / kXcds;
        if (F.xcd_mode == 2) {
            const unsigned sw = (unsigned)F.xcd_w, m = (unsigned)F.xcd_m, j = i % m;
            bx = (int)((j / sw) * (kXcds * sw) + x * sw + j % sw);
            by = (int)(i / m);
            return bx < F.tiles_x && by < F.tiles_y;
        }
        if (F.xcd_mode == 3) {
            const unsigned st = (i / 8u) * kXcds + x, p = i % 8u, gx = (unsigned)F.xcd_w;
            bx = (int)((st % gx) * 4u + p % 4u);
            by = (int)((st / gx) * 2u + p / 4u);
            return bx < F.tiles_x && by < F.tiles_y;
        }
        if (F.xcd_mode == 0) return true;
    }
    if constexpr (K > 0) {
        const unsigned nb = gridDim.x * gridDim.y, w = blockIdx.y * gridDim.x + blockIdx.x;
        const unsigned x = w % kXcds, i = w / kXcds;
        const unsigned lw = ((i / K) * kXcds + x) * K + i % K;
        if (lw < nb && (nb % (kXcds * K)) == 0) {
            bx = (int)(lw % gridDim.x);
            by = (int)(lw / gridDim.x);
        }
    }
    return true;
}

template <int MAXD, int LB, int WAVE, bool COUNT>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(waves_per_eu(MAXD, WAVE)))) void rt_trace_kernel(
    const SceneDev S, const FrameDev F, unsigned* __restrict__ rgba, float* __restrict__ rgbf,
    StatsDev* __restrict__ stats)
{
    int bx, by;
    if (!tile_of_block<WAVE>(F, bx, by)) return;
    trace_tile<MAXD, LB, WAVE, COUNT>(S, F, rgba, rgbf, stats, nullptr, bx, by);
}

// Tiny scenes (WAVE bit 32): the camera records come with the launch
// (TinyCam by value, read from the kernel-argument segment by scalar loads).
template <int MAXD, int LB, int WAVE, bool COUNT>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(waves_per_eu(MAXD, WAVE)))) void rt_trace_tiny(
    const SceneDev S, const FrameDev F, const TinyCam T, unsigned* __restrict__ rgba, float* __restrict__ rgbf,
    StatsDev* __restrict__ stats)
{
    int bx, by;
    if (!tile_of_block<WAVE>(F, bx, by)) return;
    trace_tile<MAXD, LB, WAVE, COUNT>(S, F, rgba, rgbf, stats, &T, bx, by);
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

// Bounce-ray closest hits of arbitrary rays (rt_debug_bvh_rays): lane i
// takes ray i (O, D: 6 floats) through the BVH and through every triangle;
// out_idx / out_t get both winners (file index, t) as [bvh, brute].
__global__ __launch_bounds__(64) void rt_bvh_rays_kernel(const SceneDev S, const float* __restrict__ rays, int n,
                                                           int* __restrict__ out_idx, float* __restrict__ out_t,
                                                           unsigned long long* __restrict__ tally)
{
    const int i = (int)(blockIdx.x * 64 + threadIdx.x);
    if (i >= n) return;
    const float* r = rays + 6 * (size_t)i;
    const Vec3 O = make3(r[0], r[1], r[2]), D = make3(r[3], r[4], r[5]);
    Counters cnt;
    float tb, tf;
    const int ib = closest_hit_bvh(S, O, D, tb, cnt);
    const unsigned tests = cnt.btri, nodes = cnt.bnode;
    const int jf = closest_hit<false>(S, O, D, tf, cnt);
    out_idx[2 * i] = ib;
    out_idx[2 * i + 1] = jf;
    out_t[2 * i] = tb;
    out_t[2 * i + 1] = tf;
    atomicAdd(&tally[0], (unsigned long long)tests);
    atomicAdd(&tally[1], (unsigned long long)nodes);
}

// The wave-cooperative walk (rt_debug_bvh_rays_wave): one ray per wave, its
// planes and quadrics and first BVH step by the budgeted serial walk (budget
// 1: every ray straggles), the rest by bvh_walk_wave — as the wavefront's
// straggler kernel finishes a walk.
__global__ __launch_bounds__(64) void rt_bvh_wave_kernel(const SceneDev S, const float* __restrict__ rays, int n,
                                                           int* __restrict__ out_idx, float* __restrict__ out_t)
{
    extern __shared__ float4 rt_lds_dyn[];
    int* const base = reinterpret_cast<int*>(rt_lds_dyn);
    const int i = (int)blockIdx.x;
    if (i >= n) return;
    const float* r = rays + 6 * (size_t)i;
    const Vec3 O = make3(r[0], r[1], r[2]), D = make3(r[3], r[4], r[5]);
    Counters cnt;
    float bt = -1.0f;
    int bi = -1;
    bool str = false;
    if ((threadIdx.x & 63) == 0) {
        bi = closest_hit_bvh<kWfStragCap * sizeof(int), 1>(S, O, D, bt, cnt, &str);
    }
    bt = readlanef(bt, 0);
    bi = __builtin_amdgcn_readlane(bi, 0);
    str = __builtin_amdgcn_readlane((int)str, 0) != 0;
    if (str) bvh_walk_wave(S, O, D, bt, bi, base, kWfStragCap, cnt);
    if ((threadIdx.x & 63) == 0) {
        out_idx[i] = bi;
        out_t[i] = bt;
    }
}

}  // namespace rt

// ===================================================================== host
using namespace rt;

// Frames of rt_render_sequence_async in flight at once (one stream and one
// camera slot each): a frame's camera prepasses and trace kernel overlap the
// previous frames' (measured: 1 vs 4 streams, tools/overlap_probe.py; 2
// streams gain nothing on MI355X, 3-4 do).
#ifndef RT_SEQ_STREAMS
#define RT_SEQ_STREAMS 4
#endif
constexpr int kSeqSlots = RT_SEQ_STREAMS;
constexpr int kCbWordSets = 16;  // camera buffers per context: 1 + sequence slots (spare sets)

struct rt_ctx {
    int device = 0;
    // CPU backend (rt_create_cpu): no HIP object is ever made for it
    bool cpu = false;
    int cpu_threads = 0;
    void* cpu_scene = nullptr;
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
    // A camera buffer (rt_cambuf.h): per-tile lists for the camera of key,
    // built on the stream that needs it; the entry array's capacity comes
    // from the totals of earlier builds, read back without a host sync
    // (h_tot after ev_tot), and grows when a build needed more.
    struct CamBuf {
        float4* tcone = nullptr;
        unsigned* off = nullptr;
        unsigned* cur = nullptr;
        unsigned* flag = nullptr;
        int4* box = nullptr;        // n_tri triangle screen boxes
        unsigned* tcnt = nullptr;   // n_tri + 1 box sizes -> pair offsets
        unsigned long long* rmask = nullptr;  // pass mask per run of 64 candidate pairs
        size_t rcap = 0;            // runs rmask holds
        size_t observed_pairs = 0;  // largest candidate-pair count read back
        size_t built_cap = 0, built_rcap = 0;  // capacities of the last build (for its read-back)
        int* lng = nullptr;
        int* mid = nullptr;
        unsigned* stat = nullptr;
        void* scan = nullptr;
        int2* ent = nullptr;
        float4* rec = nullptr;      // inline records (RT_OPT_CB_INLINE_MAX_MB)
        size_t cap = 0, rec_cap = 0, scan_words = 0;
        int nt_alloc = 0, big_alloc = 0;
        unsigned long long* h_tot = nullptr;  // pinned: [total][stat words 0..7 as 4 u64]
        hipEvent_t ev_tot = nullptr, ev0 = nullptr, ev1 = nullptr;
        bool tot_pending = false;   // h_tot written by an enqueued copy not yet seen
        size_t observed = 0;        // largest total read back
        size_t entries = 0;         // last total read back
        unsigned hstat[8] = {};     // last stat words read back
        bool inline_rec = false;    // rec holds the current records
        int tiles_x = 0, ntiles = 0;
        float key[30] = {};
        bool valid = false;
        // a captured render references off / flag / ent / rec: the next
        // build writes fresh arrays (the captured ones are retired intact,
        // the capture-time lists that a replay reads)
        bool pinned = false;
        double host_ms = 0.0, build_ms = 0.0;
        bool timed = false;
    };
    CamBuf cb;
    // the last async frame's camera (cb_key_of): a repeat builds the sorted lists
    float last_async_key[30] = {};
    bool last_async_valid = false;
    // Camera state of rt_render_sequence_async: kSeqSlots slots of the
    // per-camera records and camera buffers, apart from the state above;
    // frame i of a sequence uses slot i % kSeqSlots on internal stream
    // i % kSeqSlots, so up to kSeqSlots consecutive frames (different
    // cameras) are in flight at once.
    struct CamSlot {
        float4 *tricam = nullptr, *cone_cam = nullptr, *clu_cam = nullptr, *uni = nullptr;
        CamBuf cb;
    } seq[kSeqSlots];
    hipStream_t seq_streams[kSeqSlots] = {};
    hipEvent_t seq_fork = nullptr, seq_join[kSeqSlots] = {};
    int n_cu = 0;
    std::vector<void*> deferred;  // replaced buffers an enqueued render may read: freed at the next host sync
    void* d_scan = nullptr;     // u64 scratch of the light-buffer build scans
    size_t scan_words = 0;
    unsigned long long* h_word = nullptr;  // pinned: totals read back by the builds
    unsigned long long* h_cbwords = nullptr;  // pinned: kCbWordSets x 8 words, one set per camera buffer
    int n_cbwords = 0;
    // light buffer (shadow cells), rt_lb_build
    unsigned* d_lb_off = nullptr;
    float4* d_lb_ent = nullptr;
    float4* d_lb_dcap = nullptr;
    float4* d_lb_meta = nullptr;
    bool lb_ready = false;
    int lb_levels = 0;  // buffers per light: slot = level * n_lights + light
    int lb_r0 = 0;      // light 0's first buffer's resolution (cells per face edge)
    size_t lb_entries = 0;
    double lb_build_ms = 0.0;
    float cam_key[3] = {0.f, 0.f, 0.f};
    bool cam_valid = false;
    // Tiny scenes (<= kTinyMax triangles, depth 0, light buffer): the camera
    // records are computed on the host per camera and passed with the launch
    // (rt_cull.h TinyCam) — host copies of the triangle records for that.
    std::vector<float4> h_tri, h_sph, h_nrm, h_coef;
    TinyCam tiny{};
    float tiny_key[30] = {};
    bool tiny_valid = false;
    bool opt_launch_camera = true;  // RT_OPT_LAUNCH_CAMERA
    struct MaskBuf {
        hipStream_t stream = nullptr;
        unsigned* d = nullptr;
        size_t cap = 0;
        float key[30] = {};   // the camera whose masks d holds (valid)
        bool valid = false;
        float pend[30] = {};  // the camera of the stream's last computing frame (pend_valid)
        bool pend_valid = false;
        // after the kernel that stored d (a reader on a stream that only
        // shares this one's handle — a destroyed stream's successor — waits)
        hipEvent_t ev = nullptr;
        bool ev_set = false;
        unsigned long long used = 0;  // last use (LRU eviction)
    };
    std::vector<MaskBuf> tiny_masks;  // per stream, at most kMaskBufs
    unsigned long long mask_clock = 0;
    bool tricam_all = false;  // tricam holds every triangle for cam_key
    StatsDev* d_stats = nullptr;
    void* d_scratch = nullptr;  // staging for host outputs
    size_t scratch_bytes = 0;
    // Ordering of the per-camera device state across streams (rt.h, ABI 4):
    // the streams that received rt_render_async work since the last host
    // sync of the context, and the stream + event of the last write of the
    // per-camera state not yet host-synced (an async camera prepass).
    std::vector<hipStream_t> async_streams;
    hipEvent_t ev_fence = nullptr, ev_state = nullptr;
    // synchronous renders into host memory: the slab in row chunks, each
    // copied over PCIe on copy_stream while the next one renders
    hipStream_t copy_stream = nullptr;
    hipEvent_t ev_chunk[8] = {};
    hipStream_t state_stream = nullptr;
    bool state_pending = false;
    bool captured = false;                // a render was captured into a hipGraph
    std::vector<void*> retired;           // buffers a captured render may reference
    // Options (rt_set_option; rt.h RT_OPT_*)
    int opt_light_buffer = 1;
    int opt_camera_buffer = 1;  // 0 off, 1 auto, 2 async builds for every frame
    bool opt_union = true;
    double opt_lb_scale = 0.0;
    double opt_dcov_near = 0.0;
    double opt_cb_inline_mb = 0.0;
    double opt_host_chunk_mb = 8.0;
    double opt_cb_capacity = 0.0;  // camera-buffer entries; 0 = automatic
    std::vector<double> far_ladder;       // big lists' far light buffers
    double upload_parts_ms[4] = {0, 0, 0, 0};  // copy+records, prepasses, light buffer, total
    double lb_parts_ms[5] = {0, 0, 0, 0, 0};    // lb_build phases (rt_debug_upload_info out[4..8])
    int n_surf = 0, n_lights = 0;
    int n_tri = 0, n_plane = 0, n_quad = 0;
    int n_tri_opaque = 0, n_plane_opaque = 0, n_quad_opaque = 0, n_translucent = 0;
    int shadow_split = 0;
    float k_max = 0.0f;         // max(Kr, Kt) over surfaces (NaN ignored)
    // bounce-ray BVH (rt_bvh.h, built at upload for scenes that can bounce)
    float4* d_bvh_node = nullptr;
    float4* d_bvh_tri = nullptr;
    // per surface: its coherence-sort bin (WfDev::skey; triangles in the
    // BVH's leaf order, two per bin), and the bins per branch
    unsigned* d_skey = nullptr;
    unsigned nbin_half = 0;
    int bvh_inner = 0, bvh_leaves = 0, bvh_depth = 0;
    double bvh_build_ms = 0.0;
    bool opt_bvh = true;        // RT_OPT_BVH
    // Wavefront bounce queues (rt_wavefront.h), grown on demand; one set per
    // context: a wavefront frame on another stream than the last one's waits
    // for that frame (ev_wf) before it reuses them.
    struct WfBuf {
        void* mem = nullptr;      // one allocation: counters, then every level's arrays
        size_t bytes = 0;
        size_t px = 0;            // pixel capacity (level-0 nodes)
        size_t cap[kWfMaxLevels + 1] = {};   // ray slots per level (level 0: pixels)
        size_t pcap[kWfMaxLevels + 1] = {};  // parent-list slots per level
        WfDev dev{};
        // coherence sort (WfDev::kin): bins of `kcap` ray slots, sorted
        // slots, the bin counts / positions (hcap words) and their scan's
        // scratch
        unsigned *kin = nullptr, *kout = nullptr, *kout2 = nullptr, *hist = nullptr;
        unsigned long long* bsum = nullptr;
        size_t kcap = 0, hcap = 0;
        int sort = 0;  // this frame's RT_OPT_WF_SORT: bit 0 parent sort, bit 1 hit sort (bit 2: by light cell)
        hipEvent_t ev = nullptr;  // after the last wavefront frame
        hipStream_t st2 = nullptr;               // RT_OPT_WF_OVERLAP: the stragglers' stream
        hipEvent_t ev_t = nullptr, ev_s = nullptr;  // fork (after the trace) / join (after the stragglers' shading)
        hipStream_t last = nullptr;
        bool pending = false;
    } wf;
    int opt_wavefront = 1;      // RT_OPT_WAVEFRONT
    int opt_wf_sort = 1;        // RT_OPT_WF_SORT
    bool opt_wf_overlap = true; // RT_OPT_WF_OVERLAP
    int opt_xcd_deal = 1;       // RT_OPT_XCD_DEAL
    int opt_xcd_stripe = 0;     // RT_OPT_XCD_STRIPE
    bool opt_lb_unroll = true;  // RT_OPT_LB_UNROLL
    float kr_max = 0.0f, kt_max = 0.0f;  // max Kr, max Kt over surfaces
    bool uploaded = false;
    rt_stats last{};
    std::string err;
};

static void cb_free(rt_ctx::CamBuf& B);

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
    HIP_TRY(c, hipEventCreateWithFlags(&c->ev_fence, hipEventDisableTiming));
    HIP_TRY(c, hipEventCreateWithFlags(&c->ev_state, hipEventDisableTiming));
    HIP_TRY(c, hipStreamCreateWithFlags(&c->copy_stream, hipStreamNonBlocking));
    for (hipEvent_t& e : c->ev_chunk) HIP_TRY(c, hipEventCreateWithFlags(&e, hipEventDisableTiming));
    HIP_TRY(c, hipHostMalloc((void**)&c->h_word, 2 * sizeof(unsigned long long), hipHostMallocDefault));
    HIP_TRY(c, hipHostMalloc((void**)&c->h_cbwords, kCbWordSets * 8 * sizeof(unsigned long long), hipHostMallocDefault));
    HIP_TRY(c, hipMalloc(&c->d_stats, kStatSlots * sizeof(StatsDev)));
    HIP_TRY(c, hipDeviceGetAttribute(&c->n_cu, hipDeviceAttributeMultiprocessorCount, dev));
    c->far_ladder = {2.5, 6.0, 16.0, 64.0};
    return RT_OK;
}

// Free now, or — once a render was captured into a hipGraph — keep until
// rt_upload_scene / rt_destroy (a replay may still reference it).
static void release(rt_ctx* c, void* p)
{
    if (!p) return;
    if (c->captured)
        c->retired.push_back(p);
    else
        hipFree(p);
}

static void free_retired(rt_ctx* c)
{
    for (void* p : c->retired) hipFree(p);
    c->retired.clear();
    c->captured = false;
}

// ---- ordering of the per-camera state across streams (rt.h, ABI 4)
// Make stream w wait for everything already enqueued on the streams that
// received async renders (they may read the state w is about to rewrite).
static int fence_async(rt_ctx* c, hipStream_t w)
{
    for (hipStream_t s : c->async_streams) {
        if (s == w) continue;
        HIP_TRY(c, hipEventRecord(c->ev_fence, s));
        HIP_TRY(c, hipStreamWaitEvent(w, c->ev_fence, 0));
    }
    return RT_OK;
}

// A reader on stream r of state written on another stream and not yet
// host-synced waits for that write.
static int wait_state(rt_ctx* c, hipStream_t r)
{
    if (c->state_pending && c->state_stream != r) HIP_TRY(c, hipStreamWaitEvent(r, c->ev_state, 0));
    return RT_OK;
}

static void note_async(rt_ctx* c, hipStream_t s)
{
    if (std::find(c->async_streams.begin(), c->async_streams.end(), s) == c->async_streams.end())
        c->async_streams.push_back(s);
}

// Buffers replaced while renders that read them may still have been in
// flight (free_later): after a host sync of everything nothing reads them.
// The internal sequence streams are joined into the caller's stream, which
// is one of the synced async streams.
static void free_deferred(rt_ctx* c)
{
    for (void* p : c->deferred) hipFree(p);
    c->deferred.clear();
}

// Host sync of everything the context enqueued: afterwards no async render
// or state write is in flight.
static int sync_all(rt_ctx* c)
{
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    if (c->copy_stream) HIP_TRY(c, hipStreamSynchronize(c->copy_stream));
    for (hipStream_t s : c->async_streams) HIP_TRY(c, hipStreamSynchronize(s));
    c->async_streams.clear();
    c->state_pending = false;
    c->state_stream = nullptr;
    c->wf.pending = false;
    free_deferred(c);
    return RT_OK;
}

// Device scratch for the build scans (u64 words), grown on demand.
static int ensure_scan(rt_ctx* c, size_t words)
{
    if (c->scan_words >= words) return RT_OK;
    release(c, c->d_scan);
    c->d_scan = nullptr;
    c->scan_words = 0;
    HIP_TRY(c, hipMalloc(&c->d_scan, words * sizeof(unsigned long long)));
    c->scan_words = words;
    return RT_OK;
}

RT_EXPORT int rt_sync(rt_ctx* c)
{
    if (!c) return RT_E_ARG;
    if (c->cpu) return RT_OK;  // CPU renders are synchronous
    if (!c->stream) return RT_E_STATE;
    HIP_TRY(c, hipSetDevice(c->device));
    return sync_all(c);
}

RT_EXPORT int rt_set_option(rt_ctx* c, int32_t opt, double v)
{
    if (!c || !(v == v)) return RT_E_ARG;
    switch (opt) {
    case RT_OPT_LIGHT_BUFFER:
        if (v != 0 && v != 1 && v != 2) return RT_E_ARG;
        c->opt_light_buffer = (int)v;
        return RT_OK;
    case RT_OPT_CAMERA_BUFFER:
        if (v != 0 && v != 1 && v != 2) return RT_E_ARG;
        if ((int)v != c->opt_camera_buffer) c->cb.valid = false;
        c->opt_camera_buffer = (int)v;
        return RT_OK;
    case RT_OPT_UNION_PRETEST: c->opt_union = v != 0; return RT_OK;
    case RT_OPT_LB_SCALE:
        if (v < 0 || v > 1e6) return RT_E_ARG;
        c->opt_lb_scale = v;
        return RT_OK;
    case RT_OPT_DCOV_NEAR:
        if (v < 0 || (v > 0 && v < 1.0) || v > 1e6) return RT_E_ARG;
        c->opt_dcov_near = v;
        return RT_OK;
    case RT_OPT_CB_INLINE_MAX_MB:
        if (v < 0) return RT_E_ARG;
        // the layout is chosen at a camera-buffer build: rebuild at the next render
        if (v != c->opt_cb_inline_mb) c->cb.valid = false;
        c->opt_cb_inline_mb = v;
        return RT_OK;
    case RT_OPT_HOST_CHUNK_MB:
        if (v < 0) return RT_E_ARG;
        c->opt_host_chunk_mb = v;
        return RT_OK;
    case RT_OPT_LAUNCH_CAMERA: c->opt_launch_camera = v != 0; return RT_OK;
    case RT_OPT_BVH: c->opt_bvh = v != 0; return RT_OK;
    case RT_OPT_WAVEFRONT: c->opt_wavefront = v != 0; return RT_OK;
    case RT_OPT_WF_SORT:
        if (v < 0 || v > 7 || v != std::floor(v)) return RT_E_ARG;
        c->opt_wf_sort = (int)v;
        return RT_OK;
    case RT_OPT_WF_OVERLAP: c->opt_wf_overlap = v != 0; return RT_OK;
    case RT_OPT_XCD_DEAL:
        if (v != 0 && v != 1 && v != 2 && v != 3) return RT_E_ARG;
        c->opt_xcd_deal = (int)v;
        return RT_OK;
    case RT_OPT_LB_UNROLL: c->opt_lb_unroll = v != 0; return RT_OK;
    case RT_OPT_XCD_STRIPE:
        if (v < 0 || v > 4096 || v != std::floor(v)) return RT_E_ARG;
        c->opt_xcd_stripe = (int)v;
        return RT_OK;
    case RT_OPT_CB_CAPACITY:
        if (v < 0 || v > 4e9 || v != std::floor(v)) return RT_E_ARG;
        if (v != c->opt_cb_capacity) c->cb.valid = false;
        c->opt_cb_capacity = v;
        return RT_OK;
    default: return RT_E_ARG;
    }
}

RT_EXPORT int rt_get_option(rt_ctx* c, int32_t opt, double* v)
{
    if (!c || !v) return RT_E_ARG;
    switch (opt) {
    case RT_OPT_LIGHT_BUFFER: *v = c->opt_light_buffer; return RT_OK;
    case RT_OPT_CAMERA_BUFFER: *v = c->opt_camera_buffer; return RT_OK;
    case RT_OPT_UNION_PRETEST: *v = c->opt_union ? 1 : 0; return RT_OK;
    case RT_OPT_LB_SCALE: *v = c->opt_lb_scale; return RT_OK;
    case RT_OPT_DCOV_NEAR: *v = c->opt_dcov_near; return RT_OK;
    case RT_OPT_CB_INLINE_MAX_MB: *v = c->opt_cb_inline_mb; return RT_OK;
    case RT_OPT_HOST_CHUNK_MB: *v = c->opt_host_chunk_mb; return RT_OK;
    case RT_OPT_CB_CAPACITY: *v = c->opt_cb_capacity; return RT_OK;
    case RT_OPT_LAUNCH_CAMERA: *v = c->opt_launch_camera ? 1 : 0; return RT_OK;
    case RT_OPT_BVH: *v = c->opt_bvh ? 1 : 0; return RT_OK;
    case RT_OPT_WAVEFRONT: *v = c->opt_wavefront; return RT_OK;
    case RT_OPT_WF_SORT: *v = c->opt_wf_sort; return RT_OK;
    case RT_OPT_WF_OVERLAP: *v = c->opt_wf_overlap ? 1 : 0; return RT_OK;
    case RT_OPT_XCD_DEAL: *v = c->opt_xcd_deal; return RT_OK;
    case RT_OPT_XCD_STRIPE: *v = c->opt_xcd_stripe; return RT_OK;
    case RT_OPT_LB_UNROLL: *v = c->opt_lb_unroll ? 1 : 0; return RT_OK;
    default: return RT_E_ARG;
    }
}

RT_EXPORT int rt_set_far_ladder(rt_ctx* c, const double* f, int32_t n)
{
    if (!c || n > 8) return RT_E_ARG;
    if (n < 0) {
        if (f) return RT_E_ARG;
        c->far_ladder = {2.5, 6.0, 16.0, 64.0};
        return RT_OK;
    }
    if (n > 0 && !f) return RT_E_ARG;
    for (int i = 0; i < n; ++i)
        if (!(f[i] >= 1.0 && f[i] <= 1e6) || (i > 0 && !(f[i] > f[i - 1]))) return RT_E_ARG;
    c->far_ladder.assign(f, f + n);
    return RT_OK;
}

RT_EXPORT int rt_create_cpu(int32_t threads, rt_ctx** out)
{
    if (!out) return RT_E_ARG;
    rt_ctx* c = new rt_ctx();
    c->cpu = true;
    c->cpu_threads = threads;
    *out = c;
    return RT_OK;
}

// The HIP entry points refuse a CPU context (and the CPU ones a HIP context
// without a host scene): the backend is the caller's explicit choice.
static int not_cpu(rt_ctx* c)
{
    c->err = "a CPU context (rt_create_cpu) renders with rt_cpu_render / rt_cpu_render_float";
    return RT_E_STATE;
}

RT_EXPORT void rt_destroy(rt_ctx* c)
{
    if (!c) return;
    if (c->cpu) {
        cpu_free(c->cpu_scene);
        delete c;
        return;
    }
    if (c->stream) {
        (void)hipSetDevice(c->device);
        (void)sync_all(c);
    }
    free_retired(c);
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
    hipFree(c->d_bvh_node);
    hipFree(c->d_bvh_tri);
    hipFree(c->wf.mem);
    hipFree(c->wf.kin);
    hipFree(c->wf.kout);
    hipFree(c->wf.kout2);
    hipFree(c->wf.hist);
    hipFree(c->wf.bsum);
    hipFree(c->d_skey);
    if (c->wf.ev) hipEventDestroy(c->wf.ev);
    if (c->wf.ev_t) hipEventDestroy(c->wf.ev_t);
    if (c->wf.ev_s) hipEventDestroy(c->wf.ev_s);
    if (c->wf.st2) hipStreamDestroy(c->wf.st2);
    for (auto& q : c->tiny_masks) {
        hipFree(q.d);
        if (q.ev) hipEventDestroy(q.ev);
    }
    cb_free(c->cb);
    for (auto& q : c->seq) {
        hipFree(q.tricam);
        hipFree(q.cone_cam);
        hipFree(q.clu_cam);
        hipFree(q.uni);
        cb_free(q.cb);
    }
    hipFree(c->d_stats);
    hipFree(c->d_scratch);
    if (c->ev0) hipEventDestroy(c->ev0);
    if (c->ev1) hipEventDestroy(c->ev1);
    if (c->ev_fence) hipEventDestroy(c->ev_fence);
    if (c->ev_state) hipEventDestroy(c->ev_state);
    for (hipEvent_t e : c->ev_chunk)
        if (e) hipEventDestroy(e);
    if (c->copy_stream) hipStreamDestroy(c->copy_stream);
    for (int j = 0; j < kSeqSlots; ++j) {
        if (c->seq_streams[j]) hipStreamDestroy(c->seq_streams[j]);
        if (c->seq_join[j]) hipEventDestroy(c->seq_join[j]);
    }
    if (c->seq_fork) hipEventDestroy(c->seq_fork);
    if (c->h_word) hipHostFree(c->h_word);
    if (c->h_cbwords) hipHostFree(c->h_cbwords);
    hipFree(c->d_scan);
    if (c->stream) hipStreamDestroy(c->stream);
    delete c;
}

static bool nonneg_finite(float v) { return std::isfinite(v) && !std::signbit(v); }

#include "rt_bvhhost.h"
// Bounce rays walk the BVH (rt_bvh.h) in scenes of at least this many
// triangles (fewer: every triangle, by wave-uniform scalar loads).
#ifndef RT_BVH_MIN_TRIANGLES
#define RT_BVH_MIN_TRIANGLES 64
#endif

// 256 camera records = 16 KB, the scalar data cache.
static constexpr int kTricamMaxTriangles = 256;
#ifndef RT_EDGE_MAX_TRIANGLES
#define RT_EDGE_MAX_TRIANGLES 0x7fffffff  // every list size (SceneDev::use_edges)
#endif
static constexpr int kEdgeMaxTriangles = RT_EDGE_MAX_TRIANGLES;
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

// Light buffer of every light (shadow_opaque_lb, lb_cone): resolution from
// the median angular radius of the light's triangle cones (cell half-width
// ~ that radius), nearest-first cell lists built on the device in two
// levels (supercells of 16 x 16 cells, then cells), offsets by host scans.
// Shadow-ray culling covers rays up to dcov = F x the light's farthest
// triangle (the prepass sizes each pair's margin for it; lanes beyond take
// the next level, or the per-lane loop over every triangle).  Big lists: a
// ladder of buffers per light, F = 1.25 then far buffers at 2.5, 6, 16 and
// 64 — each level's cones only as wide as its distance needs (A/B: 1.5 / 4 /
// 16 / 64 against one buffer at 3 plus one at 64: C3 -10%, C5 -8.5%; this
// ladder against that one: C3 -2%, C5 -5%; a single buffer at 2
// without far levels was 120x slower: lanes beyond fell into the per-lane
// loop over 50k triangles; one buffer at 16 or 64 widens every cone: C3
// 2.3x / 8.8x slower).  Small lists (<= 1,024 triangles, no clusters, one
// level): F = RT_DCOV_FACTOR_SMALL — far ground-plane points then stay
// in the buffer (A/B against 4: 16 / 32 / 64 / 256 = C2 -8 / -10 / -11 /
// +1%, C4 -8 / -8 / -6 / +5%; C1 and the bounce scenes flat; re-tuned at the
// end of round 2: 24 against 32 C2 -2.5%, C4 -2.4%, 20 and 28 worse).
// RT_OPT_DCOV_NEAR and rt_set_far_ladder override the big-list ladder at
// upload (tests, A/B).
#ifndef RT_DCOV_FACTOR
#define RT_DCOV_FACTOR 1.25
#endif
#ifndef RT_DCOV_FACTOR_SMALL
#define RT_DCOV_FACTOR_SMALL 24.0
#endif
// Slots: one buffer per entry of `cones` (a light's cone records, built for
// the distance dcov[j]): the lights, then (big lists) their far buffers.
#ifndef RT_LB_RMIN
#define RT_LB_RMIN 128
#endif
static int lb_build(rt_ctx* c, int ntr, int n_opaque, const std::vector<const float4*>& cones,
                    const std::vector<double>& dcov)
{
    hipStream_t st = c->stream;
    const int nl = (int)cones.size();
    const auto t0 = std::chrono::steady_clock::now();
    auto tp = t0;
    auto mark = [&](int i) {
        const auto now = std::chrono::steady_clock::now();
        c->lb_parts_ms[i] = std::chrono::duration<double, std::milli>(now - tp).count();
        tp = now;
    };
    // cells of ~1/4 the median cone radius: best of 1-8 on C3 and C5; and
    // no coarser than 128 cells per face edge (small scenes: C2 -3.3%, C4
    // -2.5% against their 16-48, flat from 192 to 512).  An explicit
    // RT_OPT_LB_SCALE (A/B, the stress tests' coarse cells) sets R alone.
    // Big lists (the ladder): 1/6 of the median cone radius since the LDS
    // walks (round 2: C3 -4.5%, C5 -1.4% against 1/4, whose lists were
    // twice as long; 22 M -> 47 M entries and +24 ms of build at upload; 5
    // and 8 measured worse); small lists keep 4 (flat at C1/C2/C4).
    const bool scale_set = c->opt_lb_scale > 0.0;
    const double scale = scale_set ? c->opt_lb_scale : (ntr > kClusterMinTriangles ? 6.0 : 4.0);
    const int r_min = scale_set ? kLbGroup : RT_LB_RMIN;
    // Slot j's pieces in the concatenated device arrays: its triangles in
    // dmin order (perm) and its dcap list (dperm); its supercell counts /
    // offsets (nsup + 1 words from sob) and cell offsets (ncell + 1 words
    // from ob: the slot's lb_off) — each slot's last word stays 0 as a
    // count, so ONE exclusive scan over a whole array gives every slot its
    // absolute offsets, the last word its end.
    // Big slots (more than kLbHyperMin triangles) first filter their
    // triangles per block of kLbHyper x kLbHyper supercells (hob: that
    // level's counts / offsets, like sob).
    struct Slot {
        int R = 16;
        size_t perm0 = 0, nperm = 0, dperm0 = 0, ndperm = 0, sob = 0, ob = 0, hob = 0;
        unsigned nsup = 0, ncell = 0, nhyp = 0;
        int Gp = 0;
    };
    constexpr int kLbHyper = 4;
    constexpr size_t kLbHyperMin = 4096;
    std::vector<Slot> B((size_t)nl);
    std::vector<int> perm_all, dperm_all;
    size_t sob = 0, ob = 0, hob = 0;
    int* d_perm = nullptr;
    unsigned* d_soff = nullptr;
    int* d_slists = nullptr;
    unsigned* d_hoff = nullptr;
    int* d_hlists = nullptr;
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
        // 1. the cone records of every slot (c0, c1 per triangle): one sync
        std::vector<float4> h((size_t)nl * ntr * 2);
        for (int j = 0; j < nl; ++j)
            LB_TRY(hipMemcpyAsync(h.data() + (size_t)j * ntr * 2, cones[j], (size_t)ntr * 2 * sizeof(float4),
                                  hipMemcpyDeviceToHost, st));
        LB_TRY(hipStreamSynchronize(st));
        mark(0);
        // per slot on its own host thread (independent): cell resolution from
        // the median cone angle, the triangles in dmin order, the dcap list
        std::vector<std::vector<int>> perms((size_t)nl), dperms((size_t)nl);
        auto prep = [&](int j) {
            Slot& b = B[j];
            const float4* hj = h.data() + (size_t)j * ntr * 2;
            std::vector<double> T;
            std::vector<int>& perm = perms[j];
            std::vector<int>& dperm = dperms[j];
            for (int k = 0; k < n_opaque; ++k) {
                const float4 c0 = hj[2 * k], c1 = hj[2 * k + 1];
                if (c0.w > 0.0f && c0.w <= 1.0f) T.push_back(std::acos((double)c0.w));
                if (c0.w > 0.0f && c1.x < (float)dcov[j]) perm.push_back(k);
                if (!(c1.z >= (float)dcov[j])) dperm.push_back(k);
            }
            if (!T.empty()) {
                std::nth_element(T.begin(), T.begin() + T.size() / 2, T.end());
                const double med = std::max(T[T.size() / 2], 1e-4);
                b.R = (int)std::lround(scale / (kLbGroup * med)) * kLbGroup;
                b.R = std::min(1024, std::max(r_min, b.R));
            }
            std::sort(perm.begin(), perm.end(), [&](int x, int y) {
                return hj[2 * x + 1].x < hj[2 * y + 1].x || (hj[2 * x + 1].x == hj[2 * y + 1].x && x < y);
            });
            auto key = [&](int k) { const float z = hj[2 * k + 1].z; return z == z ? z : -INFINITY; };
            std::sort(dperm.begin(), dperm.end(),
                      [&](int x, int y) { return key(x) < key(y) || (key(x) == key(y) && x < y); });
        };
        if (nl > 1 && (size_t)n_opaque * nl > 20000) {
            std::vector<std::thread> th;
            for (int j = 0; j < nl; ++j) th.emplace_back(prep, j);
            for (auto& t : th) t.join();
        } else {
            for (int j = 0; j < nl; ++j) prep(j);
        }
        for (int j = 0; j < nl; ++j) {
            Slot& b = B[j];
            b.perm0 = perm_all.size();
            b.nperm = perms[j].size();
            perm_all.insert(perm_all.end(), perms[j].begin(), perms[j].end());
            b.dperm0 = dperm_all.size();
            b.ndperm = dperms[j].size();
            dperm_all.insert(dperm_all.end(), dperms[j].begin(), dperms[j].end());
            const unsigned G = (unsigned)(b.R / kLbGroup);
            b.nsup = 6u * G * G;
            b.ncell = 6u * (unsigned)b.R * (unsigned)b.R;
            b.sob = sob;
            sob += b.nsup + 1;
            b.ob = ob;
            ob += b.ncell + 1;
            if (b.nperm > kLbHyperMin) {
                b.Gp = (int)((G + kLbHyper - 1) / kLbHyper);
                b.nhyp = 6u * (unsigned)(b.Gp * b.Gp);
                b.hob = hob;
                hob += b.nhyp + 1;
            }
        }
        mark(1);
        // 2. device arrays; supercell lists (counts, scan, fill)
        const size_t np = perm_all.size() + dperm_all.size();
        LB_TRY(hipMalloc(&d_perm, std::max<size_t>(np, 1) * sizeof(int)));
        if (!perm_all.empty())
            LB_TRY(hipMemcpyAsync(d_perm, perm_all.data(), perm_all.size() * sizeof(int), hipMemcpyHostToDevice, st));
        if (!dperm_all.empty())
            LB_TRY(hipMemcpyAsync(d_perm + perm_all.size(), dperm_all.data(), dperm_all.size() * sizeof(int),
                                  hipMemcpyHostToDevice, st));
        LB_TRY(hipMalloc(&d_soff, sob * sizeof(unsigned) + sizeof(unsigned)));
        LB_TRY(hipMalloc(&c->d_lb_off, ob * sizeof(unsigned) + sizeof(unsigned)));
        {
            const int src = ensure_scan(c, scan_scratch(std::max(std::max(sob, ob), hob)));
            if (src) {
                rc = src;
                goto done;
            }
        }
        LB_TRY(hipMemsetAsync(d_soff, 0, sob * sizeof(unsigned), st));
        LB_TRY(hipMemsetAsync(c->d_lb_off, 0, ob * sizeof(unsigned), st));
        unsigned long long* tot = nullptr;
        // 2a. the hyper level of the big slots (counts, scan, fill)
        if (hob > 0) {
            LB_TRY(hipMalloc(&d_hoff, hob * sizeof(unsigned) + sizeof(unsigned)));
            LB_TRY(hipMemsetAsync(d_hoff, 0, hob * sizeof(unsigned), st));
            for (int j = 0; j < nl; ++j) {
                const Slot& b = B[j];
                if (!b.nhyp) continue;
                hipLaunchKernelGGL(rt_lb_super, dim3(b.nhyp), dim3(256), 0, st, cones[j], ntr, d_perm + b.perm0,
                                   (int)b.nperm, b.R, (float)dcov[j], nullptr, d_hoff + b.hob, nullptr,
                                   kLbGroup * kLbHyper, b.Gp, 2e-3, nullptr, nullptr, 1, 1);
                LB_TRY(hipGetLastError());
            }
            LB_TRY(scan_u32(d_hoff, (unsigned)hob, d_hoff, (unsigned long long*)c->d_scan, st, &tot));
            LB_TRY(hipMemcpyAsync(c->h_word, tot, sizeof(unsigned long long), hipMemcpyDeviceToHost, st));
            LB_TRY(hipStreamSynchronize(st));
            const unsigned long long nhl = *c->h_word;
            if (nhl > 0xFFFFFFF0ull) {
                c->err = "light buffer too large";
                goto done;
            }
            LB_TRY(hipMalloc(&d_hlists, std::max<size_t>(nhl, 1) * sizeof(int)));
            for (int j = 0; j < nl; ++j) {
                const Slot& b = B[j];
                if (!b.nhyp) continue;
                hipLaunchKernelGGL(rt_lb_super, dim3(b.nhyp), dim3(256), 0, st, cones[j], ntr, d_perm + b.perm0,
                                   (int)b.nperm, b.R, (float)dcov[j], d_hoff + b.hob, nullptr, d_hlists,
                                   kLbGroup * kLbHyper, b.Gp, 2e-3, nullptr, nullptr, 1, 1);
                LB_TRY(hipGetLastError());
            }
        }
        // 2b. supercells: counts, scan, fill
        for (int j = 0; j < nl; ++j) {
            const Slot& b = B[j];
            hipLaunchKernelGGL(rt_lb_super, dim3(b.nsup), dim3(256), 0, st, cones[j], ntr, d_perm + b.perm0,
                               (int)b.nperm, b.R, (float)dcov[j], nullptr, d_soff + b.sob, nullptr, kLbGroup,
                               b.R / kLbGroup, 1e-3, b.nhyp ? d_hoff + b.hob : nullptr, d_hlists, kLbHyper, b.Gp);
            LB_TRY(hipGetLastError());
        }
        LB_TRY(scan_u32(d_soff, (unsigned)sob, d_soff, (unsigned long long*)c->d_scan, st, &tot));
        LB_TRY(hipMemcpyAsync(c->h_word, tot, sizeof(unsigned long long), hipMemcpyDeviceToHost, st));
        LB_TRY(hipStreamSynchronize(st));
        const unsigned long long nsl = *c->h_word;
        mark(2);
        if (nsl > 0xFFFFFFF0ull) {
            c->err = "light buffer too large";
            goto done;
        }
        LB_TRY(hipMalloc(&d_slists, std::max<size_t>(nsl, 1) * sizeof(int)));
        for (int j = 0; j < nl; ++j) {
            const Slot& b = B[j];
            hipLaunchKernelGGL(rt_lb_super, dim3(b.nsup), dim3(256), 0, st, cones[j], ntr, d_perm + b.perm0,
                               (int)b.nperm, b.R, (float)dcov[j], d_soff + b.sob, nullptr, d_slists, kLbGroup,
                               b.R / kLbGroup, 1e-3, b.nhyp ? d_hoff + b.hob : nullptr, d_hlists, kLbHyper, b.Gp);
            LB_TRY(hipGetLastError());
        }
        // 3. cell lists (counts, scan into lb_off, fill) and the dcap lists
        for (int j = 0; j < nl; ++j) {
            const Slot& b = B[j];
            hipLaunchKernelGGL(rt_lb_cells, dim3(b.nsup), dim3(256), 0, st, cones[j], ntr, c->d_tri, b.R,
                               (float)dcov[j], d_soff + b.sob, d_slists, nullptr, c->d_lb_off + b.ob, nullptr);
            LB_TRY(hipGetLastError());
        }
        LB_TRY(scan_u32(c->d_lb_off, (unsigned)ob, c->d_lb_off, (unsigned long long*)c->d_scan, st, &tot));
        LB_TRY(hipMemcpyAsync(c->h_word, tot, sizeof(unsigned long long), hipMemcpyDeviceToHost, st));
        LB_TRY(hipStreamSynchronize(st));
        const unsigned long long total = *c->h_word;
        mark(3);
        if (total >= 0xFFFFFFF0ull / 4) {  // entry indices are 32-bit
            c->err = "light buffer too large";
            goto done;
        }
        LB_TRY(hipMalloc(&c->d_lb_ent, std::max<size_t>(total, 1) * kLbEntF * sizeof(float)));
        LB_TRY(hipMalloc(&c->d_lb_dcap, std::max<size_t>(dperm_all.size(), 1) * kLbEntF * sizeof(float)));
        LB_TRY(hipMalloc(&c->d_lb_meta, std::max(nl, 1) * 2 * sizeof(float4)));
        std::vector<float4> meta((size_t)std::max(nl, 1) * 2);
        for (int j = 0; j < nl; ++j) {
            const Slot& b = B[j];
            hipLaunchKernelGGL(rt_lb_cells, dim3(b.nsup), dim3(256), 0, st, cones[j], ntr, c->d_tri, b.R,
                               (float)dcov[j], d_soff + b.sob, d_slists, c->d_lb_off + b.ob, nullptr, (float*)c->d_lb_ent);
            LB_TRY(hipGetLastError());
            if (b.ndperm) {
                hipLaunchKernelGGL(rt_lb_dcap, dim3((unsigned)((b.ndperm + 255) / 256)), dim3(256), 0, st, cones[j],
                                   c->d_tri, d_perm + perm_all.size() + b.dperm0, (int)b.ndperm,
                                   (float*)c->d_lb_dcap + kLbEntF * b.dperm0);
                LB_TRY(hipGetLastError());
            }
            unsigned obj = (unsigned)b.ob, db = (unsigned)b.dperm0, nd = (unsigned)b.ndperm;
            float4 m0, m1 = make_float4((float)dcov[j], 0.f, 0.f, 0.f);
            std::memcpy(&m0.x, &obj, 4);
            std::memcpy(&m0.y, &db, 4);
            std::memcpy(&m0.z, &nd, 4);
            std::memcpy(&m0.w, &b.R, 4);
            if (j == 0) c->lb_r0 = b.R;
            meta[2 * j] = m0;
            meta[2 * j + 1] = m1;
        }
        LB_TRY(hipMemcpyAsync(c->d_lb_meta, meta.data(), meta.size() * sizeof(float4), hipMemcpyHostToDevice, st));
        LB_TRY(hipStreamSynchronize(st));  // meta (host) outlives the copy; the temporaries are freed below
        mark(4);
        c->lb_ready = true;
        c->lb_entries = total;
    }
done:
#undef LB_TRY
    if (rc != RT_OK || !c->lb_ready) (void)hipStreamSynchronize(st);
    hipFree(d_slists);
    hipFree(d_soff);
    hipFree(d_hlists);
    hipFree(d_hoff);
    hipFree(d_perm);
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
    if (c->cpu) {
        c->uploaded = false;
        const int rc = cpu_upload(&c->cpu_scene, s);
        if (rc) {
            c->err = "unknown surface type";
            return rc;
        }
        c->n_surf = s->n_surfaces;
        c->n_lights = s->n_lights;
        c->uploaded = true;
        return RT_OK;
    }
    if (!c->stream) return RT_E_STATE;
    HIP_TRY(c, hipSetDevice(c->device));
    // nothing in flight may still read the buffers replaced below
    if (int rc = sync_all(c)) return rc;
    free_retired(c);
    const auto tu0 = std::chrono::steady_clock::now();
    auto since = [](std::chrono::steady_clock::time_point t) {
        return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t).count();
    };
    hipStream_t st = c->stream;
    const int n = s->n_surfaces, nl = s->n_lights;
    std::vector<float> geom((size_t)std::max(n, 1) * 16, 0.0f), mat((size_t)std::max(n, 1) * 12, 0.0f),
        lig((size_t)std::max(nl, 1) * 8, 0.0f);
    bool opaque = true;
    float kmax = 0.0f, krmax = 0.0f, ktmax = 0.0f;
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
        if (m[7] > krmax) krmax = m[7];
        if (m[8] > ktmax) ktmax = m[8];
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
    c->lb_levels = 0;
    c->lb_r0 = 0;
    c->lb_entries = 0;
    hipFree(c->d_uni);
    c->d_uni = nullptr;
    hipFree(c->d_bvh_node);
    hipFree(c->d_bvh_tri);
    hipFree(c->d_skey);
    c->d_bvh_node = c->d_bvh_tri = nullptr;
    c->d_skey = nullptr;
    c->nbin_half = 0;
    c->bvh_inner = c->bvh_leaves = c->bvh_depth = 0;
    c->bvh_build_ms = 0.0;
    c->cb.valid = false;  // buffers are kept (reallocated on demand)
    c->cam_valid = false;
    c->lb_build_ms = 0.0;
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
    // the bounce-ray BVH: only a scene with a reflective or refractive
    // surface has bounce rays (Scene.cpp:1779-1823 gate on Kr, Kt > 0)
    if (kmax > 0.0f && cnt_tri >= RT_BVH_MIN_TRIANGLES && (size_t)cnt_tri <= kBvhMaxTriangles) {
        const auto tb = std::chrono::steady_clock::now();
        BvhBuilt B;
        bvh_build(tri, (size_t)cnt_tri, B);
        if (B.depth <= kBvhStack) {
            HIP_TRY(c, up((void**)&c->d_bvh_node, B.nodes.data(), B.nodes.size() * sizeof(float4)));
            HIP_TRY(c, up((void**)&c->d_bvh_tri, B.tris.data(), B.tris.size() * sizeof(float4)));
            // the sort bins: triangle at leaf position p -> p / 2 (its
            // file index is the leaf record's third float4 .y), every other
            // surface a bin of its own after them
            std::vector<unsigned> skey((size_t)n, 0u);
            std::vector<char> is_tri((size_t)n, 0);
            for (int i = 0; i < cnt_tri; ++i) {
                int fi;
                std::memcpy(&fi, &B.tris[3 * (size_t)i + 2].y, sizeof fi);
                if (fi >= 0 && fi < n) {
                    skey[(size_t)fi] = (unsigned)i >> 1;
                    is_tri[(size_t)fi] = 1;
                }
            }
            unsigned nb = ((unsigned)cnt_tri + 1u) >> 1;
            for (int i = 0; i < n; ++i)
                if (!is_tri[(size_t)i]) skey[(size_t)i] = nb++;
            HIP_TRY(c, up((void**)&c->d_skey, skey.data(), skey.size() * sizeof(unsigned)));
            c->nbin_half = nb;
            c->bvh_inner = B.inner;
            c->bvh_leaves = B.leaves;
            c->bvh_depth = B.depth;
        }
        c->bvh_build_ms = since(tb);
    }
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
    c->tiny_valid = false;
    for (auto& q : c->tiny_masks) q.valid = q.pend_valid = false;  // the old scene's triangles
    if (ntr > 0 && ntr <= (size_t)kTinyMax) {  // the launch-camera path's host records
        auto f4 = [](const std::vector<float>& v, size_t n) {
            std::vector<float4> o(n);
            std::memcpy(o.data(), v.data(), n * sizeof(float4));
            return o;
        };
        c->h_tri = f4(tri, 3 * ntr);
        c->h_sph = f4(sph, ntr);
        c->h_nrm = f4(nrm, ntr);
        c->h_coef = f4(coef, ntr);
    } else {
        c->h_tri.clear();
        c->h_sph.clear();
        c->h_nrm.clear();
        c->h_coef.clear();
    }
    HIP_TRY(c, up((void**)&c->d_trisph, sph.data(), sph.size() * sizeof(float)));
    HIP_TRY(c, up((void**)&c->d_trinrm, nrm.data(), nrm.size() * sizeof(float)));
    HIP_TRY(c, up((void**)&c->d_tricoef, coef.data(), coef.size() * sizeof(float)));
    HIP_TRY(c, hipMalloc((void**)&c->d_cone_cam, std::max<size_t>(ntr, 1) * kConeRec * sizeof(float4)));
    HIP_TRY(c, hipMalloc((void**)&c->d_cone_light, std::max<size_t>(ntr * nl, 1) * kConeRec * sizeof(float4)));
    c->upload_parts_ms[0] = since(tu0);
    const auto tp0 = std::chrono::steady_clock::now();
    std::vector<double> lb_dcov((size_t)std::max(nl, 0), 0.0);
    // RT_OPT_DCOV_NEAR / rt_set_far_ladder override the big-list factors
    // (tests: force lanes into the far buffers and beyond them)
    const double fac_near = c->opt_dcov_near > 0.0 ? c->opt_dcov_near : RT_DCOV_FACTOR;
    const std::vector<double> fac_far = c->far_ladder;
    const double dfac = ntr > (size_t)kClusterMinTriangles ? fac_near : RT_DCOV_FACTOR_SMALL;
    for (int j = 0; j < nl && ntr > 0; ++j) {
        const float* l = s->lights + 7 * (size_t)j;
        // shadow rays are culled up to dfac x the light's farthest triangle
        double far = 0;
        for (size_t k = 0; k < ntr; ++k) {
            double d2 = 0;
            for (int a = 0; a < 3; ++a) d2 += ((double)sph[4 * k + a] - l[a]) * ((double)sph[4 * k + a] - l[a]);
            far = std::max(far, std::sqrt(d2) + sph[4 * k + 3]);
        }
        hipLaunchKernelGGL(rt_cone_prepass, dim3((unsigned)((ntr + 255) / 256)), dim3(256), 0, st, c->d_tri, c->d_trisph,
                           c->d_trinrm, c->d_tricoef, (int)ntr, l[0], l[1], l[2], 0, (float)(dfac * far),
                           c->d_cone_light + kConeRec * ntr * j, (float4*)nullptr);
        HIP_TRY(c, hipGetLastError());
        lb_dcov[j] = (double)(float)(dfac * far);
    }
    if (ntr > (size_t)kClusterMinTriangles) {
        c->n_clu = (int)((ntr + 63) / 64);
        HIP_TRY(c, hipMalloc((void**)&c->d_clu_cam, (size_t)c->n_clu * 4 * sizeof(float4)));
        HIP_TRY(c, hipMalloc((void**)&c->d_clu_light, std::max<size_t>((size_t)c->n_clu * nl, 1) * 2 * sizeof(float4)));
        for (int j = 0; j < nl; ++j) {
            hipLaunchKernelGGL(rt_cluster_prepass, dim3(cluster_blocks(c->n_clu)), dim3(256), 0, st,
                               c->d_cone_light + kConeRec * ntr * j, (int)ntr, c->n_clu,
                               c->d_clu_light + 2 * (size_t)c->n_clu * j, 64);
            HIP_TRY(c, hipGetLastError());
        }
    }
    if (ntr > 0 && ntr <= (size_t)kClusterMinTriangles) {
        // union records: [camera (filled when the camera is set)] [light 0] ...
        HIP_TRY(c, hipMalloc((void**)&c->d_uni, (size_t)(nl + 1) * 2 * sizeof(float4)));
        for (int j = 0; j < nl && n_tri_o > 0; ++j) {
            hipLaunchKernelGGL(rt_cluster_prepass, dim3(1), dim3(64), 0, st, c->d_cone_light + kConeRec * ntr * j,
                               n_tri_o, 1, c->d_uni + 2 * (1 + (size_t)j), n_tri_o);  // one wave
            HIP_TRY(c, hipGetLastError());
        }
        if (n_tri_o == 0) {  // no opaque triangle: nothing for shadow rays to walk ("never" record)
            std::vector<float4> nev((size_t)nl * 2);
            for (int j = 0; j < nl; ++j) {
                nev[2 * j] = make_float4(0.f, 0.f, 0.f, 2.0f);
                nev[2 * j + 1] = make_float4(INFINITY, 0.f, INFINITY, 0.f);
            }
            if (nl) HIP_TRY(c, hipMemcpyAsync(c->d_uni + 2, nev.data(), nev.size() * sizeof(float4), hipMemcpyHostToDevice, st));
            HIP_TRY(c, hipStreamSynchronize(st));  // nev outlives the copy
        }
    }
    // the sequence slots (rt_render_sequence_async): per-camera records of
    // their own; the union records' light part is the scene's
    for (auto& q : c->seq) {
        hipFree(q.tricam);
        hipFree(q.cone_cam);
        hipFree(q.clu_cam);
        hipFree(q.uni);
        const rt_ctx::CamBuf keep = q.cb;  // its buffers are kept (resized on demand)
        q = rt_ctx::CamSlot{};
        q.cb = keep;
        q.cb.valid = false;
        if (ntr == 0) continue;
        // every triangle's camera record: the camera-buffer walk reads them
        HIP_TRY(c, hipMalloc((void**)&q.tricam, ntr * 4 * sizeof(float4)));
        HIP_TRY(c, hipMalloc((void**)&q.cone_cam, ntr * kConeRec * sizeof(float4)));
        if (c->n_clu > 0) HIP_TRY(c, hipMalloc((void**)&q.clu_cam, (size_t)c->n_clu * 4 * sizeof(float4)));
        if (c->d_uni) {
            HIP_TRY(c, hipMalloc((void**)&q.uni, (size_t)(nl + 1) * 2 * sizeof(float4)));
            HIP_TRY(c, hipMemcpyAsync(q.uni, c->d_uni, (size_t)(nl + 1) * 2 * sizeof(float4), hipMemcpyDeviceToDevice, st));
        }
    }
    HIP_TRY(c, hipStreamSynchronize(st));
    c->upload_parts_ms[1] = since(tp0);
    const auto tl0 = std::chrono::steady_clock::now();
    const int lbm = c->opt_light_buffer;  // built only where launch() will use it
    if (ntr > 0 && nl > 0 && n_tri_o > 0 && opaque && (lbm == 1 || (lbm == 2 && ntr > (size_t)kClusterMinTriangles))) {
        std::vector<const float4*> cones;
        for (int j = 0; j < nl; ++j) cones.push_back(c->d_cone_light + kConeRec * ntr * j);
        std::vector<double> dcov = lb_dcov;
        // Big lists: a far buffer per light, its cone records built for
        // RT_DCOV_FACTOR_FAR x the farthest triangle, for the lanes beyond the
        // near buffer's dcov (else the per-lane loop over every triangle).
        // (one level per factor: slots level * n_lights + light)
        float4* d_cone_far = nullptr;
        const size_t nlev = ntr > (size_t)kClusterMinTriangles ? fac_far.size() : 0;
        if (nlev > 0) {
            HIP_TRY(c, hipMalloc((void**)&d_cone_far, nlev * ntr * nl * kConeRec * sizeof(float4)));
            for (size_t v = 0; v < nlev; ++v)
                for (int j = 0; j < nl; ++j) {
                    const float* l = s->lights + 7 * (size_t)j;
                    const double dfar = lb_dcov[j] / dfac * fac_far[v];
                    float4* out = d_cone_far + kConeRec * ntr * (v * nl + j);
                    hipLaunchKernelGGL(rt_cone_prepass, dim3((unsigned)((ntr + 255) / 256)), dim3(256), 0, st,
                                       c->d_tri, c->d_trisph, c->d_trinrm, c->d_tricoef, (int)ntr, l[0], l[1], l[2], 0,
                                       (float)dfar, out, (float4*)nullptr);
                    HIP_TRY(c, hipGetLastError());
                    cones.push_back(out);
                    dcov.push_back((double)(float)dfar);
                }
        }
        const int rc = lb_build(c, (int)ntr, n_tri_o, cones, dcov);
        hipFree(d_cone_far);
        if (rc) return rc;
        c->lb_levels = c->lb_ready ? 1 + (int)nlev : 0;
    }
    c->upload_parts_ms[2] = since(tl0);
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
    c->kr_max = krmax;
    c->kt_max = ktmax;
    c->uploaded = true;
    c->upload_parts_ms[3] = since(tu0);
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
// The trace kernel of a frame: its function, bounce-stack capacity (-1:
// none compiled), lights per shadow pass, dynamic LDS per workgroup, and its
// name (rt_stats.kernel).
struct KernelPick {
    kernel_fn k = nullptr;
    int cap = 0, lb = 1, wave = 0;
    unsigned lds = 0;
    char name[48] = {};
};
template <int MAXD, int LB, int WAVE, bool COUNT>
static KernelPick kpick(unsigned lds)
{
    KernelPick p;
    p.k = (kernel_fn)&rt_trace_kernel<MAXD, LB, WAVE, COUNT>;
    p.cap = MAXD;
    p.lb = LB;
    p.wave = WAVE;
    p.lds = lds;
    std::snprintf(p.name, sizeof p.name, "rt_trace_kernel<%d,%d,%d>", MAXD, LB, WAVE);
    return p;
}
// bvh: bounce rays through the BVH (depth > 0, the scene's BVH built, light
// buffer on): WAVE bit 256 with the depth-0 kernels' camera and shadow paths
// (camera buffer bit 8 — a no-op when S.cb_tiles_x is 0 —, light buffer bit
// 4, wave culling 1 or clustered 2); its waves carry the traversal stacks in
// LDS after the staging window.
// chain: no refracted ray can pass its gate (reflect-only scenes): the
// bounce kernels keep the chain in registers (WAVE bit 1024).
// small: a frame under 4 Mpx of output rows — the big-list kernel walks the
// light buffer's per-lane lists two entries per round (WAVE bit 2048,
// rt_shade.h lb_slot: its 8 x 8 tiles see more cells there than the staged
// walk takes; C3 -6%, and no gain at C5 for the registers it holds,
// profiles/r06/lbwalk/).
template <bool COUNT>
static KernelPick pick_kernel(int depth, int n_tri, int n_lights, bool lbuf, bool cbuf, int bvh_depth = 0,
                              bool chain = false, bool small = false)
{
    const bool bvh = bvh_depth > 0;
    const unsigned win = (unsigned)kLdsWaveBytes;
    if (depth == 0 && n_tri > 0 && lbuf) {  // light-buffer shadows, one light per pass
        if (n_tri > kClusterMinTriangles) {
            if (small) return cbuf ? kpick<0, 1, 2062, COUNT>(win) : kpick<0, 1, 2054, COUNT>(win);
            return cbuf ? kpick<0, 1, 14, COUNT>(win) : kpick<0, 1, 6, COUNT>(win);
        }
        return cbuf ? kpick<0, 1, 13, COUNT>(0) : kpick<0, 1, 5, COUNT>(0);
    }
    if (depth == 0 && n_tri > kClusterMinTriangles)
        return cbuf ? kpick<0, RT_WAVE_LB, 10, COUNT>(win) : kpick<0, RT_WAVE_LB, 2, COUNT>(win);
    if (depth == 0 && n_tri > 0)
        return cbuf ? kpick<0, RT_WAVE_LB, 9, COUNT>(0) : kpick<0, RT_WAVE_LB, 1, COUNT>(0);
    if (depth == 0 && n_lights > 1) return kpick<0, 3, 0, COUNT>(0);
    const unsigned bl = (unsigned)(kLdsWaveBytes + (size_t)bvh_depth * 64 * sizeof(int));
    if (bvh && lbuf && n_tri > 0) {
#define RT_PICK_BVH(N)                                                                                     \
    if (depth <= N) {                                                                                      \
        if (chain)                                                                                         \
            return n_tri > kClusterMinTriangles ? kpick<N, 1, 1294, COUNT>(bl) : kpick<N, 1, 1293, COUNT>(bl); \
        return n_tri > kClusterMinTriangles ? kpick<N, 1, 270, COUNT>(bl) : kpick<N, 1, 269, COUNT>(bl);   \
    }
        RT_STACK_DEPTHS(RT_PICK_BVH)
#undef RT_PICK_BVH
    }
#define RT_PICK(N) \
    if (depth <= N) return chain ? kpick<N, 1, 1024, COUNT>(0) : kpick<N, 1, 0, COUNT>(0);
    RT_STACK_DEPTHS(RT_PICK)
#undef RT_PICK
    KernelPick none;
    none.cap = -1;
    return none;
}

// Launch shape of a trace kernel over `rows` output rows: one 8 x 8 tile per
// workgroup, the kernel's dynamic LDS (the big-list kernels' staging
// windows, the BVH kernels' traversal stacks).
static void trace_dims(int width, int rows, dim3& grid, dim3& block)
{
    grid = dim3((width + 7) / 8, (rows + 7) / 8);
    block = dim3(64);
}

// The launch-camera kernel (tiny scenes: camera buffer replaced by the
// launch's records, light-buffer shadows, one light per pass); SELF: the
// camera's first frame on the stream, which computes and stores the masks.
template <bool COUNT>
static const void* tiny_kernel(int mode)
{
    return mode == 2   ? (const void*)&rt_trace_tiny<0, 1, 229, COUNT>
           : mode == 1 ? (const void*)&rt_trace_tiny<0, 1, 101, COUNT>
                       : (const void*)&rt_trace_tiny<0, 1, 37, COUNT>;
}

// One trace launch over `rows` output rows (T: the launch-camera kernel with
// its records, else kernel k).
static int launch_trace(rt_ctx* c, const KernelPick& kp, const TinyCam* T, bool count, SceneDev& S, FrameDev& F,
                        int width, int rows, unsigned* oa, float* ob, StatsDev* stats, hipStream_t st, int mode = 0)
{
    dim3 grid, block;
    trace_dims(width, rows, grid, block);
    F.tiles_x = (int)grid.x;
    F.tiles_y = (int)grid.y;
    F.xcd_mode = 1;
    F.xcd_w = 0;
    F.xcd_m = 0;
    if (!T && (kp.wave & 2) && c->opt_xcd_deal != 1) {
        // the big-list kernels' padded grids (tile_of_block)
        F.xcd_mode = c->opt_xcd_deal;
        if (c->opt_xcd_deal == 2) {
            const unsigned sw = c->opt_xcd_stripe > 0 ? (unsigned)c->opt_xcd_stripe : (grid.x + kXcds - 1) / kXcds;
            F.xcd_w = (int)sw;
            F.xcd_m = (int)((grid.x + kXcds * sw - 1) / (kXcds * sw) * sw);
            grid = dim3(kXcds * (unsigned)F.xcd_m, grid.y);
        } else if (c->opt_xcd_deal == 3) {
            const unsigned gx = (grid.x + 3) / 4, gy = (grid.y + 1) / 2;
            const unsigned nst = (gx * gy + kXcds - 1) / kXcds * kXcds;  // super-tiles, a multiple of 8
            F.xcd_w = (int)gx;
            grid = dim3(8, nst);
        }
    }
    if (T) {
        TinyCam Tv = *T;
        void* args[] = {&S, &F, &Tv, &oa, &ob, &stats};
        HIP_TRY(c, hipLaunchKernel(count ? tiny_kernel<true>(mode) : tiny_kernel<false>(mode), grid, block, args, 0, st));
        return RT_OK;
    }
    void* args[] = {&S, &F, &oa, &ob, &stats};
    HIP_TRY(c, hipLaunchKernel((const void*)kp.k, grid, block, args, kp.lds, st));
    return RT_OK;
}

// Output rows of a launch: the slab, or this rank's band set.
static int frame_rows(const rt_frame* f)
{
    if (f->band_rows != 0) return std::max(0, (int)rt_band_rows(f->height, f->band_rows, f->band_count, f->band_index));
    return f->row_end - f->row_begin;
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
    // the rows whose tiles have lists (a rank's slab or band set)
    const int32_t rows[5] = {f->band_rows ? 0 : f->row_begin, f->band_rows ? 0 : f->row_end, f->band_rows,
                             f->band_rows ? f->band_count : 0, f->band_rows ? f->band_index : 0};
    std::memcpy(key + 25, rows, sizeof rows);
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
    F.wf = WfDev{};
}

// Does frame f need the per-camera prepasses (the camera position moved)?
// A camera already prepared without every tricam record — a bounce frame
// of a big scene — is prepared again for the camera buffer.
static bool camera_needs_prepass(const rt_ctx* c, const rt_frame* f, bool all_tricam)
{
    return c->n_tri > 0 && !(c->cam_valid && std::memcmp(c->cam_key, f->cam_pos, sizeof c->cam_key) == 0 &&
                             (!all_tricam || c->tricam_all));
}

// The per-camera records of camera position cp into one set of buffers:
// camera-ray triangle values, camera cone records, union / cluster records.
static int camera_records(rt_ctx* c, const float* cp, hipStream_t st, bool all_tricam, float4* tricam,
                          float4* cone_cam, float4* uni, float4* clu_cam)
{
    float4* tc = (all_tricam || c->n_tri <= kTricamMaxTriangles) ? tricam : nullptr;
    if (uni && c->n_clu == 0 && c->n_tri <= kCameraSmallMax) {  // small lists: one launch
        hipLaunchKernelGGL(rt_camera_small, dim3(1), dim3(256), 0, st, c->d_tri, c->d_trisph, c->d_trinrm,
                           c->d_tricoef, c->n_tri, cp[0], cp[1], cp[2], cone_cam, tc, uni);
        HIP_TRY(c, hipGetLastError());
        return RT_OK;
    }
    hipLaunchKernelGGL(rt_cone_prepass, dim3((c->n_tri + 255) / 256), dim3(256), 0, st, c->d_tri, c->d_trisph,
                       c->d_trinrm, c->d_tricoef, c->n_tri, cp[0], cp[1], cp[2], 1, 0.0f, cone_cam, tc);
    HIP_TRY(c, hipGetLastError());
    if (uni) {
        hipLaunchKernelGGL(rt_cluster_prepass, dim3(1), dim3(64), 0, st, cone_cam, c->n_tri, 1, uni, c->n_tri);  // one wave
        HIP_TRY(c, hipGetLastError());
    }
    if (c->n_clu > 0) {
        float4* tmp = clu_cam + 2 * (size_t)c->n_clu;  // second half: unsorted
        hipLaunchKernelGGL(rt_cluster_prepass, dim3(cluster_blocks(c->n_clu)), dim3(256), 0, st, cone_cam,
                           c->n_tri, c->n_clu, tmp, 64);
        HIP_TRY(c, hipGetLastError());
        hipLaunchKernelGGL(rt_cluster_sort, dim3(cluster_blocks(c->n_clu)), dim3(256), 0, st, tmp,
                           c->n_clu, clu_cam);
        HIP_TRY(c, hipGetLastError());
    }
    return RT_OK;
}

// Per-camera prepasses (when the camera position moved), into the
// context's state.
static int camera_prepass(rt_ctx* c, const rt_frame* f, hipStream_t st, bool all_tricam)
{
    if (!camera_needs_prepass(c, f, all_tricam)) return RT_OK;
    if (int rc = camera_records(c, f->cam_pos, st, all_tricam, c->d_tricam, c->d_cone_cam, c->d_uni, c->d_clu_cam))
        return rc;
    std::memcpy(c->cam_key, f->cam_pos, sizeof c->cam_key);
    c->cam_valid = true;
    c->tricam_all = all_tricam || c->n_tri <= kTricamMaxTriangles;
    c->cb.valid = false;
    return RT_OK;
}

static SceneDev scene_dev(rt_ctx* c, bool lbuf, bool cbuf)
{
    const int use_tricam = c->n_tri > 0 && c->n_tri <= kTricamMaxTriangles;
    return SceneDev{c->d_geom, c->d_mat, c->d_lights, c->d_tri, c->d_plane, c->d_quad, c->d_translucent, c->d_tricam,
                    use_tricam, c->n_tri <= kEdgeMaxTriangles, c->d_cone_cam, c->d_cone_light, c->d_clu_cam,
                    c->d_clu_light, c->n_clu, c->n_surf, c->n_lights, c->n_tri, c->n_plane, c->n_quad,
                    c->n_tri_opaque, c->n_plane_opaque, c->n_quad_opaque, c->n_translucent, c->shadow_split,
                    lbuf ? c->lb_levels : 0, c->d_lb_off, c->d_lb_ent, c->d_lb_dcap, c->d_lb_meta,
                    (c->d_uni && c->opt_union) ? c->d_uni : nullptr,
                    c->cb.off, c->cb.ent, c->cb.flag, cbuf ? c->cb.tiles_x : 0,
                    c->cb.inline_rec ? c->cb.rec : nullptr, c->d_bvh_node, c->d_bvh_tri};
}

// The light buffer serves this context's shadow rays (RT_OPT_LIGHT_BUFFER).
static bool lbuf_on(const rt_ctx* c)
{
    const int mode = c->opt_light_buffer;
    return c->lb_ready && (mode == 1 || (mode == 2 && c->n_tri > kClusterMinTriangles));
}
// Bounce rays walk the BVH (rt_bvh.h) in the frame's kernel (the BVH kernels
// take their shadow rays through the light buffer).
static bool bvh_on(const rt_ctx* c, int depth, bool lbuf)
{
    return depth > 0 && c->d_bvh_node && c->opt_bvh && lbuf && c->n_tri > 0;
}
// No refracted ray can pass its gate (Scene.cpp:1791: Kt * energy >
// min_energy with every Kt <= 0 and min_energy >= 0): the bounce tree of
// every pixel is a chain of reflections.
static bool reflect_chain(const rt_ctx* c, const rt_frame* f) { return !(c->kt_max > 0.0f) && f->min_energy >= 0.0f; }
// The frame's camera rays may walk a camera buffer: the depth-0 kernels and
// the BVH kernels.
static bool cam_lists(const rt_ctx* c, int depth, bool lbuf) { return depth == 0 || bvh_on(c, depth, lbuf); }

#include "rt_camhost.h"

// Make the per-camera state current for frame f, ordered on stream st: the
// camera prepass when the camera moved, and the camera buffer when the
// frame's kernel uses one and it is not current.  sync_path: a synchronous
// call on c->stream (fenced behind every async render at its start).
// Async (round 3: the camera buffer too, no host sync): a write fences st
// behind the other streams' renders and marks the state as written on st;
// otherwise st waits for a pending write made on another stream.
// Capturing: nothing may be written (an unprepared camera is RT_E_STATE; a
// prepared camera whose buffer is not current renders without it).
static int prepare_state(rt_ctx* c, const rt_frame* f, hipStream_t st, bool sync_path, bool capturing, bool cb_want)
{
    if (capturing && c->state_pending && c->state_stream != st) {
        // a wait on an event recorded outside the capture cannot be captured
        c->err = "hipGraph capture: the camera state was written by an async render on another stream "
                 "(rt_sync or a synchronous render first)";
        return RT_E_STATE;
    }
    if (!sync_path && !capturing) {
        if (int rc = wait_state(c, st)) return rc;
    }
    if (!capturing) cb_harvest(c->cb);
    const bool need_prep = camera_needs_prepass(c, f, cb_want);
    // The camera buffer is built by a synchronous render, by an async frame
    // repeating the previous async frame's camera (round 4: a static camera
    // rendered async gets its lists at its second frame), and by a new
    // camera's async frame where the build pays (cb_async_pays).
    float key[30];
    cb_key_of(f, key);
    const bool repeat = !sync_path && c->last_async_valid && std::memcmp(key, c->last_async_key, sizeof key) == 0;
    if (!sync_path) {
        std::memcpy(c->last_async_key, key, sizeof key);
        c->last_async_valid = true;
    }
    const bool current = cb_matches(c->cb, f) && !need_prep;
    const bool need_cb = cb_want && !current && (sync_path || repeat || cb_async_pays(c, f));
    if (capturing) {
        if (need_prep) {
            c->err = "hipGraph capture: the frame's camera is not prepared (rt_render or rt_prepare_camera first)";
            return RT_E_STATE;
        }
        return RT_OK;
    }
    if (!need_prep && !need_cb) return RT_OK;
    if (!sync_path) {
        if (int rc = fence_async(c, st)) return rc;
    }
    if (need_prep) {
        if (int rc = camera_prepass(c, f, st, cb_want)) return rc;
    }
    if (need_cb) {
        const SceneDev S = scene_dev(c, false, false);
        if (int rc = cb_build(c, c->cb, f, S, st, sync_path, false, true)) return rc;
    }
    if (!sync_path) {
        HIP_TRY(c, hipEventRecord(c->ev_state, st));
        c->state_stream = st;
        c->state_pending = true;
    }
    return RT_OK;
}

// sync_path: rt_render / rt_render_float on c->stream; else rt_render_async
// on the caller's stream (both build the camera buffer when it is not current).
// host_out (synchronous renders into host memory): the output is copied
// there — for a big slab in up to 8 row chunks (multiples of 16 rows, one
// per RT_OPT_HOST_CHUNK_MB of output), chunk i's copy on c->copy_stream
// overlapping chunk i + 1's kernel (the same pixels: every pixel is independent, and the chunks keep
// the unchunked launch's 8-row wave rows).
// ---- wavefront bounce levels (rt_wavefront.h)
// Children one node can spawn (the gates compare K * energy > min_energy,
// Scene.cpp:1780,1791): with min_energy >= 0 a reflected ray needs some
// Kr > 0 and a refracted one some Kt > 0; a negative (or NaN) threshold is
// passed by K = 0 too, so every node may spawn both.
static int wf_branch(const rt_ctx* c, const rt_frame* f)
{
    if (!(f->min_energy >= 0.0f)) return 2;
    return (c->kr_max > 0.0f ? 1 : 0) + (c->kt_max > 0.0f ? 1 : 0);
}

#ifndef RT_WF_TRACE_WAVES
// trace launch: workgroups (one wave each) per CU.  Fewer than the 32 that
// fit (59 VGPRs, depth x 256 B of LDS) run faster: c3r 3.447 / 3.359 / 3.355
// / 3.338 ms at 32 / 24 / 20 / 16, c5r 21.23 / 21.16 / 21.26 / 21.59
// (profiles/r05/sorder/ab_trace_waves.log)
#define RT_WF_TRACE_WAVES 24
#endif
// Steps a lane's walk may take in the trace launch before the straggler
// launch finishes it with a whole wave.  Small levels (under
// RT_WF_BUDGET_SPLIT ray slots, ~2 rays per lane) are dominated by the trace
// launch's tail of long walks and hand off early; big ones (tens of rays
// per lane) hide that tail and keep more walks on the lanes.  Measured
// (profiles/r05/sorder/ab_budget.log): c3r (2.1 M slots) 2.944 / 2.973 /
// 2.983 ms at 128 / 112 / 160; c5r (33 M) 19.17 / 18.97 / 18.97 at 256 /
// 320 / 384.
#ifndef RT_WF_BUDGET_SMALL
#define RT_WF_BUDGET_SMALL 128
#endif
#ifndef RT_WF_BUDGET_BIG
#define RT_WF_BUDGET_BIG 320
#endif
#ifndef RT_WF_BUDGET_SPLIT
#define RT_WF_BUDGET_SPLIT (6u << 20)
#endif
#ifndef RT_WF_STRAG_WAVES
// straggler launch: workgroups (one wave, one straggling ray at a time, its
// kWfStragCap-entry LDS stack) per CU: 4 / 8 / 16 waves of 16 / 16 / 8 KB,
// c3r 3.359 / 3.273 / 3.249 ms, c5r 21.13 / 19.80 / 19.19
// (profiles/r05/sorder/ab_straggle*.log); round 6, with the sorted levels:
// 32 waves of 4 KB against 16 of 8 KB, c3r 2.862 / 2.887, c5r 17.65 / 17.77
// (profiles/r06/knobs/)
#define RT_WF_STRAG_WAVES 32
#endif
#ifndef RT_WF_FOLD_BLOCKS
#define RT_WF_FOLD_BLOCKS 64  // fold launch: 256-thread blocks per CU (4: c5r +0.5%, profiles/r06/knobs2/)
#endif
#ifndef RT_WF_SHADE_WAVES
#define RT_WF_SHADE_WAVES 24  // shade launch: workgroups (one wave each) per CU (= its occupancy)
#endif
#ifndef RT_WF_SORT
// each level's rays sorted by their parent surface's bin (BVH leaf order)
// and branch before its trace (rt_wf_sort_*), for frames whose level-1
// queue holds at least this many ray slots (0: every wavefront frame).
// Round 5's hipcub radix sort ran over the queue's capacity (+6% at c3r,
// -6% at c5r, profiles/r05/wfsort/); the counting sort reads only the
// level's live rays.
#define RT_WF_SORT 0
#endif
#ifndef RT_WF_MAX_GB
#define RT_WF_MAX_GB 32.0
#endif
// The queues' layout for a frame of `tiles` level-0 tiles (one wave each)
// over px pixels, `levels` bounce levels, `branch` children per node at most
// (rt_layout.h WfDev): segment capacities that no wave's appends can
// overflow — segment s of level L + 1 receives the children of level L's
// chunks c = s (mod kWfSeg), at most 64 * branch each — then the bytes:
// counters; level-0 node records (32 B) per pixel and its parent list;
// per level L >= 1 the rays (32 B), colours (16 B) and, but for the deepest
// level, node records (32 B) and the parent list; the hit records (8 B),
// straggler queue (16 B) and stragglers' minima (8 B) of the largest level.
struct WfLayout {
    size_t cap[kWfMaxLevels + 1] = {}, pcap[kWfMaxLevels + 1] = {};
    unsigned seg[kWfMaxLevels + 1] = {}, pseg[kWfMaxLevels + 1] = {};
    size_t most = 0, bytes = 0;
};
static WfLayout wf_layout(size_t tiles, size_t px, int levels, int branch)
{
    WfLayout w;
    auto up = [](size_t a, size_t b) { return (a + b - 1) / b; };
    size_t chunks = tiles;
    for (int L = 0; L <= levels; ++L) {
        if (L > 0) {
            w.seg[L] = (unsigned)(up(chunks, kWfSeg) * 64 * (size_t)branch);
            w.cap[L] = (size_t)kWfSeg * w.seg[L];
            chunks = up(w.cap[L], 64);
            w.most = std::max(w.most, w.cap[L]);
        }
        if (L < levels) {
            w.pseg[L] = (unsigned)(up(chunks, kWfSeg) * 64);
            w.pcap[L] = (size_t)kWfSeg * w.pseg[L];
        }
    }
    auto a = [](size_t x) { return (x + 255) & ~(size_t)255; };
    size_t tot = a(kWfCountBytes) + a(px * 32) + a(w.pcap[0] * 4);
    for (int L = 1; L <= levels; ++L) {
        tot += a(w.cap[L] * 32) + a(w.cap[L] * 16);
        if (L < levels) tot += a(w.cap[L] * 32) + a(w.pcap[L] * 4);
    }
    w.bytes = tot + a(w.most * 8) + a(w.most * 16) + a(w.most * 8);  // hit, strag, hit2
    return w;
}

static size_t frame_tiles(const rt_frame* f, int rows) { return (size_t)((f->width + 7) / 8) * (size_t)((rows + 7) / 8); }

// Would frame f (depth `depth`, its kernel a BVH kernel) render as a
// wavefront?  RT_OPT_WAVEFRONT, at most kWfMaxLevels levels, a single
// output chunk, queues within RT_WF_MAX_GB.
static bool wf_fits(const rt_ctx* c, const rt_frame* f, int depth, int rows)
{
    if (!c->opt_wavefront || depth < 1 || depth > kWfMaxLevels || wf_branch(c, f) == 0) return false;
    const WfLayout w = wf_layout(frame_tiles(f, rows), (size_t)rows * f->width, depth, wf_branch(c, f));
    return (double)w.bytes <= RT_WF_MAX_GB * 1073741824.0;
}

// The queues for frame f (grown, never shrunk; not while capturing).
// Fills c->wf.dev.
static int wf_ensure(rt_ctx* c, const rt_frame* f, int rows, int levels, bool capturing, bool* ok)
{
    rt_ctx::WfBuf& W = c->wf;
    const size_t px = (size_t)rows * f->width;
    const WfLayout w = wf_layout(frame_tiles(f, rows), px, levels, wf_branch(c, f));
    *ok = false;
    if (w.bytes > W.bytes) {
        if (capturing) return RT_OK;  // (the frame renders by the BVH megakernel)
        free_later(c, W.mem);  // an enqueued frame may still use the old queues
        W.mem = nullptr;
        W.bytes = 0;
        HIP_TRY(c, hipMalloc(&W.mem, w.bytes));
        W.bytes = w.bytes;
    }
    if (!W.ev) HIP_TRY(c, hipEventCreateWithFlags(&W.ev, hipEventDisableTiming));
    char* p = (char*)W.mem;
    auto take = [&](size_t bytes) {
        char* q = p;
        p += (bytes + 255) & ~(size_t)255;
        return q;
    };
    WfDev& d = W.dev;
    d = WfDev{};
    d.count = (unsigned*)take(kWfCountBytes);
    d.node[0] = (float4*)take(px * 32);
    d.plist[0] = (unsigned*)take(w.pcap[0] * 4);
    d.pseg[0] = w.pseg[0];
    for (int L = 1; L <= levels; ++L) {
        d.ray[L] = (float4*)take(w.cap[L] * 32);
        d.res[L] = (float4*)take(w.cap[L] * 16);
        d.seg[L] = w.seg[L];
        if (L < levels) {
            d.node[L] = (float4*)take(w.cap[L] * 32);
            d.plist[L] = (unsigned*)take(w.pcap[L] * 4);
            d.pseg[L] = w.pseg[L];
        }
    }
    d.hit = (float2*)take(w.most * 8);
    d.strag = (int4*)take(w.most * 16);
    d.hit2 = (float2*)take(w.most * 8);
    d.levels = levels;
    d.kin = nullptr;
    d.kout = nullptr;
    d.skey = c->d_skey;
    d.hist = nullptr;
    d.nbin_half = c->nbin_half;
    W.sort = 0;
    if (c->d_skey && c->opt_wf_sort && levels >= 1 && w.cap[1] >= (size_t)RT_WF_SORT) {
        if (w.most > W.kcap) {
            free_later(c, W.kin);
            free_later(c, W.kout);
            free_later(c, W.kout2);
            W.kin = W.kout = W.kout2 = nullptr;
            W.kcap = 0;
            HIP_TRY(c, hipMalloc((void**)&W.kin, w.most * sizeof(unsigned)));
            HIP_TRY(c, hipMalloc((void**)&W.kout, w.most * sizeof(unsigned)));
            HIP_TRY(c, hipMalloc((void**)&W.kout2, w.most * sizeof(unsigned)));
            W.kcap = w.most;
        }
        // (the hit sort's bins: nbin_half + kWfMissBins)
        size_t bins = std::max(2 * (size_t)c->nbin_half, (size_t)c->nbin_half + kWfMissBins);
        if ((c->opt_wf_sort & 4) && c->lb_r0 > 0)  // the light-cell hit sort's bins
            bins = std::max(bins, 6 * (size_t)c->lb_r0 * (size_t)c->lb_r0 + kWfMissBins);
        if (bins + 1 > W.hcap) {
            free_later(c, W.hist);
            free_later(c, W.bsum);
            W.hist = nullptr;
            W.bsum = nullptr;
            W.hcap = 0;
            // the parent counts (hist), the hit counts, the scan's positions
            // (next): bins + 1 words each
            HIP_TRY(c, hipMalloc((void**)&W.hist, 3 * (bins + 1) * sizeof(unsigned)));
            HIP_TRY(c, hipMalloc((void**)&W.bsum, scan_scratch(bins) * sizeof(unsigned long long)));
            W.hcap = bins + 1;
        }
        W.sort = c->opt_wf_sort;
        if (W.sort & 1) d.kin = W.kin;
        d.hist = W.hist;
    }
    for (int L = 0; L <= levels; ++L) {
        W.cap[L] = L == 0 ? px : w.cap[L];
        W.pcap[L] = w.pcap[L];
    }
    W.px = px;
    *ok = true;
    return RT_OK;
}

// Level 0 of a wavefront frame: the depth-0 kernel with WAVE bit 512.
template <bool COUNT>
static KernelPick pick_wf0(int n_tri, bool cbuf, bool small = false)
{
    const unsigned win = (unsigned)kLdsWaveBytes;
    if (n_tri > kClusterMinTriangles && small)  // (the two-entry light-buffer walk, pick_kernel)
        return cbuf ? kpick<0, 1, 2574, COUNT>(win) : kpick<0, 1, 2566, COUNT>(win);
    if (n_tri > kClusterMinTriangles)
        return cbuf ? kpick<0, 1, 526, COUNT>(win) : kpick<0, 1, 518, COUNT>(win);
    return cbuf ? kpick<0, 1, 525, COUNT>(0) : kpick<0, 1, 517, COUNT>(0);
}

static bool W_px_small(const rt_ctx* c) { return (double)c->wf.px < 4e6; }

// The bounce levels and folds of a wavefront frame, after level 0 on st:
// per level a trace launch (the BVH walk; LDS = its stack) and a shade
// launch (LDS = the light-buffer staging window), then the folds.
static int wf_levels(rt_ctx* c, const SceneDev& S, const FrameDev& F, int levels, bool count, unsigned* rgba,
                     float* rgbf, StatsDev* stats, hipStream_t st)
{
    const bool big = c->n_tri > kClusterMinTriangles;
    const void* kt = count ? (const void*)&rt_wf_trace<true> : (const void*)&rt_wf_trace<false>;
    const void* kg = count ? (const void*)&rt_wf_straggle<true> : (const void*)&rt_wf_straggle<false>;
    // (frames under 4 Mpx: the two-entry light-buffer walk, pick_kernel)
    const bool small = c->opt_lb_unroll && W_px_small(c);
    const void* ks = big ? (small ? (count ? (const void*)&rt_wf_shade<2054, true> : (const void*)&rt_wf_shade<2054, false>)
                                  : (count ? (const void*)&rt_wf_shade<6, true> : (const void*)&rt_wf_shade<6, false>))
                         : (count ? (const void*)&rt_wf_shade<5, true> : (const void*)&rt_wf_shade<5, false>);
    // (RT_OPT_WF_OVERLAP: the stragglers' walks and shading on a second
    // stream, beside the level's main shade launch)
    const void* ks2 =
        big ? (small ? (count ? (const void*)&rt_wf_shade<2054, true, true> : (const void*)&rt_wf_shade<2054, false, true>)
                     : (count ? (const void*)&rt_wf_shade<6, true, true> : (const void*)&rt_wf_shade<6, false, true>))
            : (count ? (const void*)&rt_wf_shade<5, true, true> : (const void*)&rt_wf_shade<5, false, true>);
    const unsigned lds_t = (unsigned)((size_t)c->bvh_depth * 64 * sizeof(int));
    const unsigned lds_s = big ? (unsigned)kLdsWaveBytes : 0u;
    rt_ctx::WfBuf& W = c->wf;
    const bool ovl = c->opt_wf_overlap;
    if (ovl) {
        if (!W.st2) HIP_TRY(c, hipStreamCreateWithFlags(&W.st2, hipStreamNonBlocking));
        if (!W.ev_t) HIP_TRY(c, hipEventCreateWithFlags(&W.ev_t, hipEventDisableTiming));
        if (!W.ev_s) HIP_TRY(c, hipEventCreateWithFlags(&W.ev_s, hipEventDisableTiming));
    }
    for (int L = 1; L <= levels; ++L) {
        // enough waves to fill the chip; each strides over the level's queue
        const size_t waves = (W.cap[L] + 63) / 64;
        const unsigned gt = (unsigned)std::max<size_t>(1, std::min<size_t>(waves, (size_t)c->n_cu * RT_WF_TRACE_WAVES));
        const unsigned gs = (unsigned)std::max<size_t>(1, std::min<size_t>(waves, (size_t)c->n_cu * RT_WF_SHADE_WAVES));
        FrameDev Fl = F;
        Fl.wf.budget = W.cap[L] >= (size_t)RT_WF_BUDGET_SPLIT ? RT_WF_BUDGET_BIG : RT_WF_BUDGET_SMALL;
        if (!ovl) Fl.wf.hit2 = nullptr;
        const unsigned gq = (unsigned)std::max<size_t>(1, std::min<size_t>(waves, (size_t)c->n_cu * 32));
        if (W.dev.kin) {
            // the level's live rays by bin (parent surface in BVH leaf order,
            // branch): rays leaving one triangle share its normal, rays of
            // neighbouring triangles their subtree, so their walks and hits
            // stay together
            // (the counts came with the appends; the scan leaves them zero
            // for the next level's)
            const unsigned bins = 2u * c->nbin_half;
            unsigned* next = W.hist + 2 * W.hcap;
            HIP_TRY(c, scan_u32(W.hist, bins, next, W.bsum, st, nullptr, true));
            hipLaunchKernelGGL(rt_wf_sort_place<0>, dim3(gq), dim3(64), 0, st, S, F, L, (const unsigned*)nullptr, next,
                               W.kout);
            HIP_TRY(c, hipGetLastError());
            Fl.wf.kout = W.kout;
        }
        int Lv = L;
        void* args[] = {(void*)&S, (void*)&Fl, (void*)&Lv, (void*)&stats};
        HIP_TRY(c, hipLaunchKernel(kt, dim3(gt), dim3(64), args, lds_t, st));
        if (!ovl)
            HIP_TRY(c, hipLaunchKernel(kg, dim3((unsigned)c->n_cu * RT_WF_STRAG_WAVES), dim3(64), args,
                                       (unsigned)(kWfStragCap * sizeof(int)), st));
        FrameDev Fs = Fl;
        if (W.sort & 2) {
            // the level's rays by hit surface's bin for the shading (whose
            // children, appended in that order, then sit by parent bin)
            // (bit 2: by the hit point's light-buffer cell instead, wf_sort_key<2>)
            const bool cell = (W.sort & 4) != 0 && c->lb_r0 > 0;
            const unsigned hb = cell ? 6u * (unsigned)c->lb_r0 * (unsigned)c->lb_r0 + kWfMissBins
                                     : c->nbin_half + kWfMissBins;
            unsigned *hist2 = W.hist + W.hcap, *next = W.hist + 2 * W.hcap;
            // (both passes read the rays in queue order: consecutive slots,
            // coalesced hit records — the order inside a bin does not matter)
            if (cell)
                hipLaunchKernelGGL(rt_wf_hit_count<2>, dim3(gq), dim3(64), 0, st, S, F, L, (const unsigned*)nullptr,
                                   hist2);
            else
                hipLaunchKernelGGL(rt_wf_hit_count<1>, dim3(gq), dim3(64), 0, st, S, F, L, (const unsigned*)nullptr,
                                   hist2);
            HIP_TRY(c, hipGetLastError());
            HIP_TRY(c, scan_u32(hist2, hb, next, W.bsum, st, nullptr, true));
            if (cell)
                hipLaunchKernelGGL(rt_wf_sort_place<2>, dim3(gq), dim3(64), 0, st, S, F, L, (const unsigned*)nullptr,
                                   next, W.kout2);
            else
                hipLaunchKernelGGL(rt_wf_sort_place<1>, dim3(gq), dim3(64), 0, st, S, F, L, (const unsigned*)nullptr,
                                   next, W.kout2);
            HIP_TRY(c, hipGetLastError());
            Fs.wf.kout = W.kout2;
        }
        void* sargs[] = {(void*)&S, (void*)&Fs, (void*)&Lv, (void*)&stats};
        if (ovl) {
            // fork: the stragglers finish their walks (into hit2) and are
            // shaded on st2 while st shades the level's other rays; join
            // before the next level reads its queue
            HIP_TRY(c, hipEventRecord(W.ev_t, st));
            HIP_TRY(c, hipStreamWaitEvent(W.st2, W.ev_t, 0));
            HIP_TRY(c, hipLaunchKernel(kg, dim3((unsigned)c->n_cu * RT_WF_STRAG_WAVES), dim3(64), args,
                                       (unsigned)(kWfStragCap * sizeof(int)), W.st2));
            HIP_TRY(c, hipLaunchKernel(ks2, dim3(gs), dim3(64), sargs, lds_s, W.st2));
            HIP_TRY(c, hipEventRecord(W.ev_s, W.st2));
        }
        HIP_TRY(c, hipLaunchKernel(ks, dim3(gs), dim3(64), sargs, lds_s, st));
        if (ovl) HIP_TRY(c, hipStreamWaitEvent(st, W.ev_s, 0));
    }
    for (int L = levels - 1; L >= 0; --L) {
        const unsigned g = (unsigned)std::min<size_t>((c->wf.pcap[L] + 255) / 256, (size_t)c->n_cu * RT_WF_FOLD_BLOCKS);
        hipLaunchKernelGGL(rt_wf_fold, dim3(std::max(1u, g)), dim3(256), 0, st, F, L, rgba, rgbf);
        HIP_TRY(c, hipGetLastError());
    }
    return RT_OK;
}

static int launch(rt_ctx* c, const rt_frame* f, unsigned* rgba_dev, float* rgb_dev, hipStream_t st, bool timed,
                  bool sync_path, void* host_out = nullptr)
{
    if (!c || !f) return RT_E_ARG;
    if (!c->uploaded) {
        c->err = "render before rt_upload_scene";
        return RT_E_STATE;
    }
    if (!frame_ok(f)) {
        c->err = "bad rt_frame geometry";
        return RT_E_ARG;
    }
    bool capturing = false;
    if (!sync_path) {
        hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
        HIP_TRY(c, hipStreamIsCapturing(st, &cs));
        capturing = cs != hipStreamCaptureStatusNone;
    }
    const int depth = reachable_depth(c, f);
    const bool lbuf = lbuf_on(c);
    const bool bvh = bvh_on(c, depth, lbuf);
    const bool cb_want = cam_lists(c, depth, lbuf) && c->n_tri > 0 && c->opt_camera_buffer && cb_frame_ok(f);
    const int rows = frame_rows(f);
    // tiny scenes: the camera records travel with the launch (no device state)
    TinyCam Tl;
    const TinyCam* tiny = nullptr;
    int tmode = 0;  // the tile masks: 0 read, 1 computed by the kernel, 2 computed and stored (tiny_masks)
    if (tiny_ok(c, depth, lbuf)) {
        Tl = tiny_prepare(c, f);
        if (rows > 0)
            if (int rc = tiny_masks(c, f, st, capturing, Tl, &tmode)) return rc;
        tiny = &Tl;
    }
    if (rows > 0 && !tiny) {
        if (int rc = prepare_state(c, f, st, sync_path, capturing, cb_want)) return rc;
    }
    const bool cbuf = !tiny && cb_want && cb_matches(c->cb, f);
    // Wavefront: a BVH frame's bounce levels as compacted queues (rt_wavefront.h);
    // its queues are shared by the context's streams: a frame on another
    // stream than the last wavefront frame waits for that one.  A captured
    // frame renders by the BVH megakernel instead (no shared state).
    bool wf = bvh && rows > 0 && !capturing && wf_fits(c, f, depth, rows);
    if (wf) {
        bool ok = false;
        if (int rc = wf_ensure(c, f, rows, depth, capturing, &ok)) return rc;
        wf = ok;
    }
    const bool count = (f->flags & RT_FLAG_STATS) != 0;
    const bool small = (double)f->width * rows < 4e6 && c->opt_lb_unroll;
    const KernelPick kp = wf ? (count ? pick_wf0<true>(c->n_tri, cbuf, small) : pick_wf0<false>(c->n_tri, cbuf, small))
                             : (count ? pick_kernel<true>(depth, c->n_tri, c->n_lights, lbuf, cbuf,
                                                          bvh ? c->bvh_depth : 0, reflect_chain(c, f), small)
                                      : pick_kernel<false>(depth, c->n_tri, c->n_lights, lbuf, cbuf,
                                                           bvh ? c->bvh_depth : 0, reflect_chain(c, f), small));
    if (!kp.k) {
        c->err = "reachable bounce depth " + std::to_string(depth) + " exceeds the compiled stack (32)";
        return RT_E_UNSUPPORTED;
    }
    SceneDev S = scene_dev(c, lbuf, cbuf);
    FrameDev F;
    frame_dev(f, F);
    if (wf) F.wf = c->wf.dev;
    c->last = rt_stats{};
    c->last.stack_depth = wf ? depth : kp.cap;
    c->last.light_batch = kp.lb;
    if (wf)
        std::snprintf(c->last.kernel, sizeof c->last.kernel, "wavefront %s + %d levels", kp.name, depth);
    else if (tiny)
        std::snprintf(c->last.kernel, sizeof c->last.kernel, "rt_trace_tiny<0,1,%d>",
                      tmode == 2 ? 229 : (tmode == 1 ? 101 : 37));
    else
        std::memcpy(c->last.kernel, kp.name, sizeof kp.name);
    if (rows == 0) return RT_OK;
    if (f->flags & RT_FLAG_STATS) HIP_TRY(c, hipMemsetAsync(c->d_stats, 0, kStatSlots * sizeof(StatsDev), st));
    if (timed) HIP_TRY(c, hipEventRecord(c->ev0, st));
    StatsDev* stats = c->d_stats;
    const size_t px_bytes = rgba_dev ? 4 : 12;
    // a chunk per RT_OPT_HOST_CHUNK_MB (8 MiB; each copy has a fixed cost of
    // tens of us: a 1080p RGBA8 frame is one copy, 4K four chunks -10%,
    // 7680 x 4320 eight chunks -30%, tools/host_chunks.py)
    const size_t out_bytes = (size_t)rows * f->width * px_bytes;
    const double chunk = c->opt_host_chunk_mb * 1048576.0;
    const int nch = (host_out && f->band_rows == 0 && chunk > 0 && !wf)
                        ? (int)std::min(8.0, std::floor((double)out_bytes / chunk))
                        : 1;
    if (wf) {
        rt_ctx::WfBuf& W = c->wf;
        if (W.pending && W.last != st) HIP_TRY(c, hipStreamWaitEvent(st, W.ev, 0));
        HIP_TRY(c, hipMemsetAsync(W.dev.count, 0, kWfCountBytes, st));
        if (W.sort)  // the bin counts (level 1's: the level-0 kernel's appends)
            HIP_TRY(c, hipMemsetAsync(W.dev.hist, 0, 2 * W.hcap * sizeof(unsigned), st));
    }
    if (nch <= 1) {
        if (int rc = launch_trace(c, kp, tiny, f->flags & RT_FLAG_STATS, S, F, f->width, rows, rgba_dev, rgb_dev, stats,
                                  st, tmode))
            return rc;
        if (tmode == 2)
            if (int rc = tiny_masks_stored(c, st)) return rc;
        if (wf) {
            if (int rc = wf_levels(c, S, F, depth, count, rgba_dev, rgb_dev, stats, st)) return rc;
            HIP_TRY(c, hipEventRecord(c->wf.ev, st));
            c->wf.last = st;
            c->wf.pending = true;
        }
        if (host_out)
            HIP_TRY(c, hipMemcpyAsync(host_out, rgba_dev ? (void*)rgba_dev : (void*)rgb_dev,
                                      (size_t)rows * f->width * px_bytes, hipMemcpyDeviceToHost, st));
    } else {
        // every chunk's kernel first, then the copies (a copy into pageable
        // memory blocks the host; the kernels behind it keep running)
        const int step = ((rows + nch - 1) / nch + 15) / 16 * 16;
        int n = 0;
        for (int r0 = 0; r0 < rows; r0 += step, ++n) {
            const int r1 = std::min(rows, r0 + step);
            FrameDev Fc = F;
            Fc.row_begin = f->row_begin + r0;
            Fc.row_end = f->row_begin + r1;
            unsigned* oa = rgba_dev ? rgba_dev + (size_t)r0 * f->width : nullptr;
            float* ob = rgb_dev ? rgb_dev + (size_t)r0 * f->width * 3 : nullptr;
            if (int rc = launch_trace(c, kp, tiny, f->flags & RT_FLAG_STATS, S, Fc, f->width, r1 - r0, oa, ob, stats, st,
                                      tmode))
                return rc;
            HIP_TRY(c, hipEventRecord(c->ev_chunk[n], st));
        }
        if (tmode == 2)
            if (int rc = tiny_masks_stored(c, st)) return rc;
        if (timed) HIP_TRY(c, hipEventRecord(c->ev1, st));
        const char* src = (const char*)(rgba_dev ? (void*)rgba_dev : (void*)rgb_dev);
        for (int i = 0; i < n; ++i) {
            const int r0 = i * step, r1 = std::min(rows, r0 + step);
            const size_t off = (size_t)r0 * f->width * px_bytes;
            HIP_TRY(c, hipStreamWaitEvent(c->copy_stream, c->ev_chunk[i], 0));
            HIP_TRY(c, hipMemcpyAsync((char*)host_out + off, src + off, (size_t)(r1 - r0) * f->width * px_bytes,
                                      hipMemcpyDeviceToHost, c->copy_stream));
        }
        timed = false;  // ev1 already recorded after the last kernel
    }
    if (timed) HIP_TRY(c, hipEventRecord(c->ev1, st));
    if (capturing) {
        c->captured = true;
        if (cbuf) c->cb.pinned = true;
    } else if (!sync_path) {  // (uploads and rt_destroy sync every such stream)
        note_async(c, st);
    }
    return RT_OK;
}

static int finish_sync(rt_ctx* c, const rt_frame* f, hipStream_t st, bool timed)
{
    HIP_TRY(c, hipStreamSynchronize(st));
    HIP_TRY(c, hipStreamSynchronize(c->copy_stream));
    // c->stream waited for every async render enqueued before this call
    // (fence_async), so none is in flight any more
    c->async_streams.clear();
    c->state_pending = false;
    c->state_stream = nullptr;
    c->wf.pending = false;
    free_deferred(c);
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
            h.btri += q.btri;
            h.bnode += q.bnode;
        }
        c->last.primary_rays = h.primary;
        c->last.bounce_rays = h.bounce;
        c->last.shadow_rays = h.shadow;
        c->last.shadow_tests_skipped = h.skipped;
        c->last.triangle_tests = h.tri;
        c->last.plane_tests = h.pla;
        c->last.quadric_tests = h.qua;
        c->last.bounce_triangle_tests = h.btri;
        c->last.bvh_nodes_visited = h.bnode;
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
    release(c, c->d_scratch);
    c->d_scratch = nullptr;
    c->scratch_bytes = 0;
    HIP_TRY(c, hipMalloc(&c->d_scratch, bytes));
    c->scratch_bytes = bytes;
    return RT_OK;
}

static int render_sync(rt_ctx* c, const rt_frame* f, void* out, bool as_float)
{
    if (!c || !f || !out) return RT_E_ARG;
    if (c->cpu) return not_cpu(c);
    HIP_TRY(c, hipSetDevice(c->device));
    // every state write and render of this call comes after the async
    // renders already enqueued on other streams
    if (int rc = fence_async(c, c->stream)) return rc;
    if (int rc = wait_state(c, c->stream)) return rc;
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
                    true, (!dev && bytes) ? out : nullptr);
    if (rc) return rc;
    return finish_sync(c, f, c->stream, true);
}

RT_EXPORT int rt_render(rt_ctx* c, const rt_frame* f, uint8_t* rgba8_out) { return render_sync(c, f, rgba8_out, false); }

RT_EXPORT int rt_render_float(rt_ctx* c, const rt_frame* f, float* rgb_out) { return render_sync(c, f, rgb_out, true); }

RT_EXPORT int rt_render_async(rt_ctx* c, const rt_frame* f, uint8_t* rgba8_dev, float* rgb_dev, void* stream)
{
    if (!c || !f) return RT_E_ARG;
    if (c->cpu) return not_cpu(c);
    HIP_TRY(c, hipSetDevice(c->device));
    return launch(c, f, (unsigned*)rgba8_dev, rgb_dev, (hipStream_t)stream, false, false);
}

RT_EXPORT int rt_render_sequence_async(rt_ctx* c, const rt_frame* frames, int32_t n, uint8_t* rgba8_dev,
                                       size_t rgba8_stride, float* rgb_dev, size_t rgb_stride, void* stream)
{
    if (!c || (n > 0 && !frames) || n < 0) return RT_E_ARG;
    if (c->cpu) return not_cpu(c);
    if (!c->uploaded) {
        c->err = "render before rt_upload_scene";
        return RT_E_STATE;
    }
    HIP_TRY(c, hipSetDevice(c->device));
    hipStream_t st = (hipStream_t)stream;
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    HIP_TRY(c, hipStreamIsCapturing(st, &cs));
    const bool capturing = cs != hipStreamCaptureStatusNone;
    // everything is checked before anything is enqueued
    for (int i = 0; i < n; ++i) {
        const rt_frame* f = frames + i;
        if (!frame_ok(f) || (f->flags & RT_FLAG_STATS)) {
            c->err = "bad rt_frame geometry (or RT_FLAG_STATS) in a sequence";
            return RT_E_ARG;
        }
        if (!pick_kernel<false>(reachable_depth(c, f), c->n_tri, c->n_lights, false, false).k) {
            c->err = "reachable bounce depth exceeds the compiled stack (32)";
            return RT_E_UNSUPPORTED;
        }
    }
    const bool lbuf = lbuf_on(c);
    // The camera slots are shared by every sequence call: one on another
    // stream still in flight must finish first (a captured sequence's
    // ordering against work outside the graph is the caller's, as for any
    // captured launch).
    if (!capturing && n > 0) {
        if (int rc = fence_async(c, st)) return rc;
    }
    // Fork: the internal streams start after everything already on st.
    const int nstreams = std::min(n, kSeqSlots);
    if (nstreams > 1) {
        for (int j = 0; j < nstreams; ++j) {
            if (!c->seq_streams[j]) HIP_TRY(c, hipStreamCreateWithFlags(&c->seq_streams[j], hipStreamNonBlocking));
            if (!c->seq_join[j]) HIP_TRY(c, hipEventCreateWithFlags(&c->seq_join[j], hipEventDisableTiming));
        }
        if (!c->seq_fork) HIP_TRY(c, hipEventCreateWithFlags(&c->seq_fork, hipEventDisableTiming));
        HIP_TRY(c, hipEventRecord(c->seq_fork, st));
        for (int j = 0; j < nstreams; ++j) HIP_TRY(c, hipStreamWaitEvent(c->seq_streams[j], c->seq_fork, 0));
    }
    for (int i = 0; i < n; ++i) {
        const rt_frame* f = frames + i;
        rt_ctx::CamSlot& q = c->seq[i % kSeqSlots];
        hipStream_t fs = nstreams > 1 ? c->seq_streams[i % nstreams] : st;
        const int rows = frame_rows(f);
        if (rows == 0) continue;
        const int depth = reachable_depth(c, f);
        // the slot's camera buffer (round 3, big lists as for rt_render_async):
        // built on the frame's stream like its records; inside a capture only
        // into buffers already sized (a first capture renders without it —
        // the same image)
        const int nt = ((f->width + 7) / 8) * ((f->height + 7) / 8);
        TinyCam T;
        int tmode = 0;
        const bool tiny = tiny_ok(c, depth, lbuf);
        if (tiny) {
            tiny_build(c, f, T);
            if (int rc = tiny_masks(c, f, fs, capturing, T, &tmode)) return rc;
        }
        const bool bvh = bvh_on(c, depth, lbuf);
        const bool cbuf = !tiny && cam_lists(c, depth, lbuf) && c->n_tri > 0 && c->opt_camera_buffer && cb_frame_ok(f) &&
                          cb_async_pays(c, f) &&
                          (!capturing || (q.cb.cap > 0 && q.cb.rcap > 0 && q.cb.nt_alloc >= nt && q.cb.big_alloc >= c->n_tri));
        if (c->n_tri > 0 && !tiny) {
            if (int rc = camera_records(c, f->cam_pos, fs, cbuf, q.tricam, q.cone_cam, q.uni, q.clu_cam)) return rc;
        }
        const KernelPick kp =
            pick_kernel<false>(depth, c->n_tri, c->n_lights, lbuf, cbuf, bvh ? c->bvh_depth : 0, reflect_chain(c, f));
        SceneDev S = scene_dev(c, lbuf, false);
        S.tricam = q.tricam;
        S.cone_cam = q.cone_cam;
        S.clu_cam = q.clu_cam;
        S.uni = (q.uni && c->opt_union) ? q.uni : nullptr;
        if (cbuf) {
            if (int rc = cb_build(c, q.cb, f, S, fs, false, capturing, false)) return rc;
            S.cb_off = q.cb.off;
            S.cb_ent = q.cb.ent;
            S.cb_flag = q.cb.flag;
            S.cb_tiles_x = q.cb.tiles_x;
            S.cb_rec = nullptr;
        }
        FrameDev F;
        frame_dev(f, F);
        unsigned* rgba = rgba8_dev ? (unsigned*)(rgba8_dev + (size_t)i * rgba8_stride) : nullptr;
        float* rgb = rgb_dev ? (float*)((char*)rgb_dev + (size_t)i * rgb_stride) : nullptr;
        if (int rc = launch_trace(c, kp, tiny ? &T : nullptr, false, S, F, f->width, rows, rgba, rgb, c->d_stats, fs,
                                  tmode))
            return rc;
        if (tmode == 2)
            if (int rc = tiny_masks_stored(c, fs)) return rc;
    }
    // Join: st continues after every frame.
    if (nstreams > 1) {
        for (int j = 0; j < nstreams; ++j) {
            HIP_TRY(c, hipEventRecord(c->seq_join[j], c->seq_streams[j]));
            HIP_TRY(c, hipStreamWaitEvent(st, c->seq_join[j], 0));
        }
    }
    if (capturing)
        c->captured = true;
    else if (n > 0)
        note_async(c, st);
    return RT_OK;
}

RT_EXPORT int rt_prepare_camera(rt_ctx* c, const rt_frame* f)
{
    if (!c || !f) return RT_E_ARG;
    if (c->cpu) return not_cpu(c);
    if (!c->uploaded) {
        c->err = "rt_prepare_camera before rt_upload_scene";
        return RT_E_STATE;
    }
    if (!frame_ok(f)) {
        c->err = "bad rt_frame geometry";
        return RT_E_ARG;
    }
    HIP_TRY(c, hipSetDevice(c->device));
    if (int rc = fence_async(c, c->stream)) return rc;
    if (int rc = wait_state(c, c->stream)) return rc;
    const int depth = reachable_depth(c, f);
    const bool cb_want = cam_lists(c, depth, lbuf_on(c)) && c->n_tri > 0 && c->opt_camera_buffer && cb_frame_ok(f);
    if (int rc = prepare_state(c, f, c->stream, true, false, cb_want)) return rc;
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    c->async_streams.clear();
    c->state_pending = false;
    c->state_stream = nullptr;
    c->wf.pending = false;
    free_deferred(c);
    return RT_OK;
}

static int cpu_render_sync(rt_ctx* c, const rt_frame* f, uint8_t* rgba, float* rgb)
{
    if (!c || !f || (!rgba && !rgb)) return RT_E_ARG;
    if (!c->cpu) {
        c->err = "rt_cpu_render needs a CPU context (rt_create_cpu)";
        return RT_E_STATE;
    }
    if (!c->uploaded) {
        c->err = "render before rt_upload_scene";
        return RT_E_STATE;
    }
    if (!frame_ok(f)) {
        c->err = "bad rt_frame geometry";
        return RT_E_ARG;
    }
    c->last = rt_stats{};
    double ms = 0.0;
    const int rc = cpu_render(c->cpu_scene, c->cpu_threads, f, frame_rows(f), rgba, rgb, &ms);
    c->last.kernel_ms = (float)ms;
    return rc;
}

RT_EXPORT int rt_cpu_render(rt_ctx* c, const rt_frame* f, uint8_t* rgba8_out)
{
    return cpu_render_sync(c, f, rgba8_out, nullptr);
}

RT_EXPORT int rt_cpu_render_float(rt_ctx* c, const rt_frame* f, float* rgb_out)
{
    return cpu_render_sync(c, f, nullptr, rgb_out);
}

RT_EXPORT int rt_last_stats(rt_ctx* c, rt_stats* out)
{
    if (!c || !out) return RT_E_ARG;
    *out = c->last;
    return RT_OK;
}

#ifdef RT_PROF
// Diagnostic builds only (include/rt_debug.h, RT_PROF): read and clear the per-section
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

// Diagnostic (include/rt_debug.h): light-buffer summary of the uploaded
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

// Diagnostic (include/rt_debug.h): camera-buffer summary: out[0] = current
// (0/1), out[1] = entries, out[2] = the last synchronous build's device ms
// (its kernels, first to last; async builds are not timed), out[3] = tiles,
// out[4] = inline records (0/1), out[5] = the build's host wall time up to
// its last enqueue (ms); out[6..9] = candidate pairs, lists longer than
// 256, the longest of them, the entry capacity.
RT_EXPORT int rt_debug_cb_info(rt_ctx* c, double* out, int n)
{
    if (!c || !out || n < 4) return RT_E_ARG;
    if (c->cpu) return not_cpu(c);
    rt_ctx::CamBuf& B = c->cb;
    if (B.timed) {
        float ms = 0.f;
        HIP_TRY(c, hipEventSynchronize(B.ev1));
        HIP_TRY(c, hipEventElapsedTime(&ms, B.ev0, B.ev1));
        B.build_ms = ms;
        B.timed = false;
    }
    if (B.tot_pending) {
        HIP_TRY(c, hipEventSynchronize(B.ev_tot));
        cb_harvest(B);
    }
    out[0] = B.valid ? 1.0 : 0.0;
    out[1] = (double)B.entries;
    out[2] = B.build_ms;
    out[3] = (double)B.ntiles;
    if (n > 4) out[4] = B.inline_rec ? 1.0 : 0.0;
    if (n > 5) out[5] = B.host_ms;
    // binning counters: candidate (triangle, tile) pairs tested, lists
    // sorted in LDS (longer than 256), the longest of them, the capacity
    if (n > 6) out[6] = B.hstat[1];
    if (n > 7) out[7] = B.hstat[3];
    if (n > 8) out[8] = B.hstat[4];
    if (n > 9) out[9] = (double)B.cap;
    if (n > 10) out[10] = B.hstat[6];  // 1: candidate pairs past 2^32 - 1 (every tile flagged)
    return RT_OK;
}

// Diagnostic (include/rt_debug.h): the current camera buffer against brute
// force (rt_cb_verify): out[0] = tiles whose list is not exactly the
// passing triangles (or mis-keyed), out[1] = passing pairs, out[2] = tiles
// with a list.  Synchronous.
RT_EXPORT int rt_debug_cb_verify(rt_ctx* c, unsigned long long* out)
{
    if (!c || !out) return RT_E_ARG;
    if (c->cpu) return not_cpu(c);
    HIP_TRY(c, hipSetDevice(c->device));
    if (int rc = sync_all(c)) return rc;
    rt_ctx::CamBuf& B = c->cb;
    if (!B.valid) {
        c->err = "no current camera buffer";
        return RT_E_STATE;
    }
    unsigned* d = nullptr;
    HIP_TRY(c, hipMalloc((void**)&d, 2 * sizeof(unsigned)));
    int rc = RT_OK;
    if (hipMemset(d, 0, 2 * sizeof(unsigned)) != hipSuccess) rc = RT_E_HIP;
    CbDev D{};
    D.tcone = B.tcone;
    D.off = B.off;
    D.cur = B.cur;
    D.flag = B.flag;
    D.ent = B.ent;
    D.cap = (unsigned)B.cap;
    D.tiles_x = B.tiles_x;
    D.tiles_y = B.ntiles / std::max(1, B.tiles_x);
    const SceneDev S = scene_dev(c, false, true);
    unsigned h[2] = {0, 0};
    std::vector<unsigned> flags((size_t)B.ntiles);
    if (rc == RT_OK) {
        hipLaunchKernelGGL(rt_cb_verify, dim3((unsigned)((B.ntiles + 3) / 4)), dim3(256), 0, c->stream, S, D, d);
        if (hipGetLastError() != hipSuccess || hipStreamSynchronize(c->stream) != hipSuccess ||
            hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost) != hipSuccess ||
            hipMemcpy(flags.data(), B.flag, flags.size() * sizeof(unsigned), hipMemcpyDeviceToHost) != hipSuccess)
            rc = RT_E_HIP;
    }
    hipFree(d);
    out[0] = h[0];
    out[1] = h[1];
    out[2] = (unsigned long long)std::count(flags.begin(), flags.end(), 0u);
    return rc;
}

// Diagnostic (include/rt_debug.h): the last rt_upload_scene's host wall
// time by part (ms): out[0] records + device copies, out[1] cone / cluster
// prepasses, out[2] light buffer (incl. its far ladder), out[3] total.
RT_EXPORT int rt_debug_upload_info(rt_ctx* c, double* out, int n)
{
    if (!c || !out || n < 4) return RT_E_ARG;
    for (int i = 0; i < 4; ++i) out[i] = c->upload_parts_ms[i];
    // light-buffer build phases: cone records to the host, host preparation,
    // supercell counts + scan, supercell lists + cell counts + scan, entries
    for (int i = 0; i < 5 && 4 + i < n; ++i) out[4 + i] = c->lb_parts_ms[i];
    if (n > 9) out[9] = c->lb_r0;  // light 0's first buffer: cells per face edge (0: none)
    return RT_OK;
}

// Diagnostic (include/rt_debug.h): scan_u32 (the builds' device prefix sum)
// of host counts, in place like its callers: out[0..n) the exclusive
// prefixes mod 2^32, out[n] the total mod 2^32, *total the 64-bit total.
RT_EXPORT int rt_debug_scan(int device, const unsigned* in, unsigned n, unsigned* out, unsigned long long* total)
{
    if (!in || !out || !total || n == 0) return RT_E_ARG;
    if (hipSetDevice(device) != hipSuccess) return RT_E_HIP;
    unsigned* d = nullptr;
    unsigned long long* bs = nullptr;
    int rc = RT_OK;
    if (hipMalloc(&d, ((size_t)n + 1) * sizeof(unsigned)) != hipSuccess ||
        hipMalloc(&bs, scan_scratch(n) * sizeof(unsigned long long)) != hipSuccess)
        rc = RT_E_HIP;
    unsigned long long* tot = nullptr;
    if (rc == RT_OK && (hipMemcpy(d, in, (size_t)n * sizeof(unsigned), hipMemcpyHostToDevice) != hipSuccess ||
                        scan_u32(d, n, d, bs, 0, &tot) != hipSuccess || hipDeviceSynchronize() != hipSuccess ||
                        hipMemcpy(out, d, ((size_t)n + 1) * sizeof(unsigned), hipMemcpyDeviceToHost) != hipSuccess ||
                        hipMemcpy(total, tot, sizeof(unsigned long long), hipMemcpyDeviceToHost) != hipSuccess))
        rc = RT_E_HIP;
    hipFree(d);
    hipFree(bs);
    return rc;
}

// Diagnostic (include/rt_debug.h): run rt_selftest_kernel over `blocks`
// workgroups; *failures = lanes whose wave reduction or wave cone was wrong.
RT_EXPORT int rt_debug_bvh_info(rt_ctx* c, double* out, int n)
{
    if (!c || !out || n <= 0) return RT_E_ARG;
    const double v[5] = {c->d_bvh_node ? 1.0 : 0.0, (double)c->bvh_inner, (double)c->bvh_leaves, (double)c->bvh_depth,
                         c->bvh_build_ms};
    for (int i = 0; i < n; ++i) out[i] = i < 5 ? v[i] : 0.0;
    return RT_OK;
}

// Diagnostic (include/rt_debug.h): the last wavefront frame's queue counts,
// per level L = 0 .. kWfMaxLevels: out[3 L] rays of level L (L >= 1), out[3 L
// + 1] parents of level L, out[3 L + 2] straggling walks of level L.
RT_EXPORT int rt_debug_wf_counts(rt_ctx* c, unsigned* out, int n)
{
    if (!c || !out || n <= 0) return RT_E_ARG;
    if (c->cpu) return not_cpu(c);
    if (!c->wf.mem) {
        c->err = "no wavefront frame rendered";
        return RT_E_STATE;
    }
    if (int rc = sync_all(c)) return rc;
    std::vector<unsigned> w(kWfCountBytes / 4);
    HIP_TRY(c, hipMemcpy(w.data(), c->wf.dev.count, kWfCountBytes, hipMemcpyDeviceToHost));
    for (int i = 0; i < n; ++i) {
        const int L = i / 3, k = i % 3;
        unsigned v = 0;
        if (L <= kWfMaxLevels) {
            if (k == 2) {
                v = w[wf_strag(L)];
            } else {
                for (int s = 0; s < kWfSeg; ++s) v += w[k == 0 ? wf_rays(L, s) : wf_pars(L, s)];
            }
        }
        out[i] = v;
    }
    return RT_OK;
}

// Diagnostic (include/rt_debug.h): the host BVH build alone (no device) over
// n triangles of 12 floats (p0, e1, e2, normal: the upload's tri[] records);
// out3 = {depth, inner nodes, leaves}.  RT_E_UNSUPPORTED past kBvhMaxTriangles.
RT_EXPORT int rt_debug_bvh_build(const float* tri12, long long n, int* out3)
{
    if (!tri12 || !out3 || n <= kBvhLeafMax) return RT_E_ARG;
    if ((size_t)n > kBvhMaxTriangles) return RT_E_UNSUPPORTED;
    std::vector<float> tri(tri12, tri12 + 12 * (size_t)n);
    BvhBuilt B;
    bvh_build(tri, (size_t)n, B);
    out3[0] = B.depth;
    out3[1] = B.inner;
    out3[2] = B.leaves;
    return RT_OK;
}

RT_EXPORT int rt_debug_bvh_rays(rt_ctx* c, const float* rays, int n, int* out_idx, float* out_t,
                                unsigned long long* tally2)
{
    if (!c || !rays || n < 0 || !out_idx || !out_t || !tally2) return RT_E_ARG;
    if (c->cpu) return not_cpu(c);
    if (!c->uploaded || !c->d_bvh_node) {
        c->err = "no bounce-ray BVH (scene without reflective/refractive surfaces or < 64 triangles)";
        return RT_E_STATE;
    }
    HIP_TRY(c, hipSetDevice(c->device));
    if (int rc = sync_all(c)) return rc;
    if (n == 0) return RT_OK;
    float* d_rays = nullptr;
    int* d_idx = nullptr;
    float* d_t = nullptr;
    unsigned long long* d_tally = nullptr;
    int rc = RT_OK;
    auto chk = [&](hipError_t e, const char* what) {
        if (e != hipSuccess && rc == RT_OK) rc = hip_fail(c, e, what);
        return rc == RT_OK;
    };
    if (chk(hipMalloc(&d_rays, (size_t)n * 6 * sizeof(float)), "hipMalloc") &&
        chk(hipMalloc(&d_idx, (size_t)n * 2 * sizeof(int)), "hipMalloc") &&
        chk(hipMalloc(&d_t, (size_t)n * 2 * sizeof(float)), "hipMalloc") &&
        chk(hipMalloc(&d_tally, 2 * sizeof(unsigned long long)), "hipMalloc") &&
        chk(hipMemcpy(d_rays, rays, (size_t)n * 6 * sizeof(float), hipMemcpyHostToDevice), "hipMemcpy") &&
        chk(hipMemset(d_tally, 0, 2 * sizeof(unsigned long long)), "hipMemset")) {
        const SceneDev S = scene_dev(c, false, false);
        hipLaunchKernelGGL(rt_bvh_rays_kernel, dim3((unsigned)((n + 63) / 64)), dim3(64),
                           (unsigned)(kLdsWaveBytes + kBvhLdsBytes), c->stream, S, d_rays, n, d_idx, d_t, d_tally);
        if (chk(hipGetLastError(), "rt_bvh_rays_kernel") && chk(hipStreamSynchronize(c->stream), "sync") &&
            chk(hipMemcpy(out_idx, d_idx, (size_t)n * 2 * sizeof(int), hipMemcpyDeviceToHost), "hipMemcpy") &&
            chk(hipMemcpy(out_t, d_t, (size_t)n * 2 * sizeof(float), hipMemcpyDeviceToHost), "hipMemcpy"))
            chk(hipMemcpy(tally2, d_tally, 2 * sizeof(unsigned long long), hipMemcpyDeviceToHost), "hipMemcpy");
    }
    hipFree(d_rays);
    hipFree(d_idx);
    hipFree(d_t);
    hipFree(d_tally);
    return rc;
}

RT_EXPORT int rt_debug_bvh_rays_wave(rt_ctx* c, const float* rays, int n, int* out_idx, float* out_t)
{
    if (!c || !rays || n < 0 || !out_idx || !out_t) return RT_E_ARG;
    if (c->cpu) return not_cpu(c);
    if (!c->uploaded || !c->d_bvh_node) {
        c->err = "no bounce-ray BVH";
        return RT_E_STATE;
    }
    HIP_TRY(c, hipSetDevice(c->device));
    if (int rc = sync_all(c)) return rc;
    if (n == 0) return RT_OK;
    float* d_rays = nullptr;
    int* d_idx = nullptr;
    float* d_t = nullptr;
    int rc = RT_OK;
    auto chk = [&](hipError_t e, const char* what) {
        if (e != hipSuccess && rc == RT_OK) rc = hip_fail(c, e, what);
        return rc == RT_OK;
    };
    if (chk(hipMalloc(&d_rays, (size_t)n * 6 * sizeof(float)), "hipMalloc") &&
        chk(hipMalloc(&d_idx, (size_t)n * sizeof(int)), "hipMalloc") &&
        chk(hipMalloc(&d_t, (size_t)n * sizeof(float)), "hipMalloc") &&
        chk(hipMemcpy(d_rays, rays, (size_t)n * 6 * sizeof(float), hipMemcpyHostToDevice), "hipMemcpy")) {
        const SceneDev S = scene_dev(c, false, false);
        // the shared stack, then lane 0's serial stack (one step: a row)
        const unsigned lds = (unsigned)(kWfStragCap * sizeof(int) + 64 * sizeof(int) * (size_t)c->bvh_depth);
        hipLaunchKernelGGL(rt_bvh_wave_kernel, dim3((unsigned)n), dim3(64), lds, c->stream, S, d_rays, n, d_idx, d_t);
        if (chk(hipGetLastError(), "rt_bvh_wave_kernel") && chk(hipStreamSynchronize(c->stream), "sync") &&
            chk(hipMemcpy(out_idx, d_idx, (size_t)n * sizeof(int), hipMemcpyDeviceToHost), "hipMemcpy"))
            chk(hipMemcpy(out_t, d_t, (size_t)n * sizeof(float), hipMemcpyDeviceToHost), "hipMemcpy");
    }
    hipFree(d_rays);
    hipFree(d_idx);
    hipFree(d_t);
    return rc;
}

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

