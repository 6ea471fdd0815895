// rt_layout.h — device records in HBM (SceneDev / FrameDev), per-lane counters, the
// RT_PROF section clocks and the exact fast reciprocal.
// Part of the device code of rt_kernels.hip (one translation unit: the
// kernels are templates instantiated by its host half); built with the
// same exactness flags (no FMA contraction, IEEE div/sqrt).
#ifndef RT_AMD_RT_LAYOUT_H
#define RT_AMD_RT_LAYOUT_H

#include <hip/hip_runtime.h>

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
    // wave-level edge-plane test on sphere survivors: small triangle lists
    // (loose spheres of large triangles, C2 -22%, round 1) and, since round
    // 5, big lists too — the clustered per-wave path of a new camera stages
    // its survivors, so every survivor the edges reject saves a wave-serial
    // exact test: C3 moving camera 0.386 -> 0.334 ms, static frames flat
    // (round 1 measured C3 +14% before the staged batches)
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
    // that distance cap).  lb_R = 0: off; else the levels per light: slot
    // level * n_lights + l of lb_meta, each level built for a larger
    // distance than the last (the far buffers), for the lanes beyond it.
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
    // The walk's copy of the entries: per entry the triangle's 64-byte
    // tricam record with the entry's key in word 14 ([3].z), so one scalar
    // load round trip per entry instead of two (cb_ent, then tricam);
    // nullptr: the walk reads cb_ent and tricam (buffers past 128 MB, where
    // the records' extra bytes cost more: C5 +3%, against C3 -4 to -5%).
    // Walked inline by the big-list kernel only (small lists: no gain).
    const float4* __restrict__ cb_rec;
    // Bounce rays (WAVE bit 256, rt_bvh.h): BVH2 inner nodes (5 float4 each,
    // node 0 the root) over every triangle, and the triangles in leaf order
    // (tri[]'s 48-byte layout).  nullptr: none.
    const float4* __restrict__ bvh_node;
    const float4* __restrict__ bvh_tri;
};

// Wavefront bounce queues (rt_wavefront.h; the BVH scenes' bounce levels):
// level L >= 1 holds the rays of bounce L (2 float4 each: [O rior] [D
// energy]) and their colours (1 float4); level L >= 0 the node records of
// the rays (level 0: pixels) that spawned children (2 float4: [acc kr]
// [kt cR cT -], by ray / pixel index) and the list of those parents.
// Rays and parents are appended in kWfSeg segments, each with a counter of
// its own on a 128-byte line of its own (one global counter serialised
// every wave's atomic on one L2 line): a wave appends to segment chunk %
// kWfSeg (chunk = its 64-ray chunk or tile), and segment s of level L
// starts at s * seg[L] (rays) / s * pseg[L] (parents), capacities the host
// sized so that no segment can overflow.  A consumer maps a compacted index
// to its slot through the 16 counts' prefix sums (wf_slot).
// levels = 0: not a wavefront frame.
constexpr int kWfMaxLevels = 8;
constexpr int kWfSeg = 16;
constexpr int kWfCntStride = 32;  // u32 words between counters (128 bytes)
struct WfDev {
    float4* ray[kWfMaxLevels + 1];
    float4* res[kWfMaxLevels + 1];
    float4* node[kWfMaxLevels + 1];
    unsigned* plist[kWfMaxLevels + 1];
    unsigned seg[kWfMaxLevels + 1];   // ray slots per segment, level L >= 1
    unsigned pseg[kWfMaxLevels + 1];  // parent slots per segment, level L >= 0
    float2* hit;      // the level being shaded: [file index (int bits), t] per ray slot
    // RT_OPT_WF_OVERLAP: the straggling walks finish (and their rays are
    // shaded) on a second stream while the level's other rays are shaded:
    // the trace leaves kWfPending in hit[slot] for a straggler, and the
    // straggler kernel writes its minimum here instead; null: into hit.
    float2* hit2;
    int4* strag;      // the level's straggling walks: [ray slot, partial t (bits), partial index, -]
    unsigned* count;  // counters, kWfCntStride words apart: wf_rays / wf_pars / wf_strag
    // Coherence sort (round 6): a ray being appended writes its bin into
    // kin[slot] — its parent surface's spatial bin skey[surf] (triangles in
    // the BVH's leaf order), + nbin_half for a refracted ray — and before the
    // level's trace a counting sort over the level's LIVE rays (rt_wf_sort_*:
    // histogram, scan, scatter) writes the level's slots in bin order into
    // kout; the trace and shade launches take rays in kout's order (null:
    // queue order).
    unsigned* kin;
    const unsigned* kout;
    const unsigned* skey;
    unsigned* hist;       // 2 nbin_half + 1 words: bin counts, then the scatter's next positions
    unsigned nbin_half;
    int levels;
    int budget;  // steps (inner nodes + leaves) a trace-launch walk takes before the straggler hand-off
};
// counter of segment s of level L's rays / parents; level L's stragglers
__host__ __device__ inline int wf_rays(int L, int s) { return (L * kWfSeg + s) * kWfCntStride; }
__host__ __device__ inline int wf_pars(int L, int s) { return ((kWfMaxLevels + 1 + L) * kWfSeg + s) * kWfCntStride; }
__host__ __device__ inline int wf_strag(int L) { return (2 * (kWfMaxLevels + 1) * kWfSeg + L) * kWfCntStride; }
// the trace launch's fetch cursor of level L (rays handed to lanes so far)
__host__ __device__ inline int wf_fetch(int L)
{
    return (2 * (kWfMaxLevels + 1) * kWfSeg + kWfMaxLevels + 1 + L) * kWfCntStride;
}
constexpr size_t kWfCountBytes = (size_t)(2 * (kWfMaxLevels + 1) * kWfSeg + 2 * (kWfMaxLevels + 1)) * kWfCntStride * 4;

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
    // The launch's tile grid and how the big-list kernels deal tiles to the
    // XCDs (RT_OPT_XCD_DEAL, tile_of_block): tiles_x x tiles_y 8 x 8 tiles;
    // xcd_w = tiles per stripe (mode 2) or super-tile columns (mode 3);
    // xcd_m = an XCD's tile slots per tile row (mode 2).
    int tiles_x, tiles_y, xcd_mode, xcd_w, xcd_m;
    WfDev wf;
};

struct StatsDev {
    unsigned long long primary, bounce, shadow, skipped, tri, pla, qua, btri, bnode, pad;
};
// Stats tallies land in kStatSlots copies (by block) so the atomics of a
// launch spread over many addresses instead of serialising on one.
constexpr int kStatSlots = 256;
constexpr unsigned kXcds = 8;  // MI355X: 8 XCDs, one L2 each
#ifndef RT_XCD_CHUNK_BIG
#define RT_XCD_CHUNK_BIG 8
#endif
#ifndef RT_XCD_CHUNK_SMALL
#define RT_XCD_CHUNK_SMALL 0
#endif

// Per-lane tallies (RT_FLAG_STATS): rays, and the exact ray-primitive tests
// the lane's wave executed (a wave-level test counts once per lane).
struct Counters {
    unsigned primary = 0, bounce = 0, shadow = 0, skipped = 0;
    unsigned tri = 0, pla = 0, qua = 0;
    unsigned btri = 0, bnode = 0;  // bounce rays: triangle tests, BVH nodes visited
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
#define RT_EVN(cnt, i, n) ((cnt).ev[i] += (n))
__device__ unsigned long long rt_prof_ev[8];
// per-tile record (16 x u32: total clocks lo/hi, 8 section clocks >> 8, events 1 2 4 5 6 7)
__device__ unsigned* rt_prof_tiles;
__device__ int rt_prof_ntiles;
#else
#define RT_EV(cnt, i) ((void)0)
#define RT_EVN(cnt, i, n) ((void)0)
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

}  // namespace rt
#endif  // RT_AMD_RT_LAYOUT_H
