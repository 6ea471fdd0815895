// rt_cambuf.h — the camera buffer: per-tile triangle lists of the primary rays and
// their build kernels.
// Part of the device code of rt_kernels.hip (one translation unit: the
// kernels are templates instantiated by its host half); built with the
// same exactness flags (no FMA contraction, IEEE div/sqrt).
//
// What a list holds (unchanged since round 1): tile t of the full frame
// keeps triangle k iff the camera wave test of the per-wave path —
// cone_overlap(wc_t, c0_k, sinT_k) and the three edge planes, wc_t the
// wave cone of the tile's 64 camera rays (wave_cone on the clamped pixels,
// the trace kernel's own bits) — passes: the triangles the per-wave path
// would test exactly, so walking the list instead is exact.
//
// How it is built (round 3: binning by triangle, no host sync).  The test is
// evaluated only for (triangle, tile) pairs whose tile lies in the
// triangle's screen box — a box that provably contains every tile where the
// test can pass (cb_box below) — instead of every tile walking every
// cluster.  Per camera: rt_cb_tiles_boxes (the tile cones, the boxes) and a
// scan of their sizes (the candidate pairs), rt_cb_pairs<false> (the test
// of every pair: a count per tile, a pass mask per run of 64), a scan
// (offsets), rt_cb_pairs<true> (each passing pair at an atomic slot of its
// tile), rt_cb_keys_small / _wave / _long (order and early-exit keys) —
// one candidate pair per lane, only per-tile atomics.  The entry
// array has a fixed capacity chosen by the host from earlier builds; a tile
// whose list would end past it is flagged and takes the per-wave path (the
// same image), and the host grows the array once it reads the total back —
// so moving cameras rebuild on the stream, with no host round trip.
#ifndef RT_AMD_RT_CAMBUF_H
#define RT_AMD_RT_CAMBUF_H

#include "rt_cull.h"

#pragma clang fp contract(off)

namespace rt {

// ---------------------------------------------------------- camera buffer
// Does the frame's slab (or band set) cover any row of tile row ty?  Only
// those tiles get lists: a rank rendering 1/n of the frame builds 1/n of
// the buffer.  (Bands are multiples of 16 rows, so no tile straddles two.)
__device__ __forceinline__ bool cb_tile_row_needed(const FrameDev& F, int ty)
{
    if (F.band_rows > 0) return ((ty * 8) / F.band_rows) % F.band_count == F.band_index;
    return ty * 8 < F.row_end && ty * 8 + 8 > F.row_begin;
}

// Per-build device state (one per camera buffer: the context's, and one per
// sequence slot).  stat words: [1] candidate pairs, [3] lists longer than RT_CB_SORT (their tiles in
// lng[]), [4] the longest of them, [5] lists of 33..RT_CB_SORT entries
// (their tiles in mid[]), [6] 1: more than 2^32 - 1 candidate pairs (every
// tile flagged: the per-wave path).
struct CbDev {
    float4* __restrict__ tcone;   // 2 per tile: [w cosW] [sinW chord 0 0]
    unsigned* __restrict__ off;   // nt + 1: counts, scanned in place into offsets
    unsigned* __restrict__ cur;   // nt: fill cursors
    unsigned* __restrict__ flag;  // nt: 1 = no list (per-wave path)
    int2* __restrict__ ent;       // cap entries {triangle, dmin bits}
    int4* __restrict__ box;       // n_tri: triangle screen boxes (tx0, ty0, nx, tiles)
    unsigned* __restrict__ tcnt;  // n_tri + 1: box sizes, scanned in place into pair offsets
    unsigned long long* __restrict__ rmask;  // rcap: the count pass's pass mask per run of 64 pairs
    unsigned rcap;                // runs rmask holds (runs beyond: their tiles are flagged)
    int* __restrict__ lng;        // nt: tiles whose long lists rt_cb_keys_rest sorts in LDS
    int* __restrict__ mid;        // nt: tiles whose 33..256-entry lists rt_cb_keys_rest sorts
    unsigned* __restrict__ stat;  // 8 words (above)
    unsigned cap;                 // entries allocated
    int tiles_x, tiles_y;
    float wbound;                 // every listed tile's cone half-angle <= wbound (rad)
    float cos_wbound;             // >= cos(wbound): a tile with cosW below it gets no list
};

// The tile cones (one wave per tile of the full frame, 4 per workgroup):
// the trace kernel's own wave cone of the tile's 64 clamped pixels.  A tile
// outside the frame's rows, with a degenerate cone, or wider than the bound
// the boxes assume (cosW < cos_wbound; never seen: the bound is analytic)
// gets no list.  Also zeroes the counts and cursors.
__device__ __forceinline__ void cb_tiles_block(const FrameDev& F, const CbDev& B, unsigned blk)
{
    if (blk == 0 && threadIdx.x < 8) B.stat[threadIdx.x] = 0u;  // the build's counters
    const int lane = (int)(threadIdx.x & 63);
    const int t = (int)(blk * 4 + (threadIdx.x >> 6));
    const int nt = B.tiles_x * B.tiles_y;
    if (t >= nt) return;  // wave-uniform
    const int tx = t % B.tiles_x, ty = t / B.tiles_x;
    const bool present = cb_tile_row_needed(F, ty);
    WaveCone wc;
    wc.ok = false;
    if (present) {
        const int px = tx * 8 + (lane & 7), py = ty * 8 + (lane >> 3);
        const Vec3 D = camera_dir(F, px < F.width ? px : F.width - 1, py < F.height ? py : F.height - 1);
        wc = wave_cone(D, true);
    }
    const bool use = present && wc.ok && wc.cosW >= B.cos_wbound;
    if (lane == 0) {
        B.tcone[2 * t] = make_float4(wc.w.x, wc.w.y, wc.w.z, wc.cosW);
        B.tcone[2 * t + 1] = make_float4(wc.sinW, wc.chord, use ? 0.f : 1.f, 0.f);  // z: no list
        B.flag[t] = use ? 0u : 1u;
        B.off[t] = 0u;
        B.cur[t] = 0u;
    }
}

// The screen box of triangle k: tiles [tx0, tx0 + nx) x [ty0, ty0 + ny)
// containing every tile whose camera wave test with k can pass.
//
// Why.  With c0 = [a, cosT] (cosT > 0), the test passing means (float
// rounding included: dot, |w|, |a|, cosW/sinW/sinT margins, the 2e-6
// margin) cos angle(w, a) >= cos(W + T) - 4.4e-6, W = acos(cosW) <= wbound,
// T = acos(cosT), hence angle(w, a) <= acos(cos(T + wbound) - 4.4e-6)
// (at most T + wbound + 2.97e-3, at T + wbound = 0).  w is the direction of the tile's
// reference lane 36 = pixel (8tx + 4, 8ty + 4) clamped to the frame:
// normalize(d0 M), d0 = (X, Y, -1), X = (2 px inv_w - 1) half_w, likewise Y;
// M's rows r0 r1 r2 orthonormal to 1e-5 (checked by the host, which gives up
// the buffer otherwise) put w in camera coordinates as normalize(d0) within
// 2e-5.  So the reference pixel's d0 lies in the cone of half-angle
// Th = acos(cos(T + wbound) - 4.4e-6) + 3e-5 around a_c = (a.r0, a.r1, a.r2): the rays
// through the sphere of radius sin Th around the unit a_c.  Its extent in
// X = x / (-z) is that of the disk (a_c.x, a_c.z; sin Th) seen from the
// origin in the xz plane: the two tangents, when the disk misses the
// origin and both lie in front (z < 0; then so does the whole wedge, which
// is narrower than pi) — else the whole film.  Likewise Y.  Pixels from X by
// the inverse of the affine map, 2 pixels of slack each side; the tiles
// whose pixel ranges meet that span.  cosT <= 0 (an "always test" record)
// or Th >= 80 degrees: the whole film (then the edge planes alone, below).
struct CbBox {
    int tx0, ty0, nx, ny;
};
__host__ __device__ inline bool cb_span(double cx, double cz, double rho, double& lo, double& hi)
{
    const double d2 = cx * cx + cz * cz;
    if (!(d2 > rho * rho * (1.0 + 1e-9) + 1e-18)) return false;
    const double t = sqrt(d2 - rho * rho);
    const double ux1 = cx * t - cz * rho, uz1 = cx * rho + cz * t;
    const double ux2 = cx * t + cz * rho, uz2 = -cx * rho + cz * t;
    const double n1 = sqrt(ux1 * ux1 + uz1 * uz1), n2 = sqrt(ux2 * ux2 + uz2 * uz2);
    if (!(uz1 < -1e-9 * n1) || !(uz2 < -1e-9 * n2)) return false;
    const double s1 = ux1 / -uz1, s2 = ux2 / -uz2;
    lo = fmin(s1, s2);
    hi = fmax(s1, s2);
    return isfinite(lo) && isfinite(hi);
}
// tile range [t0, t1] of the pixels whose slope (X or Y) lies in [lo, hi]
// (the inverse of X = (2 px inv - 1) half, 2 pixels of slack each side).
__host__ __device__ inline void cb_tiles_of(double lo, double hi, float half, float inv, int npx, int ntiles,
                                            int& t0, int& t1)
{
    const double s = 1.0 / (2.0 * (double)inv);
    double p0 = floor((lo / (double)half + 1.0) * s) - 2.0, p1 = ceil((hi / (double)half + 1.0) * s) + 2.0;
    p0 = fmax(p0, 0.0);
    p1 = fmin(p1, (double)(npx - 1));
    if (!(p1 >= p0)) {
        t0 = 1;
        t1 = 0;
        return;
    }
    t0 = (int)(p0 / 8.0);
    const int t1p = (int)(p1 / 8.0);
    t1 = ntiles - 1 < t1p ? ntiles - 1 : t1p;
}
// Clip the convex polygon (x[i], y[i]), i < n, to a X + b Y >= c.
__host__ __device__ inline int cb_clip(double* x, double* y, int n, double a, double b, double c)
{
    double ox[8], oy[8];
    int m = 0;
    for (int i = 0; i < n; ++i) {
        const int j = i + 1 == n ? 0 : i + 1;
        const double fi = a * x[i] + b * y[i] - c, fj = a * x[j] + b * y[j] - c;
        if (fi >= 0.0 && m < 8) {
            ox[m] = x[i];
            oy[m] = y[i];
            ++m;
        }
        if ((fi >= 0.0) != (fj >= 0.0) && m < 8) {
            const double u = fi / (fi - fj);
            ox[m] = x[i] + u * (x[j] - x[i]);
            oy[m] = y[i] + u * (y[j] - y[i]);
            ++m;
        }
    }
    for (int i = 0; i < m; ++i) {
        x[i] = ox[i];
        y[i] = oy[i];
    }
    return m;
}
// The edge planes tighten the box (round 3): a tile passes only if
// edge_open holds for its reference direction w, i.e. (float rounding,
// w's 2e-5 from normalize(d0), chord <= wbound + 2e-6 included)
// w . n >= c = lim - wbound - 3.5e-5, so d0 = (X, Y, -1) with 1 <= |d0| <=
// Dm (the film's corner) satisfies d0 . n_c >= c |d0| >= (c < 0 ? c Dm :
// c): a half-plane of the film.  The box is that of the film rectangle
// (within the cone's span) clipped by the three half-planes.
__host__ __device__ inline CbBox cb_box(const float4 c0, const float4* e, const FrameDev& F, float wbound)
{
    const double hw = (double)F.half_w * (1.0 + 1e-6) + 1e-9, hh = (double)F.half_h * (1.0 + 1e-6) + 1e-9;
    double xlo = -hw, xhi = hw, ylo = -hh, yhi = hh;
    const double r[3][3] = {{F.orient[0], F.orient[1], F.orient[2]},
                            {F.orient[4], F.orient[5], F.orient[6]},
                            {F.orient[8], F.orient[9], F.orient[10]}};
    if (c0.w > 0.0f) {
        const double X = acos(fmin(1.0, (double)c0.w)) + (double)wbound;
        const double an = sqrt((double)c0.x * c0.x + (double)c0.y * c0.y + (double)c0.z * c0.z);
        if (X < 1.39 && an > 0.5 && isfinite(an)) {
            const double Th = acos(fmax(-1.0, cos(X) - 4.4e-6)) + 3e-5;  // + the orientation's 2e-5
            const double ax = c0.x / an, ay = c0.y / an, az = c0.z / an;
            const double cx = ax * r[0][0] + ay * r[0][1] + az * r[0][2];
            const double cy = ax * r[1][0] + ay * r[1][1] + az * r[1][2];
            const double cz = ax * r[2][0] + ay * r[2][1] + az * r[2][2];
            const double rho = sin(Th);
            double lo, hi;
            if (cb_span(cx, cz, rho, lo, hi)) {
                xlo = fmax(xlo, lo);
                xhi = fmin(xhi, hi);
            }
            if (cb_span(cy, cz, rho, lo, hi)) {
                ylo = fmax(ylo, lo);
                yhi = fmin(yhi, hi);
            }
            if (!(xlo <= xhi) || !(ylo <= yhi)) return CbBox{0, 0, 0, 0};
        }
    }
    double px[8] = {xlo, xhi, xhi, xlo}, py[8] = {ylo, ylo, yhi, yhi};
    int n = 4;
    const double Dm = sqrt(1.0 + hw * hw + hh * hh) * (1.0 + 1e-6);
    for (int q = 0; q < 3 && n > 0; ++q) {
        const float4 E = e[q];
        if (!(E.w > -3.0f)) continue;  // an always-open record
        const double nn = sqrt((double)E.x * E.x + (double)E.y * E.y + (double)E.z * E.z);
        if (!(nn > 0.5) || !isfinite(nn)) continue;
        const double nx = (E.x * r[0][0] + E.y * r[0][1] + E.z * r[0][2]) / nn;
        const double ny = (E.x * r[1][0] + E.y * r[1][1] + E.z * r[1][2]) / nn;
        const double nz = (E.x * r[2][0] + E.y * r[2][1] + E.z * r[2][2]) / nn;
        const double c = (double)E.w - (double)wbound - 3.5e-5;
        const double k = c < 0.0 ? c * Dm : c;
        n = cb_clip(px, py, n, nx, ny, k + nz);  // nx X + ny Y - nz >= k
    }
    if (n == 0) return CbBox{0, 0, 0, 0};
    double ax0 = px[0], ax1 = px[0], ay0 = py[0], ay1 = py[0];
    for (int i = 1; i < n; ++i) {
        ax0 = fmin(ax0, px[i]);
        ax1 = fmax(ax1, px[i]);
        ay0 = fmin(ay0, py[i]);
        ay1 = fmax(ay1, py[i]);
    }
    int x0, x1, y0, y1;
    cb_tiles_of(ax0, ax1, F.half_w, F.inv_w, F.width, (F.width + 7) / 8, x0, x1);
    cb_tiles_of(ay0, ay1, F.half_h, F.inv_h, F.height, (F.height + 7) / 8, y0, y1);
    if (x1 < x0 || y1 < y0) return CbBox{0, 0, 0, 0};
    return CbBox{x0, y0, x1 - x0 + 1, y1 - y0 + 1};
}

// The camera wave test of triangle k's records for tile t (cb_tiles_block's
// cone); false for a tile without a list.
__device__ __forceinline__ bool cb_pair_test(const CbDev& B, int t, const float4 c0, float sinT, const float4* e)
{
    const float4 a = B.tcone[2 * t], b = B.tcone[2 * t + 1];
    if (b.z != 0.0f) return false;
    WaveCone wc;
    wc.w = make3(a.x, a.y, a.z);
    wc.cosW = a.w;
    wc.sinW = b.x;
    wc.chord = b.y;
    wc.ok = true;
    return cone_overlap(wc, c0, sinT, 0.0f) && edges_open(wc, e, 0.0f);
}

// Small lists (no clusters, <= 1,024 triangles): one wave per tile tests
// every triangle, 64 per ballot — the binning's launches would cost more
// than this walk (C2: 12 triangles).  The tile's cone is cb_tiles_block's (and
// stored like it, for rt_debug_cb_verify); FILL false: the count, true: the
// entries in triangle order at the tile's offset (the keys sort them).
template <bool FILL>
__global__ __launch_bounds__(256) void rt_cb_walk(const SceneDev S, const FrameDev F, CbDev B)
{
    if (!FILL && blockIdx.x == 0 && threadIdx.x < 8) B.stat[threadIdx.x] = 0u;  // the build's counters
    const int lane = (int)(threadIdx.x & 63);
    const int t = (int)(blockIdx.x * 4 + (threadIdx.x >> 6));
    const int nt = B.tiles_x * B.tiles_y;
    if (t >= nt) return;  // wave-uniform
    const int tx = t % B.tiles_x, ty = t / B.tiles_x;
    const bool present = cb_tile_row_needed(F, ty);
    WaveCone wc;
    wc.ok = false;
    if (present) {
        const int px = tx * 8 + (lane & 7), py = ty * 8 + (lane >> 3);
        const Vec3 D = camera_dir(F, px < F.width ? px : F.width - 1, py < F.height ? py : F.height - 1);
        wc = wave_cone(D, true);
    }
    const bool use = present && wc.ok && wc.cosW >= B.cos_wbound;
    if (!FILL && lane == 0) {
        B.tcone[2 * t] = make_float4(wc.w.x, wc.w.y, wc.w.z, wc.cosW);
        B.tcone[2 * t + 1] = make_float4(wc.sinW, wc.chord, use ? 0.f : 1.f, 0.f);
        B.flag[t] = use ? 0u : 1u;
    }
    if (!use) {
        if (!FILL && lane == 0) B.off[t] = 0u;
        return;
    }
    unsigned n = 0, base = 0;
    if (FILL) {
        base = B.off[t];
        if (B.off[t + 1] > B.cap) {  // the list does not fit: the per-wave path
            if (lane == 0) B.flag[t] = 1u;
            return;
        }
    }
    const unsigned long long below = (1ull << lane) - 1ull;
    for (int k0 = 0; k0 < S.n_tri; k0 += 64) {
        const int k = k0 + lane;
        bool reach = false;
        float dmin = 0.0f;
        if (k < S.n_tri) {
            const float4 c0 = S.cone_cam[2 * k], c1 = S.cone_cam[2 * k + 1];
            dmin = c1.x;
            reach = cone_overlap(wc, c0, c1.w, 0.0f) && edges_open(wc, S.cone_cam + 2 * (size_t)S.n_tri + 3 * k, 0.0f);
        }
        const unsigned long long m = __ballot(reach);
        if (FILL && reach) B.ent[base + n + (unsigned)__popcll(m & below)] = make_int2(k, __float_as_int(dmin));
        n += (unsigned)__popcll(m);
    }
    if (!FILL && lane == 0) B.off[t] = n;
}

// Triangle boxes (one thread per triangle): box[k] = (tx0, ty0, nx, nx*ny),
// tcnt[k] = nx * ny, the candidate pairs the pair passes expand.
__device__ __forceinline__ void cb_boxes_block(const SceneDev& S, const FrameDev& F, const CbDev& B, unsigned blk)
{
    const int k = (int)(blk * 256 + threadIdx.x);
    if (k >= S.n_tri) return;
    const float4* e = S.cone_cam + 2 * (size_t)S.n_tri + 3 * (size_t)k;
    const float4 e3[3] = {e[0], e[1], e[2]};
    const CbBox b = cb_box(S.cone_cam[2 * k], e3, F, B.wbound);
    const unsigned n = (unsigned)(b.nx * b.ny);
    B.box[k] = make_int4(b.tx0, b.ty0, b.nx, (int)n);
    B.tcnt[k] = n;
}

// One launch for both (they are independent): the boxes' blocks first
// (fewer, each a long chain of double-precision steps per thread), then the
// tile cones' — one launch less per camera, and the tiles fill the machine
// while the boxes' few waves run (rocprofv3, C3: 8 + 25 us in series).
__global__ __launch_bounds__(256) void rt_cb_tiles_boxes(const SceneDev S, const FrameDev F, CbDev B, unsigned nbb)
{
    if (blockIdx.x < nbb) cb_boxes_block(S, F, B, blockIdx.x);
    else cb_tiles_block(F, B, blockIdx.x - nbb);
}

// One run of 64 pairs for the calling wave: each lane's owner triangle
// (searched from lo, which moves to the run's last owner), its tile and
// dmin; pass = the camera wave test (COUNT) or the run's pass-mask bit.
template <bool FILL>
__device__ __forceinline__ bool cb_run(const SceneDev& S, const CbDev& B, unsigned run, unsigned np,
                                       unsigned long long mask, int& lo, int& own, int& t, float& dmin)
{
    const int lane = (int)(threadIdx.x & 63);
    const unsigned p = run * 64 + (unsigned)lane;
    own = -1;
    for (int base = lo; base < S.n_tri; base += 64) {
        // window of 64 owners: lane j holds pre[base + j]
        const int kj = base + lane;
        const unsigned pj = kj < S.n_tri ? B.tcnt[kj] : 0xFFFFFFFFu;
        // my owner in this window: the last j with pre[base + j] <= p
        int j = (unsigned)__shfl((int)pj, 0) <= p ? 0 : -1;
        for (int step = 32; step > 0; step >>= 1) {
            const int c = j + step;
            const unsigned pc = (unsigned)__shfl((int)pj, c & 63);
            if (c <= 63 && pc <= p) j = c;
        }
        // j = 63 with the next window's first prefix <= p: look further
        const bool beyond = j == 63 && base + 64 < S.n_tri && B.tcnt[base + 64] <= p;
        if (own < 0 && j >= 0 && !beyond) own = base + j;
        if (!__any(own < 0 && p < np)) break;
    }
    // the next run starts at this run's last owner
    lo = __builtin_amdgcn_readlane(own < 0 ? lo : own, 63);
    bool pass = false;
    t = 0;
    dmin = 0.0f;
    if (p < np && own >= 0 && ((mask >> lane) & 1ull)) {
        const int k = own;
        const int4 bx = B.box[k];
        const unsigned q = p - B.tcnt[k];
        t = (bx.y + (int)(q / (unsigned)bx.z)) * B.tiles_x + bx.x + (int)(q % (unsigned)bx.z);
        const float4 c1 = S.cone_cam[2 * k + 1];
        dmin = c1.x;
        pass = FILL || cb_pair_test(B, t, S.cone_cam[2 * k], c1.w, S.cone_cam + 2 * (size_t)S.n_tri + 3 * (size_t)k);
    }
    return pass;
}

// One pass over every candidate (triangle, tile) pair, one pair per lane:
// a fixed grid of waves, each taking a contiguous range of runs of 64
// consecutive pairs (the pairs of triangle k are [pre[k], pre[k + 1]), pre
// = the exclusive scan of the box sizes).  The range's first owner comes
// from a 64-way ballot search over pre[]; every run then finds its lanes' owners
// among the next 64 triangles' prefixes (a search over lanes by shuffles;
// another window for runs that cross more than 64 triangles), starting
// from the previous run's last owner.
// Count pass (FILL false): the camera wave test of each pair, a count per
// passing pair's tile, and the run's pass mask (one word per run).  Fill
// pass: only runs with passing pairs, only their passing lanes — each at the
// next slot of its tile (a tile whose list would end past the capacity is
// flagged instead: the per-wave path).  Only per-tile counters are atomic:
// no global counter to serialise on.
// total (count pass): the box-size scan's 64-bit total (the fill pass, after
// the offsets' scan reused the scratch, reads the count pass's stat[6]).  The
// pair offsets are 32-bit: a
// camera with more than 2^32 - 1 candidate pairs (whole-film boxes of many
// "always test" triangles at a high tile count) would wrap them, so then no
// pair is tested — every tile is flagged (the per-wave path: the same image)
// and stat[6] tells the host.
template <bool FILL>
__global__ __launch_bounds__(256) void rt_cb_pairs(const SceneDev S, CbDev B, const unsigned long long* __restrict__ total)
{
    const int lane = (int)(threadIdx.x & 63);
    const unsigned nw = gridDim.x * (blockDim.x >> 6);
    const unsigned w = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    if (FILL ? B.stat[6] != 0u : *total > 0xFFFFFFFFull) {
        if (!FILL) {
            const unsigned nt = (unsigned)(B.tiles_x * B.tiles_y);
            for (unsigned t = w * 64 + (unsigned)lane; t < nt; t += nw * 64) B.flag[t] = 1u;
            if (w == 0 && lane == 0) B.stat[6] = 1u;
        }
        return;
    }
    const unsigned np = B.tcnt[S.n_tri];  // total candidate pairs (the scan's last word)
    const unsigned nruns = (np + 63) / 64, per = (nruns + nw - 1) / nw;
    const unsigned r0 = w * per, r1 = min(nruns, r0 + per);
    if (r0 >= r1) return;  // wave-uniform
    if (!FILL && lane == 0 && w == 0) B.stat[1] = np;
    // the last k with pre[k] <= p0 (wave-uniform): a 64-way search, each
    // round one load per lane and a ballot (3 rounds for 50k triangles,
    // instead of a binary search's 16 dependent loads)
    int lo = 0;
    {
        int span = S.n_tri;  // pre[lo] <= p0, and the answer lies in [lo, lo + span)
        const unsigned p0 = r0 * 64;
        while (span > 1) {
            const int step = (span + 63) / 64;
            const int k = lo + lane * step;
            const bool le = lane == 0 || (k < lo + span && k < S.n_tri && B.tcnt[k] <= p0);
            const unsigned long long m = __ballot(le);
            const int j = 63 - (int)__builtin_clzll(m);  // the last lane whose probe is <= p0 (pre is non-decreasing)
            lo += j * step;
            span = min(step, span - j * step);
        }
    }
    for (unsigned run = r0; run < r1; ++run) {
        unsigned long long mask = ~0ull;
        if (FILL) {
            if (run >= B.rcap) continue;  // no mask kept: its tiles were flagged
            mask = B.rmask[run];
            if (!mask) continue;  // no passing pair: nothing to place (wave-uniform)
        }
        int own, t;
        float dmin;
        const bool pass = cb_run<FILL>(S, B, run, np, mask, lo, own, t, dmin);
        if (!FILL) {
            const unsigned long long m = __ballot(pass);
            if (run < B.rcap) {
                if (lane == 0) B.rmask[run] = m;
                if (pass) atomicAdd(&B.off[t], 1u);
            } else if (pass) {
                B.flag[t] = 1u;  // past the mask capacity: the per-wave path
            }
        } else if (pass) {
            if (B.off[t + 1] > B.cap) {
                B.flag[t] = 1u;
            } else {
                const unsigned slot = B.off[t] + atomicAdd(&B.cur[t], 1u);
                B.ent[slot] = make_int2(own, __float_as_int(dmin));
            }
        }
    }
}

// Keys: entry e's key = min dmin over entries [e, end) of its tile, so a
// wave may stop at the first key beyond its hits.  Lists of up to
// RT_CB_SORT entries are first sorted nearest-first (the closest hit is
// order-free: lexicographic (t, index)), so the keys rise with the walk and
// the exit comes at the first entry beyond every lane's hit.
#ifndef RT_CB_SORT
#define RT_CB_SORT 256
#endif
__device__ __forceinline__ float cb_dmin(int2 en)
{
    const float d = __int_as_float(en.y);
    return d == d ? d : -INFINITY;
}

// Order-preserving 64-bit sort key of an entry: the dmin's float bits
// mapped to an unsigned order (NaN as -inf), then the triangle.
__device__ __forceinline__ unsigned long long cb_sort_key(int2 e)
{
    unsigned u = __float_as_uint(cb_dmin(e));
    u = (u & 0x80000000u) ? ~u : (u | 0x80000000u);
    return ((unsigned long long)u << 32) | (unsigned)e.x;
}
__device__ __forceinline__ int2 cb_unkey(unsigned long long key)
{
    unsigned u = (unsigned)(key >> 32);
    u = (u & 0x80000000u) ? (u & 0x7fffffffu) : ~u;
    return make_int2((int)(unsigned)key, (int)u);
}
// A list of up to N entries sorted in registers by a bitonic network (the
// indices are constants after unrolling; padding keys sort last).
template <int N>
__device__ __forceinline__ void cb_sort_regs(int2* __restrict__ ent, unsigned b, unsigned n)
{
    unsigned long long a[N];
#pragma unroll
    for (int i = 0; i < N; ++i) a[i] = (unsigned)i < n ? cb_sort_key(ent[b + i]) : ~0ull;
#pragma unroll
    for (int k = 2; k <= N; k <<= 1)
#pragma unroll
        for (int j = k >> 1; j > 0; j >>= 1)
#pragma unroll
            for (int i = 0; i < N; ++i) {
                const int l = i ^ j;
                if (l > i) {
                    const unsigned long long x = a[i], y = a[l];
                    const bool sw = ((i & k) == 0) ? (x > y) : (x < y);
                    a[i] = sw ? y : x;
                    a[l] = sw ? x : y;
                }
            }
#pragma unroll
    for (int i = 0; i < N; ++i)
        if ((unsigned)i < n) ent[b + i] = cb_unkey(a[i]);
}

// Rank sort of one list of up to 64 Q entries by a wave, Q per lane in
// registers: every entry's final place is its rank under (dmin, triangle).
template <int Q>
__device__ __forceinline__ void cb_sort_rank_q(int2* __restrict__ ent, unsigned b, unsigned n)
{
    const int lane = threadIdx.x & 63;
    float kd[Q];
    int id[Q];
    unsigned rk[Q];
#pragma unroll
    for (int q = 0; q < Q; ++q) {
        const unsigned i = (unsigned)(lane + 64 * q);
        kd[q] = INFINITY;
        id[q] = 0x7fffffff;
        rk[q] = 0;
        if (i < n) {
            const int2 e = ent[b + i];
            kd[q] = cb_dmin(e);
            id[q] = e.x;
        }
    }
#pragma unroll
    for (int qq = 0; qq < Q; ++qq) {
        const int lim = (int)min(64u, n - 64u * (unsigned)qq);
        for (int j = 0; j < lim; ++j) {
            const float kj = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(kd[qq]), j));
            const int ij = __builtin_amdgcn_readlane(id[qq], j);
#pragma unroll
            for (int q = 0; q < Q; ++q) rk[q] += (unsigned)((kj < kd[q]) | ((kj == kd[q]) & (ij < id[q])));
        }
    }
#pragma unroll
    for (int q = 0; q < Q; ++q)
        if ((unsigned)(lane + 64 * q) < n) ent[b + rk[q]] = make_int2(id[q], __float_as_int(kd[q]));
}
__device__ __forceinline__ void rt_cb_sort_rank(const CbDev& B, int t)
{
    const unsigned b = B.off[t], n = B.off[t + 1] - b;
    if (n <= 64)
        cb_sort_rank_q<1>(B.ent, b, n);
    else if (n <= 128)
        cb_sort_rank_q<2>(B.ent, b, n);
    else
        cb_sort_rank_q<4>(B.ent, b, n);
}

// Keys, one thread per tile (round 3: the per-tile wave cost ~1.6 us of
// latency per tile at 7680 x 4320): lists of up to 32 entries are sorted in
// registers; longer ones are queued for rt_cb_keys_rest.  Once sorted, each entry's suffix minimum is its own
// dmin, which the entry already holds.  Flagged tiles (no list, or
// overflowed) are skipped.
__global__ __launch_bounds__(256) void rt_cb_keys_small(const CbDev B, int ntiles)
{
    const int t = (int)(blockIdx.x * blockDim.x + threadIdx.x);
    if (t >= ntiles || B.flag[t]) return;
    const unsigned b = B.off[t], n = B.off[t + 1] - b;
    if (n <= 1) {
        if (n == 1) B.ent[b].y = __float_as_int(cb_dmin(B.ent[b]));
    } else if (n <= 8) {
        cb_sort_regs<8>(B.ent, b, n);
    } else if (n <= 16) {
        cb_sort_regs<16>(B.ent, b, n);
    } else if (n <= 32) {
        cb_sort_regs<32>(B.ent, b, n);
    } else if (n <= RT_CB_SORT) {
        B.mid[atomicAdd(&B.stat[5], 1u)] = t;
    } else {
        B.lng[atomicAdd(&B.stat[3], 1u)] = t;
        atomicMax(&B.stat[4], n);
    }
}

// The lists rt_cb_keys_small queued, one launch for both kinds:
// * 33..RT_CB_SORT (256) entries: one wave per tile, held in registers (up
//   to 4 per lane), every entry's final place is its rank under (dmin,
//   triangle) — the pairs are distinct (NaN dmins sort first as -inf);
// * longer: one workgroup per tile, a bitonic sort in LDS (up to kCbLongCap
//   entries; a longer list keeps its fill order with suffix-minimum keys —
//   exact, the early exit only later).
// A fixed grid walks both queues (the host does not know their lengths).
// Thread 0 of block 0 also publishes the build's total and counters to the
// host (hout, pinned and device-visible), which reads them after the build's
// event: no copy commands.
constexpr int kCbLongCap = 4096;
__global__ __launch_bounds__(256) void rt_cb_keys_rest(const CbDev B, const unsigned long long* __restrict__ total,
                                                       unsigned long long* hout)
{
    __shared__ unsigned long long sk[kCbLongCap];  // (dmin order bits << 32) | triangle
    if (hout && blockIdx.x == 0 && threadIdx.x == 0) {
        hout[0] = *total;
        for (int i = 0; i < 4; ++i)
            hout[1 + i] = (unsigned long long)B.stat[2 * i] | ((unsigned long long)B.stat[2 * i + 1] << 32);
        __threadfence_system();
    }
    const unsigned nq = B.stat[5];
    const unsigned nw = gridDim.x * 4, w0 = blockIdx.x * 4 + (threadIdx.x >> 6);
    for (unsigned qi = w0; qi < nq; qi += nw) rt_cb_sort_rank(B, B.mid[qi]);
    const unsigned* __restrict__ off = B.off;
    int2* __restrict__ ent = B.ent;
    const unsigned nlong = B.stat[3];
    for (unsigned i = blockIdx.x; i < nlong; i += gridDim.x) {  // block-uniform
        const int t = B.lng[i];
        const unsigned b = off[t], n = off[t + 1] - b;
        if (n > (unsigned)kCbLongCap) {
            if (threadIdx.x == 0) {
                float m = INFINITY;
                for (unsigned e = b + n; e > b; --e) {
                    const float d = __int_as_float(ent[e - 1].y);
                    m = d == d ? fminf(m, d) : -INFINITY;
                    ent[e - 1].y = __float_as_int(m);
                }
            }
            continue;
        }
        unsigned P = 1;
        while (P < n) P <<= 1;
        __syncthreads();
        for (unsigned q = threadIdx.x; q < P; q += blockDim.x) sk[q] = q < n ? cb_sort_key(ent[b + q]) : ~0ull;
        __syncthreads();
        for (unsigned kk = 2; kk <= P; kk <<= 1) {
            for (unsigned j = kk >> 1; j > 0; j >>= 1) {
                for (unsigned q = threadIdx.x; q < P; q += blockDim.x) {
                    const unsigned l = q ^ j;
                    if (l > q) {
                        const unsigned long long x = sk[q], y = sk[l];
                        const bool up = (q & kk) == 0;
                        if ((x > y) == up) {
                            sk[q] = y;
                            sk[l] = x;
                        }
                    }
                }
                __syncthreads();
            }
        }
        for (unsigned q = threadIdx.x; q < n; q += blockDim.x) ent[b + q] = cb_unkey(sk[q]);
    }
}

// The walk's records: entry e = the tricam record of its triangle, key in
// [3].z (tricam's [3] = [e2 . Q, file index, 0, 0]).  One thread per entry
// of the capacity; entries past the build's total are left alone.
__global__ void rt_cb_expand(const int2* __restrict__ ent, const unsigned long long* __restrict__ total,
                             unsigned cap, const float4* __restrict__ tricam, float4* __restrict__ rec)
{
    const unsigned e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= cap || (unsigned long long)e >= *total) return;
    const int2 en = ent[e];
    const float4* t = tricam + 4 * (size_t)en.x;
    float4* o = rec + 4 * (size_t)e;
    o[0] = t[0];
    o[1] = t[1];
    o[2] = t[2];
    float4 d = t[3];
    d.z = __int_as_float(en.y);
    o[3] = d;
}

// Diagnostic (rt_debug_cb_verify): a built camera buffer against brute
// force — every tile with a list against every triangle.  A tile is bad
// unless its list holds exactly the triangles whose camera wave test passes
// (as many entries as passing triangles, every entry passing: the binning
// never emits a pair twice), keyed by its own dmin, keys non-decreasing for
// sorted lists.  out[0] += bad tiles, out[1] += passing pairs.
__global__ __launch_bounds__(256) void rt_cb_verify(const SceneDev S, const CbDev B, unsigned* __restrict__ out)
{
    const int lane = (int)(threadIdx.x & 63);
    const int t = (int)(blockIdx.x * 4 + (threadIdx.x >> 6));
    if (t >= B.tiles_x * B.tiles_y || B.flag[t]) return;
    unsigned n = 0;
    for (int k0 = 0; k0 < S.n_tri; k0 += 64) {
        const int k = k0 + lane;
        bool pass = false;
        if (k < S.n_tri)
            pass = cb_pair_test(B, t, S.cone_cam[2 * k], S.cone_cam[2 * k + 1].w,
                                S.cone_cam + 2 * (size_t)S.n_tri + 3 * (size_t)k);
        n += (unsigned)__popcll(__ballot(pass));
    }
    const unsigned b = B.off[t], m = B.off[t + 1] - b;
    bool bad = m != n;
    for (unsigned i0 = 0; i0 < m; i0 += 64) {
        const unsigned i = i0 + (unsigned)lane;
        bool wrong = false;
        if (i < m) {
            const int2 e = B.ent[b + i];
            if (e.x < 0 || e.x >= S.n_tri) {
                wrong = true;
            } else {
                const float4 c1 = S.cone_cam[2 * e.x + 1];
                wrong = !cb_pair_test(B, t, S.cone_cam[2 * e.x], c1.w,
                                      S.cone_cam + 2 * (size_t)S.n_tri + 3 * (size_t)e.x);
                const float d = cb_dmin(make_int2(0, __float_as_int(c1.x)));
                if (m <= (unsigned)kCbLongCap) {
                    wrong |= __float_as_int(d) != e.y;
                    if (i + 1 < m) wrong |= !(__int_as_float(e.y) <= __int_as_float(B.ent[b + i + 1].y));
                }
            }
        }
        bad |= __any(wrong);
    }
    if (lane == 0) {
        atomicAdd(&out[1], n);
        if (bad) atomicAdd(&out[0], 1u);
    }
}

}  // namespace rt
#endif  // RT_AMD_RT_CAMBUF_H
