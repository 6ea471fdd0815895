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
// cluster.  Per camera: rt_cb_tiles (the tile cones), rt_cb_bin<false> /
// rt_cb_bin_big<false> (counts per tile), a device scan (offsets),
// rt_cb_bin<true> / rt_cb_bin_big<true> (the entries, each at an atomic slot
// of its tile), rt_cb_keys_wave (order and early-exit keys).  The entry
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
// sequence slot).  stat words: [0] triangles deferred to rt_cb_bin_big,
// [1] (triangle, tile) pairs tested, [2] (unused), [3] lists longer than
// RT_CB_SORT (their tiles in lng[]), [4] the longest of them.
struct CbDev {
    float4* __restrict__ tcone;   // 2 per tile: [w cosW] [sinW chord 0 0]
    unsigned* __restrict__ off;   // nt + 1: counts, scanned in place into offsets
    unsigned* __restrict__ cur;   // nt: fill cursors
    unsigned* __restrict__ flag;  // nt: 1 = no list (per-wave path)
    int2* __restrict__ ent;       // cap entries {triangle, dmin bits}
    int* __restrict__ big;        // n_tri: triangles deferred to the grid-wide pass
    int* __restrict__ lng;        // nt: tiles whose lists rt_cb_keys_long sorts
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
__global__ __launch_bounds__(256) void rt_cb_tiles(const FrameDev F, CbDev B)
{
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
    if (lane == 0) {
        B.tcone[2 * t] = make_float4(wc.w.x, wc.w.y, wc.w.z, wc.cosW);
        B.tcone[2 * t + 1] = make_float4(wc.sinW, wc.chord, 0.f, 0.f);
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
// T = acos(cosT), hence angle(w, a) <= T + wbound + 2.97e-3 (the worst case,
// at W + T = 0, is sqrt(2 * 4.4e-6)).  w is the direction of the tile's
// reference lane 36 = pixel (8tx + 4, 8ty + 4) clamped to the frame:
// normalize(d0 M), d0 = (X, Y, -1), X = (2 px inv_w - 1) half_w, likewise Y;
// M's rows r0 r1 r2 orthonormal to 1e-5 (checked by the host, which gives up
// the buffer otherwise) put w in camera coordinates as normalize(d0) within
// 2e-5.  So the reference pixel's d0 lies in the cone of half-angle
// Th = T + wbound + 6.2e-3 around a_c = (a.r0, a.r1, a.r2): the rays
// through the sphere of radius sin Th around the unit a_c.  Its extent in
// X = x / (-z) is that of the disk (a_c.x, a_c.z; sin Th) seen from the
// origin in the xz plane: the two tangents, when the disk misses the
// origin and both lie in front (z < 0; then so does the whole wedge, which
// is narrower than pi) — else every column.  Likewise Y.  Pixels from X by
// the inverse of the affine map, 2 pixels of slack each side; the tiles
// whose pixel ranges meet that span.  cosT <= 0 (an "always test" record)
// or Th >= 80 degrees: every tile.
struct CbBox {
    int tx0, ty0, nx, ny;
};
__device__ __forceinline__ bool cb_span(double cx, double cz, double rho, double& lo, double& hi)
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
// tile range [t0, t1] of a pixel span from slope span [lo, hi] (X or Y).
__device__ __forceinline__ void cb_tiles_of(bool bounded, double lo, double hi, float half, float inv, int npx,
                                            int ntiles, int& t0, int& t1)
{
    t0 = 0;
    t1 = ntiles - 1;
    if (!bounded) return;
    const double s = 1.0 / (2.0 * (double)inv);
    double p0 = floor((lo / (double)half + 1.0) * s) - 2.0, p1 = ceil((hi / (double)half + 1.0) * s) + 2.0;
    p0 = fmax(p0, 0.0);
    p1 = fmin(p1, (double)(npx - 1));
    if (p1 < p0) {
        t0 = 1;
        t1 = 0;
        return;
    }
    t0 = (int)(p0 / 8.0);
    t1 = min(ntiles - 1, (int)(p1 / 8.0));
}
__device__ __forceinline__ CbBox cb_box(const float4 c0, const FrameDev& F, const CbDev& B)
{
    CbBox b{0, 0, B.tiles_x, B.tiles_y};
    if (!(c0.w > 0.0f)) return b;  // always tested: every tile
    const double Th = acos(fmin(1.0, (double)c0.w)) + (double)B.wbound + 6.2e-3;
    if (!(Th < 1.396)) return b;
    const double an = sqrt((double)c0.x * c0.x + (double)c0.y * c0.y + (double)c0.z * c0.z);
    if (!(an > 0.5) || !isfinite(an)) return b;
    const double ax = c0.x / an, ay = c0.y / an, az = c0.z / an;
    const double cx = ax * F.orient[0] + ay * F.orient[1] + az * F.orient[2];
    const double cy = ax * F.orient[4] + ay * F.orient[5] + az * F.orient[6];
    const double cz = ax * F.orient[8] + ay * F.orient[9] + az * F.orient[10];
    const double rho = sin(Th);
    double xlo = 0, xhi = 0, ylo = 0, yhi = 0;
    const bool bx = cb_span(cx, cz, rho, xlo, xhi);
    const bool by = cb_span(cy, cz, rho, ylo, yhi);
    int x0, x1, y0, y1;
    cb_tiles_of(bx, xlo, xhi, F.half_w, F.inv_w, F.width, B.tiles_x, x0, x1);
    cb_tiles_of(by, ylo, yhi, F.half_h, F.inv_h, F.height, B.tiles_y, y0, y1);
    if (x1 < x0 || y1 < y0) return CbBox{0, 0, 0, 0};
    return CbBox{x0, y0, x1 - x0 + 1, y1 - y0 + 1};
}

// The camera wave test of triangle k's records for tile t (rt_cb_tiles' cone).
__device__ __forceinline__ bool cb_pair_test(const CbDev& B, int t, const float4 c0, float sinT, const float4* e)
{
    const float4 a = B.tcone[2 * t], b = B.tcone[2 * t + 1];
    WaveCone wc;
    wc.w = make3(a.x, a.y, a.z);
    wc.cosW = a.w;
    wc.sinW = b.x;
    wc.chord = b.y;
    wc.ok = true;
    return cone_overlap(wc, c0, sinT, 0.0f) && edges_open(wc, e, 0.0f);
}
// One passing pair: count it (FILL false), or write its entry at its tile's
// next slot — unless the tile's list would end past the capacity: then the
// tile is flagged (no list: the per-wave path) and nothing is written.
template <bool FILL>
__device__ __forceinline__ void cb_emit(const CbDev& B, int t, int k, float dmin)
{
    if (!FILL) {
        atomicAdd(&B.off[t], 1u);
        return;
    }
    const unsigned e1 = B.off[t + 1];
    if (e1 > B.cap) {
        B.flag[t] = 1u;
        return;
    }
    const unsigned slot = B.off[t] + atomicAdd(&B.cur[t], 1u);
    B.ent[slot] = make_int2(k, __float_as_int(dmin));
}

// Boxes up to this many tiles are binned by their own wave (rt_cb_bin);
// larger ones (an always-tested record, a triangle near the camera) by the
// whole grid (rt_cb_bin_big), so no wave walks a long box alone.
constexpr int kCbWaveTiles = 2048;

// One wave per 64 consecutive triangles (4 waves per workgroup): each lane
// boxes its triangle; the wave then walks the concatenation of the 64 boxes
// one pair per lane per step (the owner of pair p by a binary search over
// the boxes' prefix sums in LDS), so a step tests 64 pairs whatever the box
// sizes.  FILL false: count per tile and defer the big boxes; true: write.
template <bool FILL>
__global__ __launch_bounds__(256) void rt_cb_bin(const SceneDev S, const FrameDev F, CbDev B)
{
    __shared__ float4 rec[4][64][5];
    __shared__ int box[4][64][3];  // tx0, ty0, nx
    __shared__ unsigned incl[4][64];
    const int lane = (int)(threadIdx.x & 63), wv = (int)(threadIdx.x >> 6);
    const int k = (int)((blockIdx.x * 4 + wv) * 64) + lane;
    unsigned n = 0;
    if (k < S.n_tri) {
        const float4 c0 = S.cone_cam[2 * k];
        const CbBox b = cb_box(c0, F, B);
        n = (unsigned)(b.nx * b.ny);
        if (n > (unsigned)kCbWaveTiles) {
            if (!FILL) B.big[atomicAdd(&B.stat[0], 1u)] = k;
            n = 0;
        }
        if (n) {
            rec[wv][lane][0] = c0;
            rec[wv][lane][1] = S.cone_cam[2 * k + 1];
            const float4* e = S.cone_cam + 2 * (size_t)S.n_tri + 3 * (size_t)k;
            rec[wv][lane][2] = e[0];
            rec[wv][lane][3] = e[1];
            rec[wv][lane][4] = e[2];
            box[wv][lane][0] = b.tx0;
            box[wv][lane][1] = b.ty0;
            box[wv][lane][2] = b.nx;
        }
    }
    // inclusive prefix of the box sizes over the wave
    unsigned v = n;
    for (int o = 1; o < 64; o <<= 1) {
        const unsigned u = __shfl_up(v, o);
        if (lane >= o) v += u;
    }
    incl[wv][lane] = v;
    const unsigned total = (unsigned)__shfl(v, 63);
    wave_lds_sync();
    if (!FILL && lane == 0 && total) atomicAdd(&B.stat[1], total);
    for (unsigned p0 = 0; p0 < total; p0 += 64) {
        const unsigned p = p0 + (unsigned)lane;
        if (p >= total) break;
        int lo = 0, hi = 63;  // the first owner with incl > p
        while (lo < hi) {
            const int mid = (lo + hi) >> 1;
            if (incl[wv][mid] > p)
                hi = mid;
            else
                lo = mid + 1;
        }
        const unsigned q = p - (lo ? incl[wv][lo - 1] : 0u);
        const int nx = box[wv][lo][2];
        const int t = (box[wv][lo][1] + (int)(q / (unsigned)nx)) * B.tiles_x + box[wv][lo][0] + (int)(q % (unsigned)nx);
        if (B.flag[t]) continue;
        const float4 c0 = rec[wv][lo][0], c1 = rec[wv][lo][1];
        if (cb_pair_test(B, t, c0, c1.w, &rec[wv][lo][2]))
            cb_emit<FILL>(B, t, (int)((blockIdx.x * 4 + wv) * 64) + lo, c1.x);
    }
}

// The deferred (big) boxes, by the whole grid: every thread takes pairs
// g, g + G, ... of each deferred triangle in turn.
template <bool FILL>
__global__ __launch_bounds__(256) void rt_cb_bin_big(const SceneDev S, const FrameDev F, CbDev B)
{
    const unsigned nbig = min(B.stat[0], (unsigned)S.n_tri);
    const unsigned G = gridDim.x * blockDim.x, g = blockIdx.x * blockDim.x + threadIdx.x;
    for (unsigned i = 0; i < nbig; ++i) {
        const int k = B.big[i];
        const float4 c0 = S.cone_cam[2 * k], c1 = S.cone_cam[2 * k + 1];
        const float4* e = S.cone_cam + 2 * (size_t)S.n_tri + 3 * (size_t)k;
        const float4 e3[3] = {e[0], e[1], e[2]};
        const CbBox b = cb_box(c0, F, B);
        const unsigned n = (unsigned)(b.nx * b.ny);
        if (!FILL && g == 0) atomicAdd(&B.stat[1], n);
        for (unsigned q = g; q < n; q += G) {
            const int t = (b.ty0 + (int)(q / (unsigned)b.nx)) * B.tiles_x + b.tx0 + (int)(q % (unsigned)b.nx);
            if (B.flag[t]) continue;
            if (cb_pair_test(B, t, c0, c1.w, e3)) cb_emit<FILL>(B, t, k, c1.x);
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

// One wave per tile: a list of up to RT_CB_SORT (256) entries is held in
// registers (4 per lane) and every entry's final place is its rank under
// (dmin, triangle) — the pairs are distinct; once sorted, the suffix minimum
// of entry e is its own dmin (NaN dmins sort first as -inf and key -inf).
// Longer lists are sorted in LDS by rt_cb_keys_long; flagged tiles (no list,
// or overflowed) are skipped.
__global__ __launch_bounds__(256) void rt_cb_keys_wave(const CbDev B, int ntiles)
{
    const unsigned* __restrict__ off = B.off;
    int2* __restrict__ ent = B.ent;
    const int lane = threadIdx.x & 63;
    const int t = blockIdx.x * 4 + (int)(threadIdx.x >> 6);
    if (t >= ntiles || B.flag[t]) return;
    const unsigned b = off[t], n = off[t + 1] - off[t];
    if (n <= 1) {
        if (n == 1 && lane == 0) ent[b].y = __float_as_int(cb_dmin(ent[b]));
        return;
    }
    if (n > RT_CB_SORT) {
        if (lane == 0) {
            B.lng[atomicAdd(&B.stat[3], 1u)] = t;
            atomicMax(&B.stat[4], n);
        }
        return;
    }
    float kd[4];
    int id[4];
    unsigned rk[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
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
    for (int qq = 0; qq < 4; ++qq) {
        if ((unsigned)(64 * qq) >= n) break;
        const int lim = (int)min(64u, n - 64u * (unsigned)qq);
        for (int j = 0; j < lim; ++j) {
            const float kj = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(kd[qq]), j));
            const int ij = __builtin_amdgcn_readlane(id[qq], j);
#pragma unroll
            for (int q = 0; q < 4; ++q) rk[q] += (unsigned)((kj < kd[q]) | ((kj == kd[q]) & (ij < id[q])));
        }
    }
#pragma unroll
    for (int q = 0; q < 4; ++q)
        if ((unsigned)(lane + 64 * q) < n) ent[b + rk[q]] = make_int2(id[q], __float_as_int(kd[q]));
}

// Lists longer than RT_CB_SORT (their tiles listed by rt_cb_keys_wave):
// one workgroup per such tile sorts the list by (dmin, triangle) with a
// bitonic sort in LDS (up to kCbLongCap entries; a longer list keeps its fill
// order with suffix-minimum keys — exact, the early exit only later).  A
// fixed grid walks the listed tiles (the host does not know how many).
constexpr int kCbLongCap = 4096;
__global__ __launch_bounds__(1024) void rt_cb_keys_long(const CbDev B)
{
    __shared__ unsigned long long sk[kCbLongCap];  // (dmin order bits << 32) | triangle
    const unsigned* __restrict__ off = B.off;
    int2* __restrict__ ent = B.ent;
    const unsigned nlong = B.stat[3];
    for (unsigned i = blockIdx.x; i < nlong; i += gridDim.x) {
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
        for (unsigned i = threadIdx.x; i < P; i += blockDim.x) {
            unsigned long long key = ~0ull;
            if (i < n) {
                const int2 e = ent[b + i];
                // order-preserving bits of the float key (NaN as -inf)
                unsigned u = __float_as_uint(cb_dmin(e));
                u = (u & 0x80000000u) ? ~u : (u | 0x80000000u);
                key = ((unsigned long long)u << 32) | (unsigned)e.x;
            }
            sk[i] = key;
        }
        __syncthreads();
        for (unsigned kk = 2; kk <= P; kk <<= 1) {
            for (unsigned j = kk >> 1; j > 0; j >>= 1) {
                for (unsigned i = threadIdx.x; i < P; i += blockDim.x) {
                    const unsigned l = i ^ j;
                    if (l > i) {
                        const unsigned long long x = sk[i], y = sk[l];
                        const bool up = (i & kk) == 0;
                        if ((x > y) == up) {
                            sk[i] = y;
                            sk[l] = x;
                        }
                    }
                }
                __syncthreads();
            }
        }
        for (unsigned i = threadIdx.x; i < n; i += blockDim.x) {
            const unsigned long long key = sk[i];
            unsigned u = (unsigned)(key >> 32);
            u = (u & 0x80000000u) ? (u & 0x7fffffffu) : ~u;
            ent[b + i] = make_int2((int)(unsigned)key, (int)u);
        }
        __syncthreads();
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
