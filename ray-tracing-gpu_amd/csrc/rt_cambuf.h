// rt_cambuf.h — the camera buffer: per-tile triangle lists of the primary rays and
// their build kernels.
// Part of the device code of rt_kernels.hip (one translation unit: the
// kernels are templates instantiated by its host half); built with the
// same exactness flags (no FMA contraction, IEEE div/sqrt).
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
    if (!cb_tile_row_needed(F, ty)) {  // outside the frame's rows: no list
        if (!FILL && lane == 0) {
            flag[tile] = 1u;
            cnt[tile] = 0u;
        }
        return;
    }
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

// ------------------------------------------------ block pre-cull (big lists)
// rt_cb_build walks every cluster for every tile: at C5 (518k tiles, 782
// clusters) that is most of the camera buffer's cost, and the same cluster
// and member records are read by every tile.  rt_cb_block does it once per
// block of 8 x 8 tiles: one workgroup computes the 64 tile cones (the
// tiles' own wave_cone, bit for bit), a block cone that contains them all,
// culls clusters and members against the block cone into a list staged in
// LDS (member ids and cone records, cluster order), and then tests each tile
// against that list with the tile kernel's own predicate.
//
// Why the block list is a superset of every tile's (so each tile's list is
// exactly rt_cb_build's, same entries, same order): a tile keeps member k
// when (float) w_t.a >= c_t cT - s_t sT - 2e-6 (cone_overlap) and its edge
// planes are open.  With W_t = acos(c_t), s_t <= sin W_t + 1.1e-6 and the
// record's sT >= sin T, that implies cos(theta_t) >= cos(W_t + T) - m, m =
// 5e-6 (rounding included), theta_t = angle(w_t, a); so theta_t exceeds
// W_t + T by at most delta = 2 asin(sqrt(m / 2)).  The block axis w_b is
// alpha_t from w_t, and W_b >= W_t + alpha_t for every tile, so theta_b <=
// theta_t + alpha_t and cos(theta_b) >= cos(W_b + T) - m - delta sin(alpha)
// (W_b + T < 150 degrees: cT > 0, W_b < 60).  The block test uses c_b <=
// cos W_b, s_b >= sin W_b and the margin M_b = m + delta sin(alpha_max) plus
// its own rounding.  Edge planes: w_b.n >= w_t.n - |w_b - w_t|, so
// E_b = max_t(chord(alpha_t) + chord_t) + rounding bounds every tile's
// w_t.n + chord_t.  The cluster test with margin M_b + 2e-6 is implied by
// its members' block tests (rt_cluster_prepass, cosW >= 1/2).  A block with
// a degenerate tile cone, W_b >= 60 degrees or more than kCbBlockCap
// survivors runs rt_cb_build's per-tile walk for its tiles instead.
constexpr int kCbBlockCap = 320;  // staged members per block (LDS)

__device__ __forceinline__ double wave_sum_d(double v)
{
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    return v;
}
__device__ __forceinline__ double wave_max_d(double v)
{
    for (int o = 32; o > 0; o >>= 1) v = fmax(v, __shfl_xor(v, o));
    return v;
}

// rt_cb_build's per-tile walk over every cluster (global records).
template <bool FILL>
__device__ __forceinline__ unsigned cb_tile_walk(const SceneDev& S, const WaveCone& wc, unsigned base,
                                                 int2* __restrict__ ent)
{
    const int lane = threadIdx.x & 63;
    unsigned n = 0;
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
    return n;
}

// BLK = tiles per block edge: 8 at 4K and above, 4 below (a tile of a
// 1080p frame spans 4x the angle of one at 7680 wide).
template <bool FILL, int BLK>
__global__ __launch_bounds__(256) void rt_cb_block(const SceneDev S, const FrameDev F, const unsigned* __restrict__ off,
                                                   unsigned* __restrict__ cnt, unsigned* __restrict__ flag,
                                                   int2* __restrict__ ent, unsigned* __restrict__ bstat)
{
    constexpr int NT = BLK * BLK;
    __shared__ float4 tcone[NT * 2];  // [w, cosW] [sinW, chord, ok, present]
    __shared__ int lid[kCbBlockCap];
    __shared__ float4 lrec[kCbBlockCap * kConeRec];
    __shared__ int bstate[2];         // list length, use the list (0/1)
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int tiles_y = (F.height + 7) / 8;
    const int bx0 = blockIdx.x * BLK, by0 = blockIdx.y * BLK;
    // 1. the 64 tile cones (16 per wave), exactly as rt_cb_build computes them
    for (int j = 0; j < NT / 4; ++j) {
        const int lt = wave * (NT / 4) + j;
        const int tx = bx0 + (lt % BLK), ty = by0 + (lt / BLK);
        const bool inside = tx < S.cb_tiles_x && ty < tiles_y;
        const bool present = inside && cb_tile_row_needed(F, ty);
        if (inside && !present && lane == 0 && !FILL) {  // outside the frame's rows: no list
            flag[ty * S.cb_tiles_x + tx] = 1u;
            cnt[ty * S.cb_tiles_x + tx] = 0u;
        }
        WaveCone wc;
        wc.ok = false;
        if (present) {
            const int px = tx * 8 + (lane & 7), py = ty * 8 + (lane >> 3);
            const Vec3 D = camera_dir(F, px < F.width ? px : F.width - 1, py < F.height ? py : F.height - 1);
            wc = wave_cone(D, true);
        }
        if (lane == 0) {
            tcone[2 * lt] = make_float4(wc.w.x, wc.w.y, wc.w.z, wc.cosW);
            tcone[2 * lt + 1] = make_float4(wc.sinW, wc.chord, wc.ok ? 1.f : 0.f, present ? 1.f : 0.f);
        }
    }
    __syncthreads();
    // 2. the block cone (wave 0, lane t = tile t, in double) and its list
    if (wave == 0) {
        const float4 a = tcone[2 * (lane % NT)], b = tcone[2 * (lane % NT) + 1];
        const bool present = lane < NT && b.w != 0.f, ok = b.z != 0.f;
        bool use = !__any(present & !ok) && __any(present);
        const double wx = present ? (double)a.x : 0.0, wy = present ? (double)a.y : 0.0,
                     wz = present ? (double)a.z : 0.0;
        const double sx = wave_sum_d(wx), sy = wave_sum_d(wy), sz = wave_sum_d(wz);
        const double sn = sqrt(sx * sx + sy * sy + sz * sz);
        use = use && sn > 0.0;
        WaveCone bc;
        bc.ok = false;
        float Mb = 0.f, Eb = 0.f;
        if (use) {
            // the float axis the tests use, and each tile's angle to it
            bc.w = make3((float)(sx / sn), (float)(sy / sn), (float)(sz / sn));
            const double bn = sqrt((double)bc.w.x * bc.w.x + (double)bc.w.y * bc.w.y + (double)bc.w.z * bc.w.z);
            const double ux = bc.w.x / bn, uy = bc.w.y / bn, uz = bc.w.z / bn;
            double al = 0.0, wt = 0.0, ch = 0.0;
            if (present) {
                const double tn = sqrt((double)a.x * a.x + (double)a.y * a.y + (double)a.z * a.z);
                const double vx = a.x / tn, vy = a.y / tn, vz = a.z / tn;
                const double cx = uy * vz - uz * vy, cy = uz * vx - ux * vz, cz = ux * vy - uy * vx;
                // angle between the unit axes, plus the float axes' length slack
                al = atan2(sqrt(cx * cx + cy * cy + cz * cz), ux * vx + uy * vy + uz * vz) + 1e-6 +
                     fabs(tn - 1.0) + fabs(bn - 1.0);
                wt = acos(fmin(1.0, (double)a.w)) + al;
                ch = 2.0 * sin(0.5 * al) + fabs(tn - 1.0) + fabs(bn - 1.0) + (double)b.y;
            }
            const double Wb = wave_max_d(wt) * (1.0 + 1e-12) + 1e-9, amax = wave_max_d(al), Emax = wave_max_d(ch);
            const double m = 5e-6, delta = 2.0 * asin(sqrt(0.5 * m));
            double cb = cos(Wb), sb = sin(Wb);
            float cf = (float)cb;
            if ((double)cf > cb) cf = nextafterf(cf, -INFINITY);
            float sf = (float)sb;
            if ((double)sf < sb) sf = nextafterf(sf, INFINITY);
            bc.cosW = cf;
            bc.sinW = sf;
            bc.chord = 0.f;
            bc.ok = Wb < 1.0 && cf >= 0.5f;
            Mb = (float)((m + delta * sin(fmin(amax, 1.5)) + 1e-6) * (1.0 + 1e-6));
            Eb = (float)((Emax + 2e-6 + 1e-6) * (1.0 + 1e-6));
            use = bc.ok;
        }
        unsigned n = 0;
        if (use) {
            const unsigned long long below = (1ull << lane) - 1ull;
            const float Mc = Mb + 2e-6f;
            for (int c0i = 0; c0i < S.n_clu; c0i += 64) {
                const int cl = c0i + lane;
                float4 q0 = make_float4(0.f, 0.f, 0.f, 1.f), q1 = make_float4(INFINITY, 0.f, 0.f, 0.f);
                if (cl < S.n_clu) {
                    q0 = S.clu_cam[2 * cl];
                    q1 = S.clu_cam[2 * cl + 1];
                }
                const int id = __float_as_int(q1.y);
                unsigned long long cm = __ballot((cl < S.n_clu) & cone_overlap(bc, q0, q1.w, 0.0f, Mc));
                while (cm) {
                    const int bb = (int)__builtin_ctzll(cm);
                    cm &= cm - 1;
                    const int k = 64 * __builtin_amdgcn_readlane(id, bb) + lane;
                    bool reach = false;
                    float4 c0, c1, e0, e1, e2;
                    if (k < S.n_tri) {
                        c0 = S.cone_cam[2 * k];
                        c1 = S.cone_cam[2 * k + 1];
                        const float4* e = S.cone_cam + 2 * (size_t)S.n_tri + 3 * k;
                        e0 = e[0];
                        e1 = e[1];
                        e2 = e[2];
                        reach = cone_overlap(bc, c0, c1.w, 0.0f, Mb) &&
                                !(dot(bc.w, make3(e0.x, e0.y, e0.z)) + Eb < e0.w) &&
                                !(dot(bc.w, make3(e1.x, e1.y, e1.z)) + Eb < e1.w) &&
                                !(dot(bc.w, make3(e2.x, e2.y, e2.z)) + Eb < e2.w);
                    }
                    const unsigned long long mm = __ballot(reach);
                    const unsigned pos = n + (unsigned)__popcll(mm & below);
                    if (reach && pos < (unsigned)kCbBlockCap) {
                        lid[pos] = k;
                        float4* r = lrec + kConeRec * pos;
                        r[0] = c0;
                        r[1] = c1;
                        r[2] = e0;
                        r[3] = e1;
                        r[4] = e2;
                    }
                    n += (unsigned)__popcll(mm);
                }
            }
            use = n <= (unsigned)kCbBlockCap;
        }
        if (lane == 0) {
            bstate[0] = (int)n;
            bstate[1] = use ? 1 : 0;
            if (!FILL && bstat) {
                atomicAdd(bstat, 1u);
                if (!use) atomicAdd(bstat + 1, 1u);
                atomicAdd(bstat + 2, use ? n : 0u);
            }
        }
    }
    __syncthreads();
    // 3. every tile against the block list (or its own walk)
    const bool use = bstate[1] != 0;
    const unsigned nl = (unsigned)bstate[0];
    const unsigned long long below = (1ull << lane) - 1ull;
    for (int j = 0; j < NT / 4; ++j) {
        const int lt = wave * (NT / 4) + j;
        const float4 a = tcone[2 * lt], b = tcone[2 * lt + 1];
        if (b.w == 0.f) continue;  // outside the frame
        const int tx = bx0 + (lt % BLK), ty = by0 + (lt / BLK);
        const int tile = ty * S.cb_tiles_x + tx;
        WaveCone wc;
        wc.w = make3(a.x, a.y, a.z);
        wc.cosW = a.w;
        wc.sinW = b.x;
        wc.chord = b.y;
        wc.ok = b.z != 0.f;
        if (!wc.ok) {  // no list: the trace kernel's per-wave path
            if (!FILL && lane == 0) {
                flag[tile] = 1u;
                cnt[tile] = 0u;
            }
            continue;
        }
        const unsigned base = FILL ? off[tile] : 0u;
        unsigned n = 0;
        if (use) {
            for (unsigned q0 = 0; q0 < nl; q0 += 64) {
                const unsigned q = q0 + (unsigned)lane;
                bool reach = false;
                float dmin = 0.0f;
                int k = 0;
                if (q < nl) {
                    const float4* r = lrec + kConeRec * q;
                    const float4 c0 = r[0], c1 = r[1];
                    k = lid[q];
                    dmin = c1.x;
                    reach = cone_overlap(wc, c0, c1.w, 0.0f) && edges_open(wc, r + 2, 0.0f);
                }
                const unsigned long long m = __ballot(reach);
                if (FILL && reach) ent[base + n + (unsigned)__popcll(m & below)] = make_int2(k, __float_as_int(dmin));
                n += (unsigned)__popcll(m);
            }
        } else {
            n = cb_tile_walk<FILL>(S, wc, base, ent);
        }
        if (!FILL && lane == 0) {
            cnt[tile] = n;
            flag[tile] = 0u;
        }
    }
}

// Keys: entry e's key = min dmin over entries [e, end) of its tile (one
// thread per tile), so a wave may stop at the first key beyond its hits.
// Lists of up to RT_CB_SORT entries are first sorted nearest-first (the
// closest hit is order-free: lexicographic (t, index)), so the keys rise
// with the walk and the exit comes at the first entry beyond every lane's
// hit; longer lists keep cluster order.
#ifndef RT_CB_SORT
#define RT_CB_SORT 256
#endif
__device__ __forceinline__ float cb_dmin(int2 en)
{
    const float d = __int_as_float(en.y);
    return d == d ? d : -INFINITY;
}
__global__ void rt_cb_keys(const unsigned* __restrict__ off, int ntiles, int2* __restrict__ ent)
{
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= ntiles) return;
    const unsigned b = off[t], n = off[t + 1] - off[t];
    if (n <= RT_CB_SORT) {  // insertion sort by (dmin, triangle)
        for (unsigned i = 1; i < n; ++i) {
            const int2 x = ent[b + i];
            const float dx = cb_dmin(x);
            unsigned j = i;
            while (j > 0) {
                const int2 y = ent[b + j - 1];
                const float dy = cb_dmin(y);
                if (dy < dx || (dy == dx && y.x < x.x)) break;
                ent[b + j] = y;
                --j;
            }
            ent[b + j] = x;
        }
    }
    float m = INFINITY;
    for (unsigned e = off[t + 1]; e > off[t]; --e) {
        const float d = __int_as_float(ent[e - 1].y);
        m = d == d ? fminf(m, d) : -INFINITY;
        ent[e - 1].y = __float_as_int(m);
    }
}

// The same keys, one wave per tile: a list of up to RT_CB_SORT (256)
// entries is held in registers (4 per lane) and every entry's final place is
// its rank under (dmin, triangle) — the order rt_cb_keys' insertion sort
// produces, the pairs being distinct; once sorted, the suffix minimum of
// entry e is its own dmin (NaN dmins sort first as -inf and key -inf).
// Longer lists keep cluster order and get their suffix minima from lane 0.
__global__ __launch_bounds__(256) void rt_cb_keys_wave(const unsigned* __restrict__ off, int ntiles,
                                                       int2* __restrict__ ent)
{
    const int lane = threadIdx.x & 63;
    const int t = blockIdx.x * 4 + (int)(threadIdx.x >> 6);
    if (t >= ntiles) return;
    const unsigned b = off[t], n = off[t + 1] - off[t];
    if (n <= 1) {
        if (n == 1 && lane == 0) ent[b].y = __float_as_int(cb_dmin(ent[b]));
        return;
    }
    if (n > RT_CB_SORT) {
        if (lane == 0) {
            float m = INFINITY;
            for (unsigned e = off[t + 1]; e > off[t]; --e) {
                const float d = __int_as_float(ent[e - 1].y);
                m = d == d ? fminf(m, d) : -INFINITY;
                ent[e - 1].y = __float_as_int(m);
            }
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

// The walk's records: entry e = the tricam record of its triangle, key in
// [3].z (tricam's [3] = [e2 . Q, file index, 0, 0]).  One thread per entry.
__global__ void rt_cb_expand(const int2* __restrict__ ent, unsigned n, const float4* __restrict__ tricam,
                             float4* __restrict__ rec)
{
    const unsigned e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= n) return;
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

}  // namespace rt
#endif  // RT_AMD_RT_CAMBUF_H
