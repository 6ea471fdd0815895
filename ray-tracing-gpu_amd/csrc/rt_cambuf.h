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
