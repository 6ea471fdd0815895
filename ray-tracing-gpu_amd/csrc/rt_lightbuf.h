// rt_lightbuf.h — the exact light buffer: cube-map cells per light and their build
// kernels.
// Part of the device code of rt_kernels.hip (one translation unit: the
// kernels are templates instantiated by its host half); built with the
// same exactness flags (no FMA contraction, IEEE div/sqrt).
#ifndef RT_AMD_RT_LIGHTBUF_H
#define RT_AMD_RT_LIGHTBUF_H

#include "rt_cull.h"

#pragma clang fp contract(off)

namespace rt {

// ------------------------------------------------------------ light buffer
// Haines & Greenberg's light buffer, made exact: a cube map around each
// light.  The direction d from the light to a shading point (d = -L) picks
// the face of its largest |component| and the cell (i, j) of u = a/|m|,
// v = b/|m| on that face (lb_cell).  Every cell has a cone [w, W] (lb_cone,
// in double) containing every float direction the lookup can map to it,
// with the invariants of a wave cone (exact w . d >= cosW + 2e-6 for every
// such d; sinW, chord raised).  So the wave-level predicates cone_overlap and
// edges_open applied to a CELL are the proven wave-level culling with the
// wave's rays replaced by the cell's: a triangle they reject cannot be
// reported by the reference for any ray of the cell whose length is at most
// the distance dcov the angular slack was sized for (lanes beyond it, or
// with a degenerate direction, take the per-lane path).  Cell lists hold the
// kept triangles nearest-first (the per-lane dmin exit); pairs whose cull
// is not valid up to dcov (dcap < dcov, or never culled) are in a separate
// per-light list sorted by dcap, tested by the lanes with dist > dcap — the
// per-lane predicate light_reach, split in two.
constexpr int kLbGroup = 16;  // cells per supercell edge (two-level build)
// Light-buffer entry: 10 floats (40 B, 8-byte aligned) — [p0, key] [e1,
// e2.x] [e2.y, e2.z] (48 B in round 2: C3 313 -> 269 MB per frame).
constexpr int kLbEntF = 10;  // floats per light-buffer entry

__device__ __forceinline__ int lb_cell(const Vec3 d, int R)
{
    const float ax = fabsf(d.x), ay = fabsf(d.y), az = fabsf(d.z);
    int face;
    float m, a, b;
    if ((ax >= ay) & (ax >= az)) {
        face = d.x >= 0.0f ? 0 : 1;
        m = ax; a = d.y; b = d.z;
    } else if (ay >= az) {
        face = d.y >= 0.0f ? 2 : 3;
        m = ay; a = d.z; b = d.x;
    } else {
        face = d.z >= 0.0f ? 4 : 5;
        m = az; a = d.x; b = d.y;
    }
    const float inv = __builtin_amdgcn_rcpf(m);  // ~1 ulp: the cells' 1e-5 margins cover it
    const float h = 0.5f * (float)R;
    int i = (int)floorf((a * inv + 1.0f) * h);
    int j = (int)floorf((b * inv + 1.0f) * h);
    i = min(max(i, 0), R - 1);
    j = min(max(j, 0), R - 1);
    return (face * R + j) * R + i;
}

__device__ __forceinline__ void lb_face_dir(int face, double u, double v, double* o)
{
    switch (face) {
    case 0: o[0] = 1.0; o[1] = u; o[2] = v; break;
    case 1: o[0] = -1.0; o[1] = u; o[2] = v; break;
    case 2: o[0] = v; o[1] = 1.0; o[2] = u; break;
    case 3: o[0] = v; o[1] = -1.0; o[2] = u; break;
    case 4: o[0] = u; o[1] = v; o[2] = 1.0; break;
    default: o[0] = u; o[1] = v; o[2] = -1.0; break;
    }
    const double n = sqrt(o[0] * o[0] + o[1] * o[1] + o[2] * o[2]);
    o[0] /= n; o[1] /= n; o[2] /= n;
}

// Cone of the cells [i0, i1) x [j0, j1) of a face (u range widened by 1e-5
// for the lookup's rounding), its half-angle grown by `widen` (supercells).
// The farthest point of a small geodesically convex cell from its centre
// direction is a corner.  Float |d| = 1 within 1e-6 (sqrt_w/recip_w), float
// w within 1.2e-7 of the unit centre: cosW = cos(W)(1 - 2e-6) - 4e-6 keeps
// exact w.d >= cosW + 2e-6 for every direction of the cells.
__device__ WaveCone lb_cone(int face, int i0, int i1, int j0, int j1, int R, double widen)
{
    const double du = 1e-5;
    const double u0 = 2.0 * i0 / R - 1.0 - du, u1 = 2.0 * i1 / R - 1.0 + du;
    const double v0 = 2.0 * j0 / R - 1.0 - du, v1 = 2.0 * j1 / R - 1.0 + du;
    double w[3];
    lb_face_dir(face, 0.5 * (u0 + u1), 0.5 * (v0 + v1), w);
    double W = 0.0;
    for (int q = 0; q < 4; ++q) {
        double c[3];
        lb_face_dir(face, (q & 1) ? u1 : u0, (q & 2) ? v1 : v0, c);
        const double x = w[1] * c[2] - w[2] * c[1], y = w[2] * c[0] - w[0] * c[2], z = w[0] * c[1] - w[1] * c[0];
        W = fmax(W, atan2(sqrt(x * x + y * y + z * z), w[0] * c[0] + w[1] * c[1] + w[2] * c[2]));
    }
    W = W * (1.0 + 1e-9) + 1e-6 + widen;
    WaveCone k;
    k.w = make3((float)w[0], (float)w[1], (float)w[2]);
    const double cw = cos(W) * (1.0 - 2e-6) - 4e-6;
    float cf = (float)cw;
    if ((double)cf > cw) cf = nextafterf(cf, -INFINITY);
    const double sw = sqrt(fmax(0.0, 1.0 - (double)cf * (double)cf)) + 1e-6;
    float sf = (float)sw;
    if ((double)sf < sw) sf = nextafterf(sf, INFINITY);
    const double ch = sqrt(2.0 * (1.0 - (double)cf)) + 1e-6;
    float chf = (float)ch;
    if ((double)chf < ch) chf = nextafterf(chf, INFINITY);
    k.cosW = cf;
    k.sinW = sf;
    k.chord = chf;
    k.ok = W < 1.0;  // cosW >= 0.54 like every wave cone (>= 0.5)
    return k;
}

// May a ray of cone wc (up to length dcov) need light record k?  The shadow
// wave batch's predicate with dmax = dcov, minus its dcap term (the dcap
// list), with the edge planes always.  Never-culled pairs: the dcap list.
__device__ __forceinline__ bool lb_keep(const WaveCone& wc, const float4 c0, const float4 c1, const float4* e,
                                        float dcov)
{
    if (!(c0.w > 0.0f) || !(c1.x < dcov)) return false;
    if (!wc.ok) return true;
    const float ang = dcov * 1e-6f * c1.y;
    return cone_overlap(wc, c0, c1.w, ang) && edges_open(wc, e, ang);
}

// Build pass 1, per level of blocks of gs x gs cells (Gl blocks per face
// edge; the last row/column clipped to R): the triangles a block keeps, in
// input order (block-ordered compaction).  The block's cone is widened by
// `widen` (1e-3 rad for supercells of 16 x 16 cells) so that rejecting a
// triangle for it implies rejecting it for each cell it covers.  Input: the
// slot's triangles `perm` (nearest-first), or — with a parent level
// (poffs != nullptr; parents of pf x pf blocks, Gp per face edge, cones
// widened more) — the parent block's list, which already lacks what the
// parent's cone rejects (a proof for every direction inside it).  Big
// lists run a level of 4 x 4 supercells first (round 2: the supercell
// passes were O(supercells x triangles), 60 ms of a C3 upload).
// lists == nullptr: counts only.
__global__ __launch_bounds__(256) void rt_lb_super(const float4* __restrict__ cone, int n, const int* __restrict__ perm,
                                                   int np, int R, float dcov, const unsigned* __restrict__ offs,
                                                   unsigned* __restrict__ counts, int* __restrict__ lists, int gs,
                                                   int Gl, double widen, const unsigned* __restrict__ poffs,
                                                   const int* __restrict__ plists, int pf, int Gp)
{
    const int s = blockIdx.x;
    const int face = s / (Gl * Gl), rem = s % (Gl * Gl), sj = rem / Gl, si = rem % Gl;
    const WaveCone wc = lb_cone(face, si * gs, min(R, si * gs + gs), sj * gs, min(R, sj * gs + gs), R, widen);
    const int* in = perm;
    int nin = np;
    if (poffs) {
        const int p = (face * Gp + sj / pf) * Gp + si / pf;
        in = plists + poffs[p];
        nin = (int)(poffs[p + 1] - poffs[p]);
    }
    __shared__ unsigned wtot[4];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    unsigned total = 0;
    const unsigned base = lists ? offs[s] : 0u;
    for (int q0 = 0; q0 < nin; q0 += 256) {
        const int q = q0 + (int)threadIdx.x;
        int k = -1;
        bool keep = false;
        if (q < nin) {
            k = in[q];
            keep = lb_keep(wc, cone[2 * k], cone[2 * k + 1], cone + 2 * (size_t)n + 3 * (size_t)k, dcov);
        }
        const unsigned long long b = __ballot(keep);
        const unsigned pre = (unsigned)__popcll(b & ((1ull << lane) - 1ull));
        if (lane == 0) wtot[wv] = (unsigned)__popcll(b);
        __syncthreads();
        unsigned off = 0;
        for (int w = 0; w < wv; ++w) off += wtot[w];
        const unsigned blk = wtot[0] + wtot[1] + wtot[2] + wtot[3];
        if (lists && keep) lists[base + total + off + pre] = k;
        total += blk;
        __syncthreads();
    }
    if (!lists && threadIdx.x == 0) counts[s] = total;
}

// Light-buffer entry of triangle k (its tri[] record), kLbEntF floats:
//   [p0, key] [e1, e2.x] [e2.y e2.z]
// key = dmin (cell lists) or dcap (dcap list).  (A per-lane cone test in
// front of the exact test was measured to spare no wave any exact test: a
// cell's list is already what its lanes' cones can reach.)  Read as two
// 16-byte and one 8-byte load at 8-byte alignment.
typedef float lb_v4 __attribute__((ext_vector_type(4), aligned(8)));
typedef float lb_v2 __attribute__((ext_vector_type(2), aligned(8)));
__device__ __forceinline__ const float* lb_rec(const float4* base, size_t q)
{
    return reinterpret_cast<const float*>(base) + kLbEntF * q;
}
__device__ __forceinline__ float4 lb_a(const float* r)
{
    const lb_v4 v = *reinterpret_cast<const lb_v4*>(r);
    return make_float4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ float4 lb_b(const float* r)
{
    const lb_v4 v = *reinterpret_cast<const lb_v4*>(r + 4);
    return make_float4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ float2 lb_tail(const float* r)
{
    const lb_v2 v = *reinterpret_cast<const lb_v2*>(r + 8);
    return make_float2(v.x, v.y);
}

// A cell-list entry: p0 and the key; e1 and e2.x; e2.yz.
__device__ __forceinline__ void lb_cell_entry(const float4* __restrict__ ent, size_t q, float4& a, float4& b, float2& c)
{
    const float* r = lb_rec(ent, q);
    a = lb_a(r);
    b = lb_b(r);
    c = lb_tail(r);
}

__device__ __forceinline__ void lb_write(float* o, const float4* __restrict__ tri, int k, float key)
{
    const float4 a = tri[3 * k], b = tri[3 * k + 1], c = tri[3 * k + 2];
    lb_v2* w = reinterpret_cast<lb_v2*>(o);
    w[0] = lb_v2{a.x, a.y};
    w[1] = lb_v2{a.z, key};
    w[2] = lb_v2{a.w, b.x};
    w[3] = lb_v2{b.y, b.z};
    w[4] = lb_v2{b.w, c.x};
}

// Build pass 2: one thread per cell of a supercell, over the supercell's
// list (staged in LDS), in order.  ent == nullptr: counts only.
__global__ __launch_bounds__(256) void rt_lb_cells(const float4* __restrict__ cone, int n, const float4* __restrict__ tri,
                                                   int R, float dcov, const unsigned* __restrict__ soffs,
                                                   const int* __restrict__ slists, const unsigned* __restrict__ coffs,
                                                   unsigned* __restrict__ ccounts, float* __restrict__ ent)
{
    const int G = R / kLbGroup;
    const int s = blockIdx.x;
    const int face = s / (G * G), rem = s % (G * G), sj = rem / G, si = rem % G;
    const int i = si * kLbGroup + (int)(threadIdx.x & 15), j = sj * kLbGroup + (int)(threadIdx.x >> 4);
    const int cell = (face * R + j) * R + i;
    const WaveCone wc = lb_cone(face, i, i + 1, j, j + 1, R, 0.0);
    __shared__ float4 rec[256 * kConeRec];
    __shared__ int kid[256];
    const unsigned b0 = soffs[s], b1 = soffs[s + 1];
    unsigned cnt = 0, out = ent ? coffs[cell] : 0u;
    for (unsigned q0 = b0; q0 < b1; q0 += 256) {
        __syncthreads();
        const unsigned q = q0 + threadIdx.x;
        if (q < b1) {
            const int k = slists[q];
            kid[threadIdx.x] = k;
            rec[kConeRec * threadIdx.x] = cone[2 * k];
            rec[kConeRec * threadIdx.x + 1] = cone[2 * k + 1];
            for (int e = 0; e < 3; ++e) rec[kConeRec * threadIdx.x + 2 + e] = cone[2 * (size_t)n + 3 * (size_t)k + e];
        }
        __syncthreads();
        const int m = (int)min(256u, b1 - q0);
        for (int x = 0; x < m; ++x) {
            const float4 c0 = rec[kConeRec * x], c1 = rec[kConeRec * x + 1];
            if (!lb_keep(wc, c0, c1, rec + kConeRec * x + 2, dcov)) continue;
            if (ent) lb_write(ent + kLbEntF * (size_t)out++, tri, kid[x], c1.x);
            else ++cnt;
        }
    }
    if (!ent) ccounts[cell] = cnt;
}

// The dcap list of one light: entries of perm (sorted by dcap), key = dcap.
__global__ void rt_lb_dcap(const float4* __restrict__ cone, const float4* __restrict__ tri, const int* __restrict__ perm,
                           int m, float* __restrict__ out)
{
    const int q = blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= m) return;
    const int k = perm[q];
    const float4 c1 = cone[2 * k + 1];
    lb_write(out + kLbEntF * (size_t)q, tri, k, c1.z == c1.z ? c1.z : -INFINITY);
}

}  // namespace rt
#endif  // RT_AMD_RT_LIGHTBUF_H
