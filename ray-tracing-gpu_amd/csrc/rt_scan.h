// rt_scan.h — exclusive prefix sums of u32 counts on the device: the offsets
// of the camera-buffer and light-buffer builds, computed where the counts
// are instead of round-tripping them through the host.
// Part of the device code of rt_kernels.hip (one translation unit).
#ifndef RT_AMD_RT_SCAN_H
#define RT_AMD_RT_SCAN_H

#include <hip/hip_runtime.h>

#include <algorithm>

namespace rt {

constexpr int kScanThreads = 256, kScanItems = 16;
constexpr int kScanTile = kScanThreads * kScanItems;  // counts per block

// Exclusive scan of one value per thread of a 256-thread block (LDS,
// Hillis-Steele); *total = the block's sum.
__device__ __forceinline__ unsigned long long block_exscan(unsigned long long v, unsigned long long* sh,
                                                           unsigned long long* total)
{
    const int t = threadIdx.x;
    sh[t] = v;
    __syncthreads();
    for (int o = 1; o < kScanThreads; o <<= 1) {
        const unsigned long long x = t >= o ? sh[t - o] : 0ull;
        __syncthreads();
        sh[t] += x;
        __syncthreads();
    }
    const unsigned long long incl = sh[t];
    *total = sh[kScanThreads - 1];
    __syncthreads();
    return incl - v;
}

// Pass 1: bsum[b] = sum of block b's tile of counts.
__global__ __launch_bounds__(kScanThreads) void rt_scan_reduce(const unsigned* __restrict__ in, unsigned n,
                                                               unsigned long long* __restrict__ bsum)
{
    __shared__ unsigned long long sh[kScanThreads];
    const size_t base = (size_t)blockIdx.x * kScanTile;
    unsigned long long v = 0;
    for (int q = 0; q < kScanItems; ++q) {
        const size_t i = base + (size_t)q * kScanThreads + threadIdx.x;  // coalesced
        if (i < n) v += in[i];
    }
    unsigned long long tot;
    block_exscan(v, sh, &tot);
    if (threadIdx.x == 0) bsum[blockIdx.x] = tot;
}

// Pass 2 (one block): bsum[0..nb) -> exclusive prefixes, bsum[nb] = total.
__global__ __launch_bounds__(kScanThreads) void rt_scan_blocks(unsigned long long* __restrict__ bsum, unsigned nb)
{
    __shared__ unsigned long long sh[kScanThreads];
    unsigned long long carry = 0;
    for (unsigned b0 = 0; b0 < nb; b0 += kScanThreads) {
        const unsigned b = b0 + threadIdx.x;
        const unsigned long long v = b < nb ? bsum[b] : 0ull;
        unsigned long long tot;
        const unsigned long long ex = block_exscan(v, sh, &tot);
        if (b < nb) bsum[b] = carry + ex;
        carry += tot;
    }
    if (threadIdx.x == 0) bsum[nb] = carry;
}

// Pass 3: out[i] = exclusive prefix of in[i] (out may alias in), out[n] =
// total; both truncated to 32 bits — the caller checks bsum[nb] (64-bit).
// Thread t owns the 16 consecutive counts [16t, 16t + 16) of its block's tile.
// zero_in: in (distinct from out) is left all zeros (a counter array that
// is scanned and then counts again: the wavefront's sort bins).
__global__ __launch_bounds__(kScanThreads) void rt_scan_apply(const unsigned* in, unsigned n,
                                                              const unsigned long long* __restrict__ bsum,
                                                              unsigned nb, unsigned* out, bool zero_in = false)
{
    __shared__ unsigned long long sh[kScanThreads];
    const size_t base = (size_t)blockIdx.x * kScanTile + (size_t)threadIdx.x * kScanItems;
    unsigned v[kScanItems];
    unsigned long long s = 0;
    for (int q = 0; q < kScanItems; ++q) {
        v[q] = base + q < n ? in[base + q] : 0u;
        s += v[q];
        if (zero_in && base + q < n) const_cast<unsigned*>(in)[base + q] = 0u;
    }
    unsigned long long tot;
    unsigned long long run = bsum[blockIdx.x] + block_exscan(s, sh, &tot);
    for (int q = 0; q < kScanItems; ++q) {
        if (base + q < n) out[base + q] = (unsigned)run;
        run += v[q];
    }
    if (blockIdx.x == nb - 1 && threadIdx.x == 0) out[n] = (unsigned)bsum[nb];
}

// Small scans (n <= kScanSmallMax: the per-camera builds scan a count per
// triangle, 50,176 for the C3 mesh, and per 8x8 tile, 32,400 at 1080p): two
// launches over blocks of kScanSmallTile counts.  A block's four waves own
// 256 consecutive counts each, as four chunks of 64 (lane l: count c * 64 +
// l of chunk c), so every load and store is one coalesced wave access and
// the four chunk scans are independent.  Pass 1 sums each block (bsum[b],
// exact); pass 2 takes its block's prefix from the <= 64 sums before it (one
// wave), scans its chunks, and block 0 writes the total.  Round 3: one
// 1024-thread block with thread-owned runs of 64 consecutive counts made
// each access 64 cache lines in one CU (57 us for the mesh's counts); a
// wave walk of its chunks in series waited one load latency per chunk
// (36 us); all chunks in registers spilled (77 us).  The prefixes are mod
// 2^32 (the outputs are 32-bit); the total is 64-bit: bsum[nb].  out may
// alias in (pass 2 reads each count before writing it, in the same block).
constexpr int kScanSmallThreads = 256, kScanSmallTile = 1024;
constexpr unsigned kScanSmallMax = 64u * kScanSmallTile;  // pass 2 sums <= 64 block totals in one wave
__global__ __launch_bounds__(kScanSmallThreads) void rt_scan_small_reduce(const unsigned* __restrict__ in, unsigned n,
                                                                          unsigned long long* __restrict__ bsum)
{
    __shared__ unsigned long long ws[kScanSmallThreads / 64];
    const unsigned base = blockIdx.x * (unsigned)kScanSmallTile + threadIdx.x;
    unsigned long long s = 0;
#pragma unroll
    for (int q = 0; q < kScanSmallTile / kScanSmallThreads; ++q) {
        const unsigned i = base + (unsigned)q * kScanSmallThreads;
        s += i < n ? in[i] : 0u;
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
    if ((threadIdx.x & 63) == 0) ws[threadIdx.x >> 6] = s;
    __syncthreads();
    if (threadIdx.x == 0) bsum[blockIdx.x] = ws[0] + ws[1] + ws[2] + ws[3];
}
__global__ __launch_bounds__(kScanSmallThreads) void rt_scan_small_apply(const unsigned* in, unsigned n,
                                                                         unsigned long long* __restrict__ bsum,
                                                                         unsigned nb, unsigned* out,
                                                                         bool zero_in = false)
{
    __shared__ unsigned ws[kScanSmallThreads / 64];
    __shared__ unsigned long long pre;
    const int lane = (int)(threadIdx.x & 63), w = (int)(threadIdx.x >> 6);
    const unsigned base = blockIdx.x * (unsigned)kScanSmallTile + (unsigned)w * 256u + (unsigned)lane;
    unsigned v[4], ex[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        const unsigned i = base + (unsigned)c * 64u;
        v[c] = i < n ? in[i] : 0u;
        if (zero_in && i < n) const_cast<unsigned*>(in)[i] = 0u;
    }
    if (w == 0) {  // this block's prefix; block 0: the total
        const unsigned long long x = (unsigned)lane < nb ? bsum[lane] : 0ull;
        unsigned long long p = (unsigned)lane < blockIdx.x ? x : 0ull, t = x;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            p += __shfl_xor(p, o);
            t += __shfl_xor(t, o);
        }
        if (lane == 0) {
            pre = p;
            if (blockIdx.x == 0) {
                out[n] = (unsigned)t;
                bsum[nb] = t;
            }
        }
    }
    unsigned carry = 0;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        unsigned x = v[c];
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const unsigned y = __shfl_up(x, o);
            if (lane >= o) x += y;
        }
        ex[c] = carry + x - v[c];
        carry += __shfl(x, 63);
    }
    if (lane == 0) ws[w] = carry;
    __syncthreads();
    unsigned off = (unsigned)pre;
    for (int k = 0; k < w; ++k) off += ws[k];
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        const unsigned i = base + (unsigned)c * 64u;
        if (i < n) out[i] = off + ex[c];
    }
}

// Scratch words (u64) rt_scan needs for n counts.
inline size_t scan_scratch(size_t n)
{
    return std::max((n + kScanTile - 1) / kScanTile, (n + kScanSmallTile - 1) / kScanSmallTile) + 1;
}

// Exclusive scan of in[0..n) into out[0..n], out[n] = total, on stream st;
// bsum (scan_scratch(n) u64) receives the 64-bit total at bsum[nb].  n >= 1.
// zero_in: in (then distinct from out) is left all zeros.
inline hipError_t scan_u32(const unsigned* in, unsigned n, unsigned* out, unsigned long long* bsum, hipStream_t st,
                           unsigned long long** total_dev, bool zero_in = false)
{
    if (n <= kScanSmallMax) {
        const unsigned nb = (n + kScanSmallTile - 1) / kScanSmallTile;
        hipLaunchKernelGGL(rt_scan_small_reduce, dim3(nb), dim3(kScanSmallThreads), 0, st, in, n, bsum);
        hipLaunchKernelGGL(rt_scan_small_apply, dim3(nb), dim3(kScanSmallThreads), 0, st, in, n, bsum, nb, out,
                           zero_in);
        if (total_dev) *total_dev = bsum + nb;
        return hipGetLastError();
    }
    const unsigned nb = (unsigned)((n + kScanTile - 1) / kScanTile);
    hipLaunchKernelGGL(rt_scan_reduce, dim3(nb), dim3(kScanThreads), 0, st, in, n, bsum);
    hipLaunchKernelGGL(rt_scan_blocks, dim3(1), dim3(kScanThreads), 0, st, bsum, nb);
    hipLaunchKernelGGL(rt_scan_apply, dim3(nb), dim3(kScanThreads), 0, st, in, n, (const unsigned long long*)bsum, nb,
                       out, zero_in);
    if (total_dev) *total_dev = bsum + nb;
    return hipGetLastError();
}

}  // namespace rt
#endif  // RT_AMD_RT_SCAN_H
