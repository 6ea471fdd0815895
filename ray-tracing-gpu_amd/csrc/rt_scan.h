// rt_scan.h — exclusive prefix sums of u32 counts on the device: the offsets
// of the camera-buffer and light-buffer builds, computed where the counts
// are instead of round-tripping them through the host.
// Part of the device code of rt_kernels.hip (one translation unit).
#ifndef RT_AMD_RT_SCAN_H
#define RT_AMD_RT_SCAN_H

#include <hip/hip_runtime.h>

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
__global__ __launch_bounds__(kScanThreads) void rt_scan_apply(const unsigned* in, unsigned n,
                                                              const unsigned long long* __restrict__ bsum,
                                                              unsigned nb, unsigned* out)
{
    __shared__ unsigned long long sh[kScanThreads];
    const size_t base = (size_t)blockIdx.x * kScanTile + (size_t)threadIdx.x * kScanItems;
    unsigned v[kScanItems];
    unsigned long long s = 0;
    for (int q = 0; q < kScanItems; ++q) {
        v[q] = base + q < n ? in[base + q] : 0u;
        s += v[q];
    }
    unsigned long long tot;
    unsigned long long run = bsum[blockIdx.x] + block_exscan(s, sh, &tot);
    for (int q = 0; q < kScanItems; ++q) {
        if (base + q < n) out[base + q] = (unsigned)run;
        run += v[q];
    }
    if (blockIdx.x == nb - 1 && threadIdx.x == 0) out[n] = (unsigned)bsum[nb];
}

// Small scans (n <= kScanSmallMax): one 1024-thread block, 64 consecutive
// counts per thread — one launch instead of three (the per-camera builds
// scan a count per 8x8 tile: 32,400 at 1080p).  bsum[0] = the 64-bit total.
constexpr int kScanSmallThreads = 1024, kScanSmallItems = 64;
constexpr unsigned kScanSmallMax = kScanSmallThreads * kScanSmallItems;
__global__ __launch_bounds__(kScanSmallThreads) void rt_scan_small(const unsigned* in, unsigned n,
                                                                   unsigned long long* __restrict__ bsum,
                                                                   unsigned* out)
{
    __shared__ unsigned long long sh[kScanSmallThreads];
    const int t = threadIdx.x;
    const unsigned base = (unsigned)t * kScanSmallItems;
    unsigned long long s = 0;
    // all 64 loads issued before the sum (a dependent loop waited on each)
    unsigned v[kScanSmallItems];
#pragma unroll
    for (int q = 0; q < kScanSmallItems; ++q) v[q] = base + q < n ? in[base + q] : 0u;
#pragma unroll
    for (int q = 0; q < kScanSmallItems; ++q) s += v[q];
    sh[t] = s;
    __syncthreads();
    for (int o = 1; o < kScanSmallThreads; o <<= 1) {
        const unsigned long long x = t >= o ? sh[t - o] : 0ull;
        __syncthreads();
        sh[t] += x;
        __syncthreads();
    }
    unsigned long long run = sh[t] - s;
#pragma unroll
    for (int q = 0; q < kScanSmallItems; ++q) {
        if (base + q < n) out[base + q] = (unsigned)run;
        run += v[q];
    }
    if (t == kScanSmallThreads - 1) {
        out[n] = (unsigned)sh[t];
        bsum[0] = sh[t];
    }
}

// Scratch words (u64) rt_scan needs for n counts.
inline size_t scan_scratch(size_t n) { return (n + kScanTile - 1) / kScanTile + 1; }

// Exclusive scan of in[0..n) into out[0..n], out[n] = total, on stream st;
// bsum (scan_scratch(n) u64) receives the 64-bit total at bsum[nb].  n >= 1.
inline hipError_t scan_u32(const unsigned* in, unsigned n, unsigned* out, unsigned long long* bsum, hipStream_t st,
                           unsigned long long** total_dev)
{
    if (n <= kScanSmallMax) {
        hipLaunchKernelGGL(rt_scan_small, dim3(1), dim3(kScanSmallThreads), 0, st, in, n, bsum, out);
        if (total_dev) *total_dev = bsum;
        return hipGetLastError();
    }
    const unsigned nb = (unsigned)((n + kScanTile - 1) / kScanTile);
    hipLaunchKernelGGL(rt_scan_reduce, dim3(nb), dim3(kScanThreads), 0, st, in, n, bsum);
    hipLaunchKernelGGL(rt_scan_blocks, dim3(1), dim3(kScanThreads), 0, st, bsum, nb);
    hipLaunchKernelGGL(rt_scan_apply, dim3(nb), dim3(kScanThreads), 0, st, in, n, (const unsigned long long*)bsum, nb,
                       out);
    if (total_dev) *total_dev = bsum + nb;
    return hipGetLastError();
}

}  // namespace rt
#endif  // RT_AMD_RT_SCAN_H
