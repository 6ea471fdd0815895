// Exhaustive check of a short reciprocal sequence against IEEE 1.0f/x on
// gfx950, over every float32 bit pattern (2^32).  Used to decide whether the
// triangle test may replace the compiler's full division expansion for
// InvDet = 1/Det (Triangle.cpp:147) without changing a single bit.
//
//   hipcc -O3 --offload-arch=gfx950 -ffp-contract=off tools/rcp_exhaustive.hip -o /tmp/rcpx && /tmp/rcpx
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstring>

#pragma clang fp contract(off)

__device__ __forceinline__ float rcp_nr1(float x)
{
    const float r = __builtin_amdgcn_rcpf(x);
    const float e = __builtin_fmaf(-x, r, 1.0f);
    return __builtin_fmaf(e, r, r);
}
__device__ __forceinline__ float rcp_nr2(float x)
{
    float r = rcp_nr1(x);
    const float e = __builtin_fmaf(-x, r, 1.0f);
    return __builtin_fmaf(e, r, r);
}

struct Counts {
    unsigned long long tested, bad1, bad2, bad0;
    unsigned first_bad1[8];
};

__global__ void check(unsigned long long base, Counts* c)
{
    const unsigned long long i = base + (unsigned long long)blockIdx.x * blockDim.x + threadIdx.x;
    const unsigned bits = (unsigned)i;
    const float x = __uint_as_float(bits);
    const float ax = fabsf(x);
    // domain used by the kernel: finite, |x| in [2^-125, 2^125] (the caller
    // falls back to the IEEE division outside it)
    const bool in = ax >= 0x1p-125f && ax <= 0x1p125f;
    const float ref = 1.0f / x;
    const float a = rcp_nr1(x), b = rcp_nr2(x), z = __builtin_amdgcn_rcpf(x);
    const bool b1 = in && __float_as_uint(a) != __float_as_uint(ref);
    const unsigned long long mt = __ballot(in), m1 = __ballot(b1),
                             m2 = __ballot(in && __float_as_uint(b) != __float_as_uint(ref)),
                             m0 = __ballot(in && __float_as_uint(z) != __float_as_uint(ref));
    if ((threadIdx.x & 63) == 0) {
        atomicAdd(&c->tested, (unsigned long long)__popcll(mt));
        if (m0) atomicAdd(&c->bad0, (unsigned long long)__popcll(m0));
        if (m2) atomicAdd(&c->bad2, (unsigned long long)__popcll(m2));
    }
    if (b1) {
        unsigned long long k = atomicAdd(&c->bad1, 1ull);
        if (k < 8) c->first_bad1[k] = bits;
    }
}

int main()
{
    Counts* d;
    hipMalloc(&d, sizeof(Counts));
    hipMemset(d, 0, sizeof(Counts));
    const unsigned long long total = 1ull << 32, chunk = 1ull << 28;
    for (unsigned long long b = 0; b < total; b += chunk) check<<<(unsigned)(chunk / 256), 256>>>(b, d);
    Counts h;
    hipMemcpy(&h, d, sizeof h, hipMemcpyDeviceToHost);
    std::printf("{\"tested\": %llu, \"rcp_only_mismatch\": %llu, \"rcp_nr1_mismatch\": %llu, \"rcp_nr2_mismatch\": %llu, \"first_nr1_bad\": [",
                h.tested, h.bad0, h.bad1, h.bad2);
    for (int k = 0; k < 8 && k < (int)h.bad1; ++k) {
        float f;
        std::memcpy(&f, &h.first_bad1[k], 4);
        std::printf("%s\"0x%08x (%a)\"", k ? ", " : "", h.first_bad1[k], f);
    }
    std::printf("]}\n");
    return 0;
}
