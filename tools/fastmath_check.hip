// Verifies ray-tracing-gpu_amd/csrc/rt_fastmath.h against the compiler's IEEE
// f32 operations on gfx950 (run on an MI355X):
//   rcp_nr  vs 1.0f/x   — exhaustive over every float with |x| in [2^-125, 2^125]
//   sqrt_cr vs sqrtf(x) — exhaustive over every float in [2^-100, 2^100]
//   div_nr  vs a/b      — (i) every numerator mantissa x 4096 divisors (random +
//                         structured: all-ones / all-zeros / single-bit
//                         mantissas), (ii) 2^36 random pairs over the domain
//                         exponents [-60, 60] with random signs, plus a = +-0.
//
//   hipcc -O3 --offload-arch=gfx950 -ffp-contract=off tools/fastmath_check.hip -o tools/fastmath_check
#include <hip/hip_runtime.h>

#include <cstdio>

#include "../ray-tracing-gpu_amd/csrc/rt_fastmath.h"

#pragma clang fp contract(off)

using namespace rt;

struct Counts {
    unsigned long long rcp_tested, rcp_bad, sqrt_tested, sqrt_bad, div1_tested, div1_bad, div2_tested, div2_bad;
    unsigned bad_examples[8][2];
    unsigned n_examples;
};

__device__ void note_bad(Counts* c, unsigned a, unsigned b)
{
    unsigned k = atomicAdd(&c->n_examples, 1u);
    if (k < 8) {
        c->bad_examples[k][0] = a;
        c->bad_examples[k][1] = b;
    }
}

__device__ void wave_count(unsigned long long* tested, unsigned long long* bad, bool t, bool b)
{
    const unsigned long long mt = __ballot(t), mb = __ballot(b);
    if ((threadIdx.x & 63) == 0) {
        atomicAdd(tested, (unsigned long long)__popcll(mt));
        if (mb) atomicAdd(bad, (unsigned long long)__popcll(mb));
    }
}

__global__ void unary(unsigned long long base, Counts* c)
{
    const unsigned bits = (unsigned)(base + (unsigned long long)blockIdx.x * blockDim.x + threadIdx.x);
    const float x = __uint_as_float(bits);
    const bool in_r = in_rcp_domain(x);
    const bool bad_r = in_r && __float_as_uint(rcp_nr(x)) != __float_as_uint(1.0f / x);
    wave_count(&c->rcp_tested, &c->rcp_bad, in_r, bad_r);
    const bool in_s = in_sqrt_domain(x);
    const bool bad_s = in_s && __float_as_uint(sqrt_cr(x)) != __float_as_uint(sqrtf(x));
    wave_count(&c->sqrt_tested, &c->sqrt_bad, in_s, bad_s);
    if (bad_r || bad_s) note_bad(c, bits, bad_r ? 1u : 2u);
}

__device__ __forceinline__ unsigned hash32(unsigned long long x)
{
    x ^= x >> 33;
    x *= 0xff51afd7ed558ccdull;
    x ^= x >> 33;
    x *= 0xc4ceb9fe1a85ec53ull;
    x ^= x >> 33;
    return (unsigned)x;
}

__device__ unsigned divisor_bits(unsigned j)
{
    // 4096 divisors: mantissa patterns x exponents
    const unsigned e = 127 - 40 + (j % 81);  // exponents 2^-40 .. 2^40
    unsigned m;
    switch ((j / 81) % 8) {
    case 0: m = 0x7FFFFFu; break;                       // all ones
    case 1: m = 0u; break;                              // power of two
    case 2: m = 1u << (hash32(j) % 23); break;          // one bit
    case 3: m = 0x7FFFFFu ^ (1u << (hash32(j) % 23)); break;
    default: m = hash32(j * 7919ull + 17) & 0x7FFFFFu; break;
    }
    return ((hash32(j + 99) & 1u) << 31) | (e << 23) | m;
}

// (i) numerator mantissas x divisors; numerator exponent varies with j.
__global__ void div_grid(unsigned j0, Counts* c)
{
    const unsigned m = blockIdx.x * blockDim.x + threadIdx.x;  // 2^23 mantissas
    const unsigned j = j0 + blockIdx.y;
    const unsigned ea = 127 - 50 + (hash32(j * 31ull + m / 4096) % 101);
    const unsigned abits = ((m & 1u) << 31) | (ea << 23) | (m & 0x7FFFFFu);
    const float a = __uint_as_float(abits), b = __uint_as_float(divisor_bits(j));
    const bool in = in_div_domain(a, b);
    const bool bad = in && __float_as_uint(div_nr(a, b, rcp_nr(b))) != __float_as_uint(a / b);
    wave_count(&c->div1_tested, &c->div1_bad, in, bad);
    if (bad) note_bad(c, abits, __float_as_uint(b));
}

// (ii) random pairs, exponents uniform over the domain, zero numerators.
__global__ void div_random(unsigned long long base, Counts* c)
{
    const unsigned long long i = base + (unsigned long long)blockIdx.x * blockDim.x + threadIdx.x;
    const unsigned h1 = hash32(2 * i + 1), h2 = hash32(2 * i + 2), h3 = hash32(i * 0x9E3779B97F4A7C15ull);
    const unsigned ea = 127 - 60 + (h3 % 121), eb = 127 - 60 + ((h3 >> 8) % 121);
    unsigned abits = (h1 & 0x807FFFFFu) | (ea << 23);
    if ((h3 >> 24) == 0) abits &= 0x80000000u;  // +-0 numerators
    const unsigned bbits = (h2 & 0x807FFFFFu) | (eb << 23);
    const float a = __uint_as_float(abits), b = __uint_as_float(bbits);
    const bool in = in_div_domain(a, b);
    const bool bad = in && __float_as_uint(div_nr(a, b, rcp_nr(b))) != __float_as_uint(a / b);
    wave_count(&c->div2_tested, &c->div2_bad, in, bad);
    if (bad) note_bad(c, abits, bbits);
}

int main()
{
    Counts* d;
    (void)hipMalloc(&d, sizeof(Counts));
    (void)hipMemset(d, 0, sizeof(Counts));
    const unsigned long long chunk = 1ull << 28;
    for (unsigned long long b = 0; b < (1ull << 32); b += chunk) unary<<<(unsigned)(chunk / 256), 256>>>(b, d);
    for (unsigned j0 = 0; j0 < 4096; j0 += 256) div_grid<<<dim3((1u << 23) / 256, 256), 256>>>(j0, d);
    for (unsigned long long b = 0; b < (1ull << 36); b += chunk) div_random<<<(unsigned)(chunk / 256), 256>>>(b, d);
    Counts h;
    (void)hipMemcpy(&h, d, sizeof h, hipMemcpyDeviceToHost);
    std::printf("{\"rcp_nr\": {\"tested\": %llu, \"mismatch\": %llu}, \"sqrt_cr\": {\"tested\": %llu, \"mismatch\": %llu}, "
                "\"div_nr_grid\": {\"tested\": %llu, \"mismatch\": %llu}, \"div_nr_random\": {\"tested\": %llu, \"mismatch\": %llu}, "
                "\"examples\": [",
                h.rcp_tested, h.rcp_bad, h.sqrt_tested, h.sqrt_bad, h.div1_tested, h.div1_bad, h.div2_tested, h.div2_bad);
    for (unsigned k = 0; k < h.n_examples && k < 8; ++k)
        std::printf("%s[\"0x%08x\", \"0x%08x\"]", k ? ", " : "", h.bad_examples[k][0], h.bad_examples[k][1]);
    std::printf("]}\n");
    return (h.rcp_bad || h.sqrt_bad || h.div1_bad || h.div2_bad) ? 1 : 0;
}
