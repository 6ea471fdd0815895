// rt_fastmath.h — short instruction sequences on gfx950 that return EXACTLY
// the IEEE-754 results hipcc's default (correctly rounded) f32 division,
// reciprocal and square root return, on a bounded operand domain.  Outside the
// domain (and for 0/Inf/NaN) the caller's wave takes the IEEE path.
//
// Verified on MI355X by tools/fastmath_check.hip, which includes THIS header:
//   rcp_nr    — every float with |x| in [2^-125, 2^125] (exhaustive);
//   sqrt_cr   — every float in [2^-100, 2^100] (exhaustive);
//   div_nr    — Markstein's theorem (y = RN(1/b) exactly, q within 1 ulp,
//               r = a - b*q exact by FMA => RN(q + r*y) = RN(a/b) absent
//               under/overflow) plus randomised and structured operand sweeps.
#pragma once

#include <hip/hip_runtime.h>

namespace rt {

// RN(1/x): v_rcp_f32 then one FMA Newton step.
__device__ __forceinline__ float rcp_nr(float x)
{
    const float r = __builtin_amdgcn_rcpf(x);
    const float e = __builtin_fmaf(-x, r, 1.0f);
    return __builtin_fmaf(e, r, r);
}

// RN(a/b) from y = RN(1/b): q0 = RN(a*y), remainder by FMA, one correction.
// A zero numerator returns q0 = a*y directly: it carries the IEEE sign of
// a/b, which the correction step (+0 + -0 = +0) would lose.
__device__ __forceinline__ float div_nr(float a, float b, float y)
{
    const float q = a * y;
    const float r = __builtin_fmaf(-b, q, a);
    const float q1 = __builtin_fmaf(r, y, q);
    return a == 0.0f ? q : q1;
}

// RN(sqrt(x)) for normal x: v_sqrt_f32 (within 1 ulp) and the same
// neighbour fix-up LLVM emits for its IEEE expansion, minus the denormal
// scaling and the 0/Inf/NaN class handling the domain excludes.
__device__ __forceinline__ float sqrt_cr(float x)
{
    const float s = __builtin_amdgcn_sqrtf(x);
    const float sm = __uint_as_float(__float_as_uint(s) - 1u);
    const float sp = __uint_as_float(__float_as_uint(s) + 1u);
    const float rm = __builtin_fmaf(-sm, s, x);
    const float rp = __builtin_fmaf(-sp, s, x);
    float r = (rm <= 0.0f) ? sm : s;
    r = (rp > 0.0f) ? sp : r;
    return r;
}

// Domain predicates.
__device__ __forceinline__ bool in_rcp_domain(float x)
{
    const float a = fabsf(x);
    return a >= 0x1p-125f && a <= 0x1p125f;
}
__device__ __forceinline__ bool in_div_domain(float a, float b)
{
    const float aa = fabsf(a), ab = fabsf(b);
    return ab >= 0x1p-60f && ab <= 0x1p60f && (aa == 0.0f || (aa >= 0x1p-60f && aa <= 0x1p60f));
}
__device__ __forceinline__ bool in_sqrt_domain(float x) { return x >= 0x1p-100f && x <= 0x1p100f; }

// Wave-uniform dispatch: the fast sequence when every active lane is in its
// domain, otherwise the compiler's IEEE expansion for the whole wave.
__device__ __forceinline__ float recip_w(float x)
{
    if (__builtin_expect(__any(!in_rcp_domain(x)), 0)) return 1.0f / x;
    return rcp_nr(x);
}
__device__ __forceinline__ float div_w(float a, float b)
{
    if (__builtin_expect(__any(!in_div_domain(a, b)), 0)) return a / b;
    return div_nr(a, b, rcp_nr(b));
}
__device__ __forceinline__ float sqrt_w(float x)
{
    if (__builtin_expect(__any(!in_sqrt_domain(x)), 0)) return sqrtf(x);
    return sqrt_cr(x);
}

}  // namespace rt
