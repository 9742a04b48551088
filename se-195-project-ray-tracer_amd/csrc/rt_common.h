// rt_common.h -- shared device helpers for the gfx950 ray-trace kernels.
//
// All kernels are compiled with -ffp-contract=off and IEEE float division /
// sqrt (hipcc's default correctly-rounded f32 div/sqrt): the parity contract
// is bit-exactness with the reference's x86-64 SSE float arithmetic, so every
// float expression below is written in the reference's evaluation order and
// no multiply-add may be fused.
#ifndef RT_COMMON_H
#define RT_COMMON_H

#include <hip/hip_runtime.h>
#include <stdint.h>
#include "../../include/rt_hip.h"

namespace rt {

struct v3 { float x, y, z; };
struct ray3 { v3 o, d; };

__device__ __forceinline__ v3 mk(float x, float y, float z) { v3 r; r.x = x; r.y = y; r.z = z; return r; }

// Correctly rounded sqrtf in 14 VALU ops.  hipcc's sqrtf (gfx950) is: 2^32
// pre-scale of x < 2^-96, v_sqrt_f32 (<= 1 ulp), the two-residual fixup
// (s -/+ 1 ulp tested with fma(-s', s, x)), 2^-16 post-scale, and a final
// class select returning x itself for +-0 / +inf.  That last select is
// redundant after the fixup (v_sqrt gives +-0 / +inf exactly and both residual
// tests then leave it), so it is dropped; everything else is kept.  Checked
// against sqrtf for all 2^32 inputs on the device (tests/test_gpu_math.py).
__device__ __forceinline__ float sqrt_rn(float x)
{
    const bool tiny = x < 0x1p-96f;
    const float xs = tiny ? x * 0x1p32f : x;
    float s = __builtin_amdgcn_sqrtf(xs);
    const float s_dn = __uint_as_float(__float_as_uint(s) - 1u);
    const float s_up = __uint_as_float(__float_as_uint(s) + 1u);
    const float r_dn = __builtin_fmaf(-s_dn, s, xs);
    const float r_up = __builtin_fmaf(-s_up, s, xs);
    s = (r_dn <= 0.f) ? s_dn : s;
    s = (r_up > 0.f) ? s_up : s;
    return tiny ? s * 0x1p-16f : s;
}

// Short correctly rounded forms on the normal range, each checked against the
// IEEE result for all 2^32 inputs on the device (tests/test_gpu_math.py):
//  * sqrt_nr: s = x * v_rsq_f32(x), then one residual correction
//    s + (x - s*s) * rsq(x) / 2 -- equal to sqrtf(x) for x in [2^-96, inf)
//    (differences start below 2^-102).  One transcendental: a form with both
//    v_sqrt_f32 and v_rsq_f32 was measured 7 % slower on the smallpt kernel;
//  * rcp_nr: v_rcp_f32 and one Newton step -- equal to 1.f / x for
//    2^-126 <= |x| < 2^126 (outside it the result or input is denormal).
// Callers guard the domain with a wave-uniform branch to the general
// sequences (sqrt_rn, '/'), so a wave only pays for those when one of its
// lanes is outside the range.
__device__ __forceinline__ bool sqrt_nr_ok(float x)     // 2^-96 <= x < +inf (not NaN)
{
    return (__float_as_uint(x) - 0x0f800000u) < 0x70000000u;
}

__device__ __forceinline__ float sqrt_nr(float x)
{
    const float y = __builtin_amdgcn_rsqf(x);
    const float s = x * y;
    const float r = __builtin_fmaf(-s, s, x);
    return __builtin_fmaf(r, 0.5f * y, s);
}

__device__ __forceinline__ float rcp_nr(float x)
{
    const float y = __builtin_amdgcn_rcpf(x);
    const float e = __builtin_fmaf(-x, y, 1.f);
    return __builtin_fmaf(e, y, y);
}

__device__ __forceinline__ bool wave_any(bool p) { return __builtin_amdgcn_ballot_w64(p) != 0; }

// sqrtf(x), bit-exact for every x.
__device__ __forceinline__ float sqrt_exact(float x)
{
    if (!wave_any(!sqrt_nr_ok(x))) return sqrt_nr(x);
    return sqrt_rn(x);
}

// 1.f / sqrtf(d), bit-exact for every d (the reference's normalisation factor:
// vec.h:50 vnorm, common.h:19 NORMALIZE).  For d in sqrt_nr's range sqrtf(d)
// lies in [2^-48, 2^64), inside rcp_nr's range.
__device__ __forceinline__ float inv_len(float d)
{
    if (!wave_any(!sqrt_nr_ok(d))) return rcp_nr(sqrt_nr(d));
    return 1.f / sqrt_rn(d);
}

// (int)f as the reference's x86-64 build converts it (cvttss2si): truncation,
// and INT_MIN -- the "integer indefinite" value -- for NaN and for values
// outside [-2^31, 2^31).  v_cvt_i32_f32 saturates instead (and maps NaN to
// 0), which would turn an overflowing accumulator into 255 where the
// reference packs (unsigned char)INT_MIN = 0.
__device__ __forceinline__ int cvt_i32_x86(float f)
{
    return (f >= -2147483648.0f && f < 2147483648.0f) ? (int)f : (int)0x80000000u;
}

// Wave-level u64 sum (64 lanes) used for the optional work counters.
__device__ __forceinline__ unsigned long long wave_sum_u64(unsigned long long v)
{
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
    return v;
}

// Adds per-lane counters into d[0..N) with one atomic per wave.  Every lane
// of the wave must call it (full-wave shuffles).
template <int N>
__device__ __forceinline__ void flush_counters(unsigned long long *d, const unsigned long long (&c)[N])
{
#pragma unroll
    for (int k = 0; k < N; k++) {
        unsigned long long s = wave_sum_u64(c[k]);
        if ((threadIdx.x & 63) == 0 && s) atomicAdd(d + k, s);
    }
}

}  // namespace rt

#endif
