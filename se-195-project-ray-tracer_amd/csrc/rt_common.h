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

// Correctly rounded sqrtf.  hipcc's sqrtf expands to v_sqrt_f32 (<= 1 ulp)
// plus a two-residual fixup (s -/+ 1 ulp against fma(-s', s, x)), wrapped in
// a 2^32 pre-scale for x < 2^-96 and a +-0/inf class select.  For x >= 2^-96,
// x = +-0, +inf and NaN the fixup alone is exact (v_sqrt of 0 / inf / NaN
// needs no correction and the residual tests leave it unchanged), so only
// x below 2^-96 other than +-0 (tiny or negative) take the library path -- a
// divergent branch the ray-trace path never enters (its arguments are sums of
// squares or checked non-negative).  Checked against sqrtf for every float on the
// device (tests/test_gpu_math.py).
__device__ __forceinline__ float sqrt_rn(float x)
{
    float s = __builtin_amdgcn_sqrtf(x);
    const float s_dn = __uint_as_float(__float_as_uint(s) - 1u);
    const float s_up = __uint_as_float(__float_as_uint(s) + 1u);
    const float r_dn = __builtin_fmaf(-s_dn, s, x);
    const float r_up = __builtin_fmaf(-s_up, s, x);
    s = (r_dn <= 0.f) ? s_dn : s;
    s = (r_up > 0.f) ? s_up : s;
    if (x < 0x1p-96f && x != 0.f) s = sqrtf(x);   // tiny or negative (v_sqrt flushes -denormals)
    return s;
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
