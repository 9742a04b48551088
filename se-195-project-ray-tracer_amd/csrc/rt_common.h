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
