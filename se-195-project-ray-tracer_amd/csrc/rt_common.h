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
