// Exhaustive device-side check of candidate correctly-rounded sequences
// against the library's IEEE f32 division / sqrt, all 2^32 inputs, with
// mismatches bucketed by input exponent.  Exploration tool, not product code.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

__device__ __forceinline__ float rcp_cand(float x)
{
    const float y = __builtin_amdgcn_rcpf(x);
    const float e = __builtin_fmaf(-x, y, 1.f);
    return __builtin_fmaf(e, y, y);
}

__device__ __forceinline__ float sqrt_cand(float x)
{
    // s = v_sqrt; residual r = x - s*s; correction with h ~ 1/(2s)
    const float s = __builtin_amdgcn_sqrtf(x);
    const float h = 0.5f * __builtin_amdgcn_rsqf(x);
    const float r = __builtin_fmaf(-s, s, x);
    return __builtin_fmaf(r, h, s);
}

__device__ __forceinline__ float sqrt_fix(float x)   // LLVM fixup without the tiny scaling
{
    float s = __builtin_amdgcn_sqrtf(x);
    const float s_dn = __uint_as_float(__float_as_uint(s) - 1u);
    const float s_up = __uint_as_float(__float_as_uint(s) + 1u);
    const float r_dn = __builtin_fmaf(-s_dn, s, x);
    const float r_up = __builtin_fmaf(-s_up, s, x);
    s = (r_dn <= 0.f) ? s_dn : s;
    s = (r_up > 0.f) ? s_up : s;
    return s;
}

__global__ void check(int fn, uint32_t hi_bits, unsigned long long *bucket)
{
    const uint32_t lo = threadIdx.x + blockIdx.x * blockDim.x;   // low 24 bits
    const uint32_t bits = (hi_bits << 24) | (lo & 0xffffffu);
    const float x = __uint_as_float(bits);
    float ref, got;
    if (fn == 0) { ref = 1.f / x; got = rcp_cand(x); }
    else if (fn == 1) { ref = sqrtf(x); got = sqrt_cand(x); }
    else { ref = sqrtf(x); got = sqrt_fix(x); }
    const bool same = (ref != ref && got != got) || __float_as_uint(ref) == __float_as_uint(got);
    if (!same) atomicAdd(&bucket[(bits >> 23) & 0x1ff], 1ull);
}

int main()
{
    unsigned long long *d;
    hipMalloc(&d, 512 * 8 * 3);
    hipMemset(d, 0, 512 * 8 * 3);
    for (int fn = 0; fn < 3; fn++)
        for (uint32_t hb = 0; hb < 256; hb++)
            hipLaunchKernelGGL(check, dim3(1 << 16), dim3(256), 0, 0, fn, hb, d + 512 * fn);
    unsigned long long h[512 * 3];
    hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
    const char *names[3] = {"rcp_newton", "sqrt_newton", "sqrt_fix_notiny"};
    for (int fn = 0; fn < 3; fn++) {
        unsigned long long tot = 0;
        for (int b = 0; b < 512; b++) tot += h[512 * fn + b];
        printf("%s: %llu mismatches\n", names[fn], tot);
        for (int b = 0; b < 512; b++)
            if (h[512 * fn + b]) printf("   sign %d exp %3d (2^%d): %llu\n", b >> 8, b & 255, (b & 255) - 127, h[512 * fn + b]);
    }
    return 0;
}
