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

__device__ __forceinline__ float sqrt_rsq1(float x)     // one transcendental
{
    const float y = __builtin_amdgcn_rsqf(x);
    const float s0 = x * y;
    const float r = __builtin_fmaf(-s0, s0, x);
    return __builtin_fmaf(r, 0.5f * y, s0);
}

__device__ __forceinline__ float inv_len_rsq1(float d)  // 1/sqrtf(d) (double rounding), one transcendental
{
    const float y = __builtin_amdgcn_rsqf(d);
    const float s0 = d * y;
    const float r = __builtin_fmaf(-s0, s0, d);
    const float s = __builtin_fmaf(r, 0.5f * y, s0);
    const float e = __builtin_fmaf(-s, y, 1.f);
    return __builtin_fmaf(e, y, y);
}

__device__ __forceinline__ float inv_len_rsq1b(float d)  // variant: Newton on the reciprocal twice
{
    const float y = __builtin_amdgcn_rsqf(d);
    const float s0 = d * y;
    const float r = __builtin_fmaf(-s0, s0, d);
    const float s = __builtin_fmaf(r, 0.5f * y, s0);
    float z = y;
    float e = __builtin_fmaf(-s, z, 1.f);
    z = __builtin_fmaf(e, z, z);
    e = __builtin_fmaf(-s, z, 1.f);
    return __builtin_fmaf(e, z, z);
}

__global__ void check(int fn, uint32_t hi_bits, unsigned long long *bucket, unsigned long long *dump)
{
    const uint32_t lo = threadIdx.x + blockIdx.x * blockDim.x;   // low 24 bits
    const uint32_t bits = (hi_bits << 24) | (lo & 0xffffffu);
    const float x = __uint_as_float(bits);
    float ref, got;
    if (fn == 0) { ref = 1.f / x; got = rcp_cand(x); }
    else if (fn == 1) { ref = sqrtf(x); got = sqrt_cand(x); }
    else if (fn == 2) { ref = sqrtf(x); got = sqrt_fix(x); }
    else if (fn == 3) { ref = sqrtf(x); got = sqrt_rsq1(x); }
    else if (fn == 4) { ref = 1.f / sqrtf(x); got = inv_len_rsq1(x); }
    else { ref = 1.f / sqrtf(x); got = inv_len_rsq1b(x); }
    const bool same = (ref != ref && got != got) || __float_as_uint(ref) == __float_as_uint(got);
    if (!same) {
        atomicAdd(&bucket[(bits >> 23) & 0x1ff], 1ull);
        const uint32_t e = (bits >> 23) & 0xff;
        if (fn == 4 && e >= 60 && e <= 70 && !(bits >> 31)) {
            const unsigned long long k = atomicAdd(&dump[0], 1ull);
            if (k < 16) { dump[1 + 2 * k] = bits; dump[2 + 2 * k] = __float_as_uint(got) | ((unsigned long long)__float_as_uint(ref) << 32); }
        }
    }
}

int main()
{
    unsigned long long *d;
    hipMalloc(&d, 8 * 4096);
    hipMemset(d, 0, 8 * 4096);
    for (int fn = 0; fn < 6; fn++)
        for (uint32_t hb = 0; hb < 256; hb++)
            hipLaunchKernelGGL(check, dim3(1 << 16), dim3(256), 0, 0, fn, hb, d + 512 * fn, d + 3500);
    static unsigned long long h[4096];
    hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
    for (int k = 0; k < 16 && k < (int)h[3500]; k++) printf("inv_len bad x=%08llx got=%08llx ref=%08llx\n", h[3501 + 2 * k], h[3502 + 2 * k] & 0xffffffffull, h[3502 + 2 * k] >> 32);
    const char *names[6] = {"rcp_newton", "sqrt_newton", "sqrt_fix_notiny", "sqrt_rsq1", "inv_len_rsq1", "inv_len_rsq1b"};
    for (int fn = 0; fn < 6; fn++) {
        unsigned long long tot = 0;
        for (int b = 0; b < 512; b++) tot += h[512 * fn + b];
        printf("%s: %llu mismatches\n", names[fn], tot);
        for (int b = 0; b < 512; b++)
            if (h[512 * fn + b]) printf("   sign %d exp %3d (2^%d): %llu\n", b >> 8, b & 255, (b & 255) - 127, h[512 * fn + b]);
    }
    return 0;
}
