// rt_glibc_math.h -- bit-exact float libm for the ray-trace hot path, host + gfx950 device.
//
// The reference's CPU paths (the parity oracle) call glibc's float libm:
//   Whitted  powf(dot, 20)            raytracer3.0.06.no_rec.samp/raytracer.cpp:165
//            expf(absorbance)         raytracer.cpp:487-489 (exp(float) -> expf)
//   smallpt  sinf/cosf(2*PI*u)        smallptgpu-v1.6/geomfunc.h:65-66,261-262
//            powf(clamp(c), 1/2.2f)   smallptgpu-v1.6/vec.h:62 (toInt)
// glibc 2.35 on x86-64 (this image and the GPU box) dispatches these to its
// FMA builds of the ARM optimized-routines algorithms: double-precision
// table + polynomial evaluations rounded once to float.  This header restates
// those evaluations operation for operation (every fma below is one fused op
// in glibc's FMA build), so the same source compiled for the host and for
// gfx950 (v_fma_f64 / v_mul_f64 / v_cvt_f32_f64, all IEEE round-to-nearest)
// returns glibc's bits.  Constants are glibc 2.35's published tables
// (__powf_log2_data, __exp2f_data, __sincosf_table).  Equality with the host
// libm is checked exhaustively over the path's input domains by
// tests/test_glibc_math.py (host) and tests/test_gpu_math.py (device).
//
// Domains covered: powf for x >= 0 (any finite y), expf for all x,
// sinf/cosf for |x| < 120 (the path only evaluates 2*PI*u, u in [0,1)).
#ifndef RT_GLIBC_MATH_H
#define RT_GLIBC_MATH_H

#include <stdint.h>
#include "rt_glibc_pow_tables.h"

#if defined(__HIPCC__)
#define RTM_HD __host__ __device__ __forceinline__
#else
#define RTM_HD static inline
#endif

namespace rtm {

RTM_HD uint32_t f2u(float f) { uint32_t u; __builtin_memcpy(&u, &f, 4); return u; }
RTM_HD float u2f(uint32_t u) { float f; __builtin_memcpy(&f, &u, 4); return f; }
RTM_HD uint64_t d2u(double d) { uint64_t u; __builtin_memcpy(&u, &d, 8); return u; }
RTM_HD double u2d(uint64_t u) { double d; __builtin_memcpy(&d, &u, 8); return d; }
RTM_HD double fma_d(double a, double b, double c) { return __builtin_fma(a, b, c); }

// __exp2f_data.tab: asuint64(2^(i/32)) - (i << 47)
RTM_HD uint64_t exp2f_tab(uint32_t i)
{
    constexpr uint64_t T[32] = {
        0x3ff0000000000000ull, 0x3fefd9b0d3158574ull, 0x3fefb5586cf9890full, 0x3fef9301d0125b51ull,
        0x3fef72b83c7d517bull, 0x3fef54873168b9aaull, 0x3fef387a6e756238ull, 0x3fef1e9df51fdee1ull,
        0x3fef06fe0a31b715ull, 0x3feef1a7373aa9cbull, 0x3feedea64c123422ull, 0x3feece086061892dull,
        0x3feebfdad5362a27ull, 0x3feeb42b569d4f82ull, 0x3feeab07dd485429ull, 0x3feea47eb03a5585ull,
        0x3feea09e667f3bcdull, 0x3fee9f75e8ec5f74ull, 0x3feea11473eb0187ull, 0x3feea589994cce13ull,
        0x3feeace5422aa0dbull, 0x3feeb737b0cdc5e5ull, 0x3feec49182a3f090ull, 0x3feed503b23e255dull,
        0x3feee89f995ad3adull, 0x3feeff76f2fb5e47ull, 0x3fef199bdd85529cull, 0x3fef3720dcef9069ull,
        0x3fef5818dcfba487ull, 0x3fef7c97337b9b5full, 0x3fefa4afa2a490daull, 0x3fefd0765b6e4540ull};
    return T[i & 31];
}

// __powf_log2_data.tab: {invc, logc}, 16 subintervals around 1.
RTM_HD double powf_invc(uint32_t i)
{
    constexpr double T[16] = {
        0x1.661ec79f8f3bep+0, 0x1.571ed4aaf883dp+0, 0x1.49539f0f010b0p+0, 0x1.3c995b0b80385p+0,
        0x1.30d190c8864a5p+0, 0x1.25e227b0b8ea0p+0, 0x1.1bb4a4a1a343fp+0, 0x1.12358f08ae5bap+0,
        0x1.0953f419900a7p+0, 0x1.0000000000000p+0, 0x1.e608cfd9a47acp-1, 0x1.ca4b31f026aa0p-1,
        0x1.b2036576afce6p-1, 0x1.9c2d163a1aa2dp-1, 0x1.886e6037841edp-1, 0x1.767dcf5534862p-1};
    return T[i & 15];
}
RTM_HD double powf_logc(uint32_t i)
{
    constexpr double T[16] = {
        -0x1.efec65b963019p-2, -0x1.b0b6832d4fca4p-2, -0x1.7418b0a1fb77bp-2, -0x1.39de91a6dcf7bp-2,
        -0x1.01d9bf3f2b631p-2, -0x1.97c1d1b3b7af0p-3, -0x1.2f9e393af3c9fp-3, -0x1.960cbbf788d5cp-4,
        -0x1.a6f9db6475fcep-5, 0x0.0p+0, 0x1.338ca9f24f53dp-4, 0x1.476a9543891bap-3,
        0x1.e840b4ac4e4d2p-3, 0x1.40645f0c6651cp-2, 0x1.88e9c2c1b9ff8p-2, 0x1.ce0a44eb17bccp-2};
    return T[i & 15];
}

// exp2_inline of e_powf.c: 2^xd rounded once to float; sign_bias selects -.
RTM_HD float powf_exp2(double xd, uint32_t sign_bias)
{
    const double SHIFT = 0x1.8p+47;   // 0x1.8p+52 / 32
    double kd = xd + SHIFT;
    uint64_t ki = d2u(kd);
    kd -= SHIFT;
    double r = xd - kd;
    uint64_t t = exp2f_tab((uint32_t)(ki & 31));
    t += (ki + sign_bias) << 47;
    double s = u2d(t);
    double z = fma_d(r, 0x1.c6af84b912394p-5, 0x1.ebfce50fac4f3p-3);
    double r2 = r * r;
    double y = fma_d(r, 0x1.62e42ff0c52d6p-1, 1.0);
    y = fma_d(z, r2, y);
    y = y * s;
    return (float)y;
}

// log2_inline of e_powf.c (POWF_SCALE_BITS = 0).
RTM_HD double powf_log2(uint32_t ix)
{
    uint32_t tmp = ix - 0x3f330000u;
    uint32_t i = (tmp >> 19) & 15;
    uint32_t top = tmp & 0xff800000u;
    uint32_t iz = ix - top;
    int32_t k = (int32_t)top >> 23;
    double invc = powf_invc(i), logc = powf_logc(i);
    double z = (double)u2f(iz);
    double r = fma_d(z, invc, -1.0);
    double y0 = logc + (double)k;
    double y = fma_d(r, 0x1.27616c9496e0bp-2, -0x1.71969a075c67ap-2);
    double p = fma_d(r, 0x1.ec70a6ca7baddp-2, -0x1.7154748bef6c8p-1);
    double r2 = r * r;
    double q = fma_d(r, 0x1.71547652ab82bp+0, y0);
    double r4 = r2 * r2;
    q = fma_d(r2, p, q);
    y = fma_d(y, r4, q);
    return y;
}

RTM_HD bool zeroinfnan(uint32_t ix) { return 2 * ix - 1 >= 2u * 0x7f800000u - 1; }

// glibc 2.35 __powf (e_powf.c), round-to-nearest.  Negative x is handled only
// for the sign of zero (the ray-trace path never passes x < 0).
RTM_HD float powf(float x, float y)
{
    uint32_t ix = f2u(x), iy = f2u(y);
    if (ix - 0x00800000u >= 0x7f800000u - 0x00800000u || zeroinfnan(iy)) {
        if (zeroinfnan(iy)) {
            if (2 * iy == 0) return 1.0f;
            if (ix == 0x3f800000u) return 1.0f;
            if (2 * ix > 2u * 0x7f800000u || 2 * iy > 2u * 0x7f800000u) return x + y;
            if (2 * ix == 2u * 0x3f800000u) return 1.0f;
            if ((2 * ix < 2u * 0x3f800000u) == !(iy & 0x80000000u)) return 0.0f;
            return y * y;
        }
        if (zeroinfnan(ix)) {
            float x2 = x * x;   // +0 for x = -0 unless y is an odd integer (not used here)
            return (iy & 0x80000000u) ? 1 / x2 : x2;
        }
        if (ix & 0x80000000u) return (x - x) / (x - x);
        if (ix < 0x00800000u) {   // subnormal x: normalise
            ix = f2u(x * 0x1p23f);
            ix &= 0x7fffffffu;
            ix -= 23u << 23;
        }
    }
    double logx = powf_log2(ix);
    double ylogx = (double)y * logx;
    if (((d2u(ylogx) >> 47) & 0xffff) >= (d2u(126.0) >> 47)) {
        if (ylogx > 0x1.fffffffd1d571p+6) return 0x1p97f * 0x1p97f;
        if (ylogx <= -150.0) return 0x1p-95f * 0x1p-95f;
        if (ylogx < -149.0) return 0x1.4p-75f * 0x1.4p-75f;
    }
    return powf_exp2(ylogx, 0);
}

// glibc 2.35 __expf (e_expf.c, FMA build: z*InvLn2N + SHIFT and the
// reduction r are single fused operations).
RTM_HD float expf(float x)
{
    double xd = (double)x;
    uint32_t abstop = (f2u(x) >> 20) & 0x7ff;
    if (abstop >= 0x42b) {   // |x| >= 88 or inf/nan
        if (f2u(x) == 0xff800000u) return 0.0f;
        if (abstop >= 0x7f8) return x + x;
        if (x > 0x1.62e42ep6f) return 0x1p97f * 0x1p97f;
        if (x < -0x1.9fe368p6f) return 0x1p-95f * 0x1p-95f;
        if (x < -0x1.9d1d9ep6f) return 0x1.4p-75f * 0x1.4p-75f;
    }
    const double InvLn2N = 0x1.71547652b82fep+5, SHIFT = 0x1.8p+52;
    double kd = fma_d(InvLn2N, xd, SHIFT);
    uint64_t ki = d2u(kd);
    kd -= SHIFT;
    double r = fma_d(InvLn2N, xd, -kd);
    uint64_t t = exp2f_tab((uint32_t)(ki & 31));
    t += ki << 47;
    double s = u2d(t);
    double z = fma_d(r, 0x1.c6af84b912394p-20, 0x1.ebfce50fac4f3p-13);
    double r2 = r * r;
    double yy = fma_d(r, 0x1.62e42ff0c52d6p-6, 1.0);
    yy = fma_d(z, r2, yy);
    yy = yy * s;
    return (float)yy;
}

// __sincosf_table[0] / [1] polynomial coefficients (s_sincosf.h, sincos_t).
struct sincos_poly { double c0, c1, s1, c2, s2, c3, s3, c4; };
RTM_HD sincos_poly sincos_tab(bool second)
{
    sincos_poly p;
    p.s1 = -0x1.555545995a603p-3;
    p.s2 = 0x1.1107605230bc4p-7;
    p.s3 = -0x1.994eb3774cf24p-13;
    if (!second) {
        p.c0 = 0x1.0000000000000p+0; p.c1 = -0x1.ffffffd0c621cp-2; p.c2 = 0x1.55553e1068f19p-5;
        p.c3 = -0x1.6c087e89a359dp-10; p.c4 = 0x1.99343027bf8c3p-16;
    } else {
        p.c0 = -0x1.0000000000000p+0; p.c1 = 0x1.ffffffd0c621cp-2; p.c2 = -0x1.55553e1068f19p-5;
        p.c3 = 0x1.6c087e89a359dp-10; p.c4 = -0x1.99343027bf8c3p-16;
    }
    return p;
}

// sinf_poly (s_sincosf.h): n even -> sine polynomial in xs, odd -> cosine in s.
RTM_HD float sincos_poly_eval(double xs, double s, const sincos_poly &p, int n)
{
    if ((n & 1) == 0) {
        double s1 = fma_d(s, p.s3, p.s2);
        double x3 = s * xs;
        double x7 = s * x3;
        double ss = fma_d(x3, p.s1, xs);
        return (float)fma_d(s1, x7, ss);
    }
    double x4 = s * s;
    double c1 = fma_d(s, p.c1, p.c0);
    double c2 = fma_d(s, p.c4, p.c3);
    double x6 = s * x4;
    double c = fma_d(x4, p.c2, c1);
    return (float)fma_d(c2, x6, c);
}

// reduce_fast (s_sincosf.h) for |x| < 120: n = round(x * 2/pi), xr = x - n*pi/2.
RTM_HD double sincos_reduce(double xd, int &n)
{
    double r = xd * 0x1.45f306dc9c883p+23;      // hpi_inv (2/pi * 2^24)
    n = ((int32_t)r + 0x800000) >> 24;
    return fma_d(-(double)n, 0x1.921fb54442d18p+0, xd);
}

RTM_HD double sincos_sign(int q) { return (q == 0 || q == 3) ? 1.0 : -1.0; }

// glibc 2.35 sinf for |x| < 120.
RTM_HD float sinf(float x)
{
    double xd = (double)x;
    uint32_t abstop = (f2u(x) >> 20) & 0x7ff;
    if (abstop < 0x3f4) {                 // |x| < pi/4
        if (abstop < 0x398) return x;     // |x| < 2^-12
        return sincos_poly_eval(xd, xd * xd, sincos_tab(false), 0);
    }
    int n;
    double xr = sincos_reduce(xd, n);
    return sincos_poly_eval(xr * sincos_sign(n & 3), xr * xr, sincos_tab((n & 2) != 0), n);
}

// glibc 2.35 cosf for |x| < 120.
RTM_HD float cosf(float x)
{
    double xd = (double)x;
    uint32_t abstop = (f2u(x) >> 20) & 0x7ff;
    if (abstop < 0x3f4) {
        if (abstop < 0x398) return 1.0f;
        return sincos_poly_eval(xd, xd * xd, sincos_tab(false), 1);
    }
    int n;
    double xr = sincos_reduce(xd, n);
    return sincos_poly_eval(xr * sincos_sign(n & 3), xr * xr, sincos_tab((n & 2) != 0), n ^ 1);
}

// Branch-free sinf and cosf of one argument, |x| < 120, bit-identical to the
// two glibc calls above (checked exhaustively by the same tests):
//  * for |x| < pi/4 reduce_fast yields n = 0 and xr = x exactly, so the
//    "small" path of sinf/cosf is the n = 0 case of the reduced path;
//  * __sincosf_table[1] is table[0] with the cosine coefficients negated, and
//    RN(-a*b - c) = -RN(a*b + c), so its cosine polynomial is the exact
//    negation of table[0]'s;
//  * |x| < 2^-12 returns x / 1.0f as glibc's tiny path does.
// One reduction and both polynomials are evaluated for every lane: no
// divergent branches in the wave.
RTM_HD void sincosf(float x, float &sn, float &cs)
{
    const double xd = (double)x;
    const uint32_t abstop = (f2u(x) >> 20) & 0x7ff;
    int n;
    const double xr = sincos_reduce(xd, n);
    const double sg = ((n & 3) == 0 || (n & 3) == 3) ? 1.0 : -1.0;
    const double xs = xr * sg, s = xr * xr;
    // sine polynomial (coefficients common to both tables)
    const double s1 = fma_d(s, -0x1.994eb3774cf24p-13, 0x1.1107605230bc4p-7);
    const double x3 = s * xs;
    const double x7 = s * x3;
    const double ss = fma_d(x3, -0x1.555545995a603p-3, xs);
    const float ps = (float)fma_d(s1, x7, ss);
    // cosine polynomial of table[0]
    const double x4 = s * s;
    const double c1 = fma_d(s, -0x1.ffffffd0c621cp-2, 0x1.0000000000000p+0);
    const double c2 = fma_d(s, 0x1.99343027bf8c3p-16, -0x1.6c087e89a359dp-10);
    const double x6 = s * x4;
    const double c = fma_d(x4, 0x1.55553e1068f19p-5, c1);
    float pc = (float)fma_d(c2, x6, c);
    if (n & 2) pc = -pc;
    const bool odd = (n & 1) != 0;
    sn = odd ? pc : ps;
    cs = odd ? ps : pc;
    if (abstop < 0x398) { sn = x; cs = 1.0f; }
}

// glibc 2.35 double pow (e_pow.c), as its FMA build (__pow_fma, selected on
// every x86-64 host with FMA/AVX2) evaluates it: every fma_d below is one
// vfmadd/vfmsub of that build, every other op a plain IEEE double op, in its
// order.  Used by the Raytracer3.2.03 queue tracer, whose g++-compiled
// `pow(float, 20)` is this function at (double)x, 20.0
// (raytracer_non_OpenCL.c:270).  Covers x > 0 normal and y with
// 0x3be <= top12(y) < 0x43e (|y| in [2^-65, 2^63)); checked against the host
// libm over every float x in (0, 4] at y = 20 (tests/test_glibc_math.py,
// tests/test_gpu_math.py).
RTM_HD double pow_d(double x, double y)
{
    using namespace powtab;
    // log_inline: log(x) = k*ln2 + log(c) + log1p(z/c - 1) as hi + tail.
    const uint64_t ix = d2u(x);
    const uint64_t tmp = ix - 0x3fe6955500000000ull;
    const int i = (int)((tmp >> 45) & 127u);
    const double kd = (double)(int)((int64_t)tmp >> 52);
    const double z = u2d(ix - (tmp & 0xfff0000000000000ull));
    const double invc = LOG[i].invc, logc = LOG[i].logc, logctail = LOG[i].logctail;
    const double r = fma_d(z, invc, -1.0);
    const double t1 = fma_d(kd, LN2HI, logc);
    const double t2 = r + t1;
    const double lo1 = fma_d(kd, LN2LO, logctail);
    const double lo2 = (t1 - t2) + r;
    const double ar = r * A[0];
    const double ar2 = r * ar;
    const double ar3 = r * ar2;
    const double hi = t2 + ar2;
    const double lo3 = fma_d(ar, r, -ar2);
    const double lo4 = (t2 - hi) + ar2;
    const double q1 = fma_d(fma_d(r, A[6], A[5]), ar2, fma_d(r, A[4], A[3]));
    const double q2 = fma_d(ar2, q1, fma_d(r, A[2], A[1]));
    const double lo = fma_d(ar3, q2, ((lo1 + lo2) + lo3) + lo4);
    const double lhi = hi + lo;
    const double ltail = (hi - lhi) + lo;
    // y * log(x) as ehi + elo.
    const double ehi = y * lhi;
    const double elo = fma_d(y, ltail, fma_d(lhi, y, -ehi));
    // exp_inline(ehi, elo, sign_bias = 0).
    const uint32_t abstop = (uint32_t)(d2u(ehi) >> 52) & 0x7ffu;
    bool special = false;
    if (abstop - 0x3c9u > 0x3eu) {
        if ((int)(abstop - 0x3c9u) < 0) return 1.0 + ehi;          // |ehi| < 2^-54
        if (abstop > 0x408u) return (d2u(ehi) >> 63) ? 0.0 : __builtin_inf();   // __math_uflow / oflow
        special = true;                                            // 512 <= |ehi| < 1024
    }
    double kk = fma_d(ehi, INVLN2N, SHIFT);
    const uint64_t ki = d2u(kk);
    kk = kk - SHIFT;
    double er = fma_d(kk, NEGLN2HIN, ehi);
    er = fma_d(kk, NEGLN2LON, er);
    const uint32_t idx = 2u * (uint32_t)(ki & 127u);
    uint64_t sbits = EXP[idx + 1] + (ki << 45);
    er = elo + er;
    const double p23 = fma_d(er, C[1], C[0]);
    const double tr = er + u2d(EXP[idx]);
    const double r2 = er * er;
    const double p45 = fma_d(er, C[3], C[2]);
    const double e1 = fma_d(p23, r2, tr);
    const double etmp = fma_d(p45, r2 * r2, e1);
    if (!special) {
        const double scale = u2d(sbits);
        return fma_d(etmp, scale, scale);
    }
    // specialcase of e_exp.c (the scale's exponent over- or underflowed).
    if ((ki & 0x80000000u) == 0) {
        sbits -= 1009ull << 52;
        const double scale = u2d(sbits);
        return fma_d(scale, etmp, scale) * 0x1p1009;
    }
    sbits += 1022ull << 52;
    const double scale = u2d(sbits);
    double yy = scale + etmp * scale;
    if (__builtin_fabs(yy) < 1.0) {
        const double one = yy < 0.0 ? -1.0 : 1.0;
        const double lo_ = (scale - yy) + etmp * scale;
        const double hi_ = yy + one;
        yy = ((((one - hi_) + yy) + lo_) + hi_) - one;
        if (yy == 0) yy = u2d(sbits & 0x8000000000000000ull);
    }
    return yy * 0x1p-1022;
}

}  // namespace rtm

#endif
