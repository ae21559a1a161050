// rtw_libm.h -- the f32 transcendental functions the reference's hot path calls,
// restated from the algorithms the Zig toolchain compiles them to, for the device
// (and any C/C++ host: the qualifiers vanish outside hipcc).
//
//   Sphere.getSphereUV (objects.zig:109-110):  std.math.acos(f32), std.math.atan2(f32)
//      Zig std lib/std/math/acos.zig acos32 and atan2.zig atan2_32 / atan.zig atan32:
//      ports of musl acosf / atan2f / atanf (FreeBSD e_acosf.c, e_atan2f.c, s_atanf.c).
//   NoiseTexture.value (textures.zig:120):  @sin(f32)
//   ConstantMedium.hit (objects.zig:484):   @log(f32)
//      lowered by LLVM to the sinf / logf libcalls, which Zig's compiler_rt provides as
//      ports of musl sinf (__sindf / __cosdf double kernels, __rem_pio2f) and the
//      FreeBSD-derived logf (Lg1..Lg4).  (When the reference links a C library those two
//      symbols may resolve to its libm instead -- parity unpinned at that boundary; the
//      CPU restatement, oracle/rtw_oracle.c, restates the same algorithms independently.)
//
// Same fp32/fp64 operations in the same order on every target (-ffp-contract=off, IEEE
// division and sqrt), so the device and the CPU restatement agree bit for bit.  Domain:
// rtw_sinf implements the medium-size reduction (|x| < 2^28 * pi/2, far beyond any scene
// coordinate); larger arguments, which the reference would reduce with __rem_pio2_large,
// return NaN here.
#pragma once
#include <stdint.h>
#include <string.h>
#ifndef __cplusplus
#include <stdbool.h>
#endif

#if defined(__HIPCC__)
#define RTW_LIBM_FN __host__ __device__ static inline
#else
#define RTW_LIBM_FN static inline
#endif

#pragma clang fp contract(off)

RTW_LIBM_FN uint32_t rtw_lm_bits(float x) {
    uint32_t u;
    memcpy(&u, &x, 4);
    return u;
}
RTW_LIBM_FN float rtw_lm_float(uint32_t u) {
    float x;
    memcpy(&x, &u, 4);
    return x;
}

// acos.zig r32
RTW_LIBM_FN float rtw_lm_acos_r(float z) {
    const float pS0 = 1.6666586697e-01f, pS1 = -4.2743422091e-02f, pS2 = -8.6563630030e-03f,
                qS1 = -7.0662963390e-01f;
    const float p = z * (pS0 + z * (pS1 + z * pS2));
    const float q = 1.0f + z * qS1;
    return p / q;
}

// acos.zig acos32 (musl acosf).  The three ranges are evaluated with selects (the wave
// would execute every branch its lanes take): each result is the same fp32 expression
// of the source, so the selected value is bit-identical to the branchy form.
RTW_LIBM_FN float rtw_acosf(float x) {
    const float pio2_hi = 1.5707962513e+00f, pio2_lo = 7.5497894159e-08f;
    const uint32_t hx = rtw_lm_bits(x);
    const uint32_t ix = hx & 0x7FFFFFFFu;
    if (ix >= 0x3F800000u) {  // |x| >= 1 or nan
        if (ix == 0x3F800000u) return (hx >> 31) ? 2.0f * pio2_hi + 0x1.0p-120f : 0.0f;
        return rtw_lm_float(0x7FC00000u);
    }
    const bool small = ix < 0x3F000000u;       // |x| < 0.5
    const bool neg = (hx >> 31) != 0;          // (big) x < -0.5
    const float zb = neg ? (1.0f + x) * 0.5f : (1.0f - x) * 0.5f;
    const float z = small ? x * x : zb;
    const float r = rtw_lm_acos_r(z);
    const float s = __builtin_sqrtf(zb);
    // |x| < 0.5
    const float v_small = (ix <= 0x32800000u) ? pio2_hi + 0x1.0p-120f : pio2_hi - (x - (pio2_lo - x * r));
    // x < -0.5
    const float v_neg = 2.0f * (pio2_hi - (s + (r * s - pio2_lo)));
    // x > 0.5
    const float df = rtw_lm_float(rtw_lm_bits(s) & 0xFFFFF000u);
    const float c = (zb - df * df) / (s + df);
    const float v_pos = 2.0f * (df + (r * s + c));
    return small ? v_small : (neg ? v_neg : v_pos);
}

// atan.zig atan32 (musl atanf).  The argument reduction's five forms are one quotient
// (a*x + b) / (c*x + d) with per-range constants that reproduce each form's fp32
// operations exactly (2x and 0*x, 1*x, x + 0 are exact for these finite x), so no lane
// diverges; the result is bit-identical to the branchy source.
RTW_LIBM_FN float rtw_atanf(float x_) {
    const float aT0 = 3.3333328366e-01f, aT1 = -1.9999158382e-01f, aT2 = 1.4253635705e-01f,
                aT3 = -1.0648017377e-01f, aT4 = 6.1687607318e-02f;
    uint32_t ix = rtw_lm_bits(x_);
    const uint32_t sign = ix >> 31;
    ix &= 0x7FFFFFFFu;
    if (ix >= 0x4C800000u) {  // |x| >= 2^26
        if (ix > 0x7F800000u) return x_;  // nan
        const float z = 1.5707962513e+00f + 0x1.0p-120f;
        return sign ? -z : z;
    }
    if (ix < 0x39800000u) return x_;  // |x| < 2^-12
    // id: -1 |x| < 0.4375, 0 < 11/16, 1 < 19/16, 2 < 2.4375, 3 beyond
    const int id = ix < 0x3EE00000u ? -1 : ix < 0x3F300000u ? 0 : ix < 0x3F980000u ? 1 : ix < 0x401C0000u ? 2 : 3;
    const float ax = id < 0 ? x_ : __builtin_fabsf(x_);
    //            num = a*x + b           den = c*x + d
    // id -1:     1*x + 0                 0*x + 1        -> x
    // id  0:     2*x - 1                 1*x + 2        -> (2x - 1) / (2 + x)
    // id  1:     1*x - 1                 1*x + 1        -> (x - 1) / (x + 1)
    // id  2:     1*x - 1.5               1.5*x + 1      -> (x - 1.5) / (1 + 1.5x)
    // id  3:     0*x - 1                 1*x + 0        -> -1 / x
    const float ka = id == 0 ? 2.0f : (id == 3 ? 0.0f : 1.0f);
    const float kb = id < 0 ? 0.0f : (id == 2 ? -1.5f : (id == 0 || id == 1 || id == 3 ? -1.0f : 0.0f));
    const float kc = id < 0 ? 0.0f : (id == 2 ? 1.5f : 1.0f);
    const float kd = id < 0 ? 1.0f : (id == 0 ? 2.0f : (id == 3 ? 0.0f : 1.0f));
    const float x = (ka * ax + kb) / (kc * ax + kd);
    const float z = x * x;
    const float w = z * z;
    const float s1 = z * (aT0 + w * (aT2 + w * aT4));
    const float s2 = w * (aT1 + w * aT3);
    const float hi = id == 0 ? 4.6364760399e-01f : id == 1 ? 7.8539812565e-01f : id == 2 ? 9.8279368877e-01f
                                                                                      : 1.5707962513e+00f;
    const float lo = id == 0 ? 5.0121582440e-09f : id == 1 ? 3.7748947079e-08f : id == 2 ? 3.4473217170e-08f
                                                                                      : 7.5497894159e-08f;
    if (id < 0) return x - x * (s1 + s2);
    const float zz = hi - ((x * (s1 + s2) - lo) - x);
    return sign ? -zz : zz;
}

// atan2.zig atan2_32 (musl atan2f)
RTW_LIBM_FN float rtw_atan2f(float y, float x) {
    const float pi = 3.1415927410e+00f, pi_lo = -8.7422776573e-08f;
    if (x != x || y != y) return x + y;
    uint32_t ix = rtw_lm_bits(x), iy = rtw_lm_bits(y);
    if (ix == 0x3F800000u) return rtw_atanf(y);  // x = 1.0
    const uint32_t m = ((iy >> 31) & 1u) | ((ix >> 30) & 2u);  // 2 * sign(x) + sign(y)
    ix &= 0x7FFFFFFFu;
    iy &= 0x7FFFFFFFu;
    if (iy == 0) {  // y = 0
        switch (m) {
            case 0:
            case 1: return y;
            case 2: return pi;
            default: return -pi;
        }
    }
    if (ix == 0) return (m & 1u) ? -pi / 2.0f : pi / 2.0f;  // x = 0
    if (ix == 0x7F800000u) {  // x = inf
        if (iy == 0x7F800000u) {
            switch (m) {
                case 0: return pi / 4.0f;
                case 1: return -pi / 4.0f;
                case 2: return 3.0f * pi / 4.0f;
                default: return -3.0f * pi / 4.0f;
            }
        }
        switch (m) {
            case 0: return 0.0f;
            case 1: return -0.0f;
            case 2: return pi;
            default: return -pi;
        }
    }
    if (ix + (26u << 23) < iy || iy == 0x7F800000u) return (m & 1u) ? -pi / 2.0f : pi / 2.0f;  // |y/x| > 2^26
    float z;
    if ((m & 2u) && iy + (26u << 23) < ix)  // |y/x| < 2^-26, x < 0
        z = 0.0f;
    else
        z = rtw_atanf(__builtin_fabsf(y / x));
    switch (m) {
        case 0: return z;
        case 1: return -z;
        case 2: return pi - (z - pi_lo);
        default: return (z - pi_lo) - pi;
    }
}

// trig.zig __sindf / __cosdf (musl): double kernels on |x| <~ pi/4
RTW_LIBM_FN float rtw_lm_sindf(double x) {
    const double S1 = -0x15555554cbac77.0p-55, S2 = 0x111110896efbb2.0p-59, S3 = -0x1a00f9e2cae774.0p-65,
                 S4 = 0x16cd878c3b46a7.0p-71;
    const double z = x * x;
    const double w = z * z;
    const double r = S3 + z * S4;
    const double s = z * x;
    return (float)((x + s * (S1 + z * S2)) + s * w * r);
}
RTW_LIBM_FN float rtw_lm_cosdf(double x) {
    const double C0 = -0x1ffffffd0c5e81.0p-54, C1 = 0x155553e1053a42.0p-57, C2 = -0x16c087e80f1e27.0p-62,
                 C3 = 0x199342e0ee5069.0p-68;
    const double z = x * x;
    const double w = z * z;
    const double r = C2 + z * C3;
    return (float)(((1.0 + z * C0) + w * C1) + (w * z) * r);
}

// rem_pio2f.zig (musl __rem_pio2f), medium-size arguments: n and y = x - n*pi/2 in double
RTW_LIBM_FN int rtw_lm_rem_pio2f(float x, double* y) {
    const double toint = 1.5 / 2.220446049250313080847e-16;  // 1.5 / DBL_EPSILON
    const double pio4 = 0x1.921fb6p-1, invpio2 = 6.36619772367581382433e-01,
                 pio2_1 = 1.57079631090164184570e+00, pio2_1t = 1.58932547735281966916e-08;
    double fn = (double)x * invpio2 + toint - toint;
    int n = (int)fn;
    *y = (double)x - fn * pio2_1 - fn * pio2_1t;
    if (*y < -pio4) {
        n--;
        fn--;
        *y = (double)x - fn * pio2_1 - fn * pio2_1t;
    } else if (*y > pio4) {
        n++;
        fn++;
        *y = (double)x - fn * pio2_1 - fn * pio2_1t;
    }
    return n;
}

// sin.zig sinf (musl).  The five argument ranges and the medium-size reduction give
// (y, kernel, sign) with the source's exact double operations (x + c == x - (-c) and
// -(a + b) == (-a) + (-b) in IEEE arithmetic); both kernels are evaluated and selected,
// so the wave runs one path: bit-identical to the branchy source.
RTW_LIBM_FN float rtw_sinf(float x) {
    const double s1pio2 = 1 * 1.57079632679489661923, s2pio2 = 2 * 1.57079632679489661923,
                 s3pio2 = 3 * 1.57079632679489661923, s4pio2 = 4 * 1.57079632679489661923;
    uint32_t ix = rtw_lm_bits(x);
    const bool sign = (ix >> 31) != 0;
    ix &= 0x7FFFFFFFu;
    if (ix < 0x39800000u) return x;  // |x| < 2^-12 (and +-0)
    if (ix >= 0x7F800000u) return x - x;  // sin(inf or nan) = nan
    if (ix >= 0x4DC90FDBu) return rtw_lm_float(0x7FC00000u);  // beyond the medium-size reduction
    const double xd = (double)x;
    double y;
    bool use_cos, neg_out = false;
    if (ix <= 0x40E231D5u) {  // |x| ~<= 9*pi/4: one subtraction of a multiple of pi/2
        double off;
        bool neg_in = false;
        if (ix <= 0x3F490FDAu) {  // |x| ~<= pi/4: sin(x)
            off = 0.0;
            use_cos = false;
        } else if (ix <= 0x4016CBE3u) {  // ~<= 3pi/4: sign ? -cos(x + pi/2) : cos(x - pi/2)
            off = sign ? -s1pio2 : s1pio2;
            use_cos = true;
            neg_out = sign;
        } else if (ix <= 0x407B53D1u) {  // ~<= 5pi/4: sin(-(x -+ pi))
            off = sign ? -s2pio2 : s2pio2;
            use_cos = false;
            neg_in = true;
        } else if (ix <= 0x40AFEDDFu) {  // ~<= 7pi/4: sign ? cos(x + 3pi/2) : -cos(x - 3pi/2)
            off = sign ? -s3pio2 : s3pio2;
            use_cos = true;
            neg_out = !sign;
        } else {  // ~<= 9pi/4: sin(x -+ 2pi)
            off = sign ? -s4pio2 : s4pio2;
            use_cos = false;
        }
        y = (ix <= 0x3F490FDAu) ? xd : xd - off;
        if (neg_in) y = -y;
    } else {
        const int n = rtw_lm_rem_pio2f(x, &y);
        use_cos = (n & 1) != 0;
        neg_out = (n & 3) == 3;
        if ((n & 3) == 2) y = -y;
    }
    // __sindf and __cosdf as one evaluation with selected operands, each step the same IEEE
    // double operation as in the kernel it stands for:
    //   sin: (y + s*(S1 + z*S2)) + (s*w)*(S3 + z*S4),   s = z*y
    //   cos: ((1 + z*C0) + w*C1) + (w*z)*(C2 + z*C3)
    const double S1 = -0x15555554cbac77.0p-55, S2 = 0x111110896efbb2.0p-59, S3 = -0x1a00f9e2cae774.0p-65,
                 S4 = 0x16cd878c3b46a7.0p-71;
    const double C0 = -0x1ffffffd0c5e81.0p-54, C1 = 0x155553e1053a42.0p-57, C2 = -0x16c087e80f1e27.0p-62,
                 C3 = 0x199342e0ee5069.0p-68;
    const double z = y * y;
    const double w = z * z;
    const double sz = z * y;
    const double a = use_cos ? 1.0 + z * C0 : y;
    const double b = use_cos ? w : sz;
    const double c = use_cos ? C1 : S1 + z * S2;
    const double r = (use_cos ? C2 : S3) + z * (use_cos ? C3 : S4);
    const float v = (float)((a + b * c) + (w * (use_cos ? z : sz)) * r);
    return neg_out ? -v : v;
}

// log.zig logf (FreeBSD e_logf.c as ported by musl / Zig compiler_rt)
RTW_LIBM_FN float rtw_logf(float x_) {
    const float ln2_hi = 6.9313812256e-01f, ln2_lo = 9.0580006145e-06f;
    const float Lg1 = 0xaaaaaa.0p-24f, Lg2 = 0xccce13.0p-25f, Lg3 = 0x91e9ee.0p-25f, Lg4 = 0xf89e26.0p-26f;
    float x = x_;
    uint32_t ix = rtw_lm_bits(x);
    int k = 0;
    if (ix < 0x00800000u || (ix >> 31)) {  // x < 2^-126 or negative
        if ((ix << 1) == 0) return -__builtin_inff();  // log(+-0) = -inf
        if (ix >> 31) return rtw_lm_float(0x7FC00000u);  // log(-#) = nan
        k -= 25;  // subnormal: scale x
        x *= 0x1.0p25f;
        ix = rtw_lm_bits(x);
    } else if (ix >= 0x7F800000u) {
        return x;
    } else if (ix == 0x3F800000u) {
        return 0.0f;
    }
    // x into [sqrt(2) / 2, sqrt(2)]
    ix += 0x3F800000u - 0x3F3504F3u;
    k += (int)(ix >> 23) - 0x7F;
    ix = (ix & 0x007FFFFFu) + 0x3F3504F3u;
    x = rtw_lm_float(ix);
    const float f = x - 1.0f;
    const float s = f / (2.0f + f);
    const float z = s * s;
    const float w = z * z;
    const float t1 = w * (Lg2 + w * Lg4);
    const float t2 = z * (Lg1 + w * Lg3);
    const float R = t2 + t1;
    const float hfsq = 0.5f * f * f;
    const float dk = (float)k;
    return s * (hfsq + R) + dk * ln2_lo - hfsq + f + dk * ln2_hi;
}
