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

// acos.zig acos32 (musl acosf)
RTW_LIBM_FN float rtw_acosf(float x) {
    const float pio2_hi = 1.5707962513e+00f, pio2_lo = 7.5497894159e-08f;
    const uint32_t hx = rtw_lm_bits(x);
    const uint32_t ix = hx & 0x7FFFFFFFu;
    if (ix >= 0x3F800000u) {  // |x| >= 1 or nan
        if (ix == 0x3F800000u) return (hx >> 31) ? 2.0f * pio2_hi + 0x1.0p-120f : 0.0f;
        return rtw_lm_float(0x7FC00000u);
    }
    if (ix < 0x3F000000u) {  // |x| < 0.5
        if (ix <= 0x32800000u) return pio2_hi + 0x1.0p-120f;  // |x| < 2^-26
        return pio2_hi - (x - (pio2_lo - x * rtw_lm_acos_r(x * x)));
    }
    if (hx >> 31) {  // x < -0.5
        const float z = (1.0f + x) * 0.5f;
        const float s = __builtin_sqrtf(z);
        const float w = rtw_lm_acos_r(z) * s - pio2_lo;
        return 2.0f * (pio2_hi - (s + w));
    }
    // x > 0.5
    const float z = (1.0f - x) * 0.5f;
    const float s = __builtin_sqrtf(z);
    const float df = rtw_lm_float(rtw_lm_bits(s) & 0xFFFFF000u);
    const float c = (z - df * df) / (s + df);
    const float w = rtw_lm_acos_r(z) * s + c;
    return 2.0f * (df + w);
}

// atan.zig atan32 (musl atanf)
RTW_LIBM_FN float rtw_atanf(float x_) {
    const float atanhi[4] = {4.6364760399e-01f, 7.8539812565e-01f, 9.8279368877e-01f, 1.5707962513e+00f};
    const float atanlo[4] = {5.0121582440e-09f, 3.7748947079e-08f, 3.4473217170e-08f, 7.5497894159e-08f};
    const float aT[5] = {3.3333328366e-01f, -1.9999158382e-01f, 1.4253635705e-01f, -1.0648017377e-01f,
                         6.1687607318e-02f};
    float x = x_;
    uint32_t ix = rtw_lm_bits(x);
    const uint32_t sign = ix >> 31;
    ix &= 0x7FFFFFFFu;
    int id;
    if (ix >= 0x4C800000u) {  // |x| >= 2^26
        if (ix > 0x7F800000u) return x;  // nan
        const float z = atanhi[3] + 0x1.0p-120f;
        return sign ? -z : z;
    }
    if (ix < 0x3EE00000u) {  // |x| < 0.4375
        if (ix < 0x39800000u) return x;  // |x| < 2^-12
        id = -1;
    } else {
        x = __builtin_fabsf(x);
        if (ix < 0x3F980000u) {  // |x| < 1.1875
            if (ix < 0x3F300000u) {  // 7/16 <= |x| < 11/16
                id = 0;
                x = (2.0f * x - 1.0f) / (2.0f + x);
            } else {  // 11/16 <= |x| < 19/16
                id = 1;
                x = (x - 1.0f) / (x + 1.0f);
            }
        } else {
            if (ix < 0x401C0000u) {  // |x| < 2.4375
                id = 2;
                x = (x - 1.5f) / (1.0f + 1.5f * x);
            } else {  // 2.4375 <= |x| < 2^26
                id = 3;
                x = -1.0f / x;
            }
        }
    }
    const float z = x * x;
    const float w = z * z;
    const float s1 = z * (aT[0] + w * (aT[2] + w * aT[4]));
    const float s2 = w * (aT[1] + w * aT[3]);
    if (id < 0) return x - x * (s1 + s2);
    const float zz = atanhi[id] - ((x * (s1 + s2) - atanlo[id]) - x);
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

// sin.zig sinf (musl)
RTW_LIBM_FN float rtw_sinf(float x) {
    const double s1pio2 = 1 * 1.57079632679489661923, s2pio2 = 2 * 1.57079632679489661923,
                 s3pio2 = 3 * 1.57079632679489661923, s4pio2 = 4 * 1.57079632679489661923;
    uint32_t ix = rtw_lm_bits(x);
    const uint32_t sign = ix >> 31;
    ix &= 0x7FFFFFFFu;
    if (ix <= 0x3F490FDAu) {  // |x| ~<= pi/4
        if (ix < 0x39800000u) return x;  // |x| < 2^-12
        return rtw_lm_sindf(x);
    }
    if (ix <= 0x407B53D1u) {  // |x| ~<= 5*pi/4
        if (ix <= 0x4016CBE3u) {  // |x| ~<= 3*pi/4
            if (sign) return -rtw_lm_cosdf((double)x + s1pio2);
            return rtw_lm_cosdf((double)x - s1pio2);
        }
        return rtw_lm_sindf(sign ? -((double)x + s2pio2) : -((double)x - s2pio2));
    }
    if (ix <= 0x40E231D5u) {  // |x| ~<= 9*pi/4
        if (ix <= 0x40AFEDDFu) {  // |x| ~<= 7*pi/4
            if (sign) return rtw_lm_cosdf((double)x + s3pio2);
            return -rtw_lm_cosdf((double)x - s3pio2);
        }
        return rtw_lm_sindf(sign ? (double)x + s4pio2 : (double)x - s4pio2);
    }
    if (ix >= 0x7F800000u) return x - x;  // sin(inf or nan) = nan
    if (ix >= 0x4DC90FDBu) return rtw_lm_float(0x7FC00000u);  // beyond the medium-size reduction
    double y;
    const int n = rtw_lm_rem_pio2f(x, &y);
    switch (n & 3) {
        case 0: return rtw_lm_sindf(y);
        case 1: return rtw_lm_cosdf(y);
        case 2: return rtw_lm_sindf(-y);
        default: return -rtw_lm_cosdf(y);
    }
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
