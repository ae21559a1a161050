/* zig_libm.h -- TEST INFRASTRUCTURE (the oracle's restatement, independent of the
 * product's csrc/rtw_libm.h): the f32 transcendentals of the reference's hot path as
 * the Zig toolchain computes them.
 *   std.math.acos / std.math.atan2 (objects.zig:109-110): lib/std/math/acos.zig acos32,
 *     atan2.zig atan2_32, atan.zig atan32 -- ports of musl acosf / atan2f / atanf.
 *   @sin (textures.zig:120), @log (objects.zig:484): LLVM libcalls sinf / logf, provided
 *     by Zig's compiler_rt as ports of musl sinf (__sindf, __cosdf, __rem_pio2f) and the
 *     FreeBSD-derived logf.  Parity unpinned where the reference resolves them to a C
 *     library's libm instead.
 * Plain C, -ffp-contract=off (oracle/Makefile): the same fp32 / fp64 operations in the
 * same order as those sources. */
#ifndef ZIG_LIBM_H
#define ZIG_LIBM_H
#include <stdint.h>
#include <string.h>

static inline uint32_t zl_u(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }
static inline float zl_f(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }
static inline float zl_nan(void) { return zl_f(0x7FC00000u); }

static float zl_acos_r(float z) {               /* acos.zig r32 */
    const float pS0 = 1.6666586697e-01f, pS1 = -4.2743422091e-02f, pS2 = -8.6563630030e-03f;
    const float qS1 = -7.0662963390e-01f;
    float p = z * (pS0 + z * (pS1 + z * pS2));
    float q = 1.0f + z * qS1;
    return p / q;
}

static float zig_acosf(float x) {               /* acos.zig acos32 */
    const float pio2_hi = 1.5707962513e+00f, pio2_lo = 7.5497894159e-08f;
    uint32_t hx = zl_u(x), ix = hx & 0x7FFFFFFFu;
    float z, s, w, df, c;
    if (ix >= 0x3F800000u) {
        if (ix == 0x3F800000u) return (hx >> 31) ? 2.0f * pio2_hi + 0x1.0p-120f : 0.0f;
        return zl_nan();
    }
    if (ix < 0x3F000000u) {
        if (ix <= 0x32800000u) return pio2_hi + 0x1.0p-120f;
        return pio2_hi - (x - (pio2_lo - x * zl_acos_r(x * x)));
    }
    if (hx >> 31) {
        z = (1 + x) * 0.5f;
        s = sqrtf(z);
        w = zl_acos_r(z) * s - pio2_lo;
        return 2 * (pio2_hi - (s + w));
    }
    z = (1.0f - x) * 0.5f;
    s = sqrtf(z);
    df = zl_f(zl_u(s) & 0xFFFFF000u);
    c = (z - df * df) / (s + df);
    w = zl_acos_r(z) * s + c;
    return 2 * (df + w);
}

static float zig_atanf(float x) {               /* atan.zig atan32 */
    static const float hi[4] = {4.6364760399e-01f, 7.8539812565e-01f, 9.8279368877e-01f, 1.5707962513e+00f};
    static const float lo[4] = {5.0121582440e-09f, 3.7748947079e-08f, 3.4473217170e-08f, 7.5497894159e-08f};
    static const float aT[5] = {3.3333328366e-01f, -1.9999158382e-01f, 1.4253635705e-01f,
                                -1.0648017377e-01f, 6.1687607318e-02f};
    uint32_t ix = zl_u(x), sign = ix >> 31;
    int id;
    float z, w, s1, s2, zz;
    ix &= 0x7FFFFFFFu;
    if (ix >= 0x4C800000u) {
        if (ix > 0x7F800000u) return x;
        z = hi[3] + 0x1.0p-120f;
        return sign ? -z : z;
    }
    if (ix < 0x3EE00000u) {
        if (ix < 0x39800000u) return x;
        id = -1;
    } else {
        x = fabsf(x);
        if (ix < 0x3F980000u) {
            if (ix < 0x3F300000u) { id = 0; x = (2.0f * x - 1.0f) / (2.0f + x); }
            else { id = 1; x = (x - 1.0f) / (x + 1.0f); }
        } else {
            if (ix < 0x401C0000u) { id = 2; x = (x - 1.5f) / (1.0f + 1.5f * x); }
            else { id = 3; x = -1.0f / x; }
        }
    }
    z = x * x;
    w = z * z;
    s1 = z * (aT[0] + w * (aT[2] + w * aT[4]));
    s2 = w * (aT[1] + w * aT[3]);
    if (id < 0) return x - x * (s1 + s2);
    zz = hi[id] - ((x * (s1 + s2) - lo[id]) - x);
    return sign ? -zz : zz;
}

static float zig_atan2f(float y, float x) {     /* atan2.zig atan2_32 */
    const float pi = 3.1415927410e+00f, pi_lo = -8.7422776573e-08f;
    uint32_t ix, iy, m;
    float z;
    if (x != x || y != y) return x + y;
    ix = zl_u(x);
    iy = zl_u(y);
    if (ix == 0x3F800000u) return zig_atanf(y);
    m = ((iy >> 31) & 1u) | ((ix >> 30) & 2u);
    ix &= 0x7FFFFFFFu;
    iy &= 0x7FFFFFFFu;
    if (iy == 0) return m == 0 || m == 1 ? y : (m == 2 ? pi : -pi);
    if (ix == 0) return (m & 1u) ? -pi / 2 : pi / 2;
    if (ix == 0x7F800000u) {
        if (iy == 0x7F800000u) {
            switch (m) {
                case 0: return pi / 4;
                case 1: return -pi / 4;
                case 2: return 3 * pi / 4;
                default: return -3 * pi / 4;
            }
        }
        switch (m) {
            case 0: return 0.0f;
            case 1: return -0.0f;
            case 2: return pi;
            default: return -pi;
        }
    }
    if (ix + (26u << 23) < iy || iy == 0x7F800000u) return (m & 1u) ? -pi / 2 : pi / 2;
    if ((m & 2u) && iy + (26u << 23) < ix) z = 0.0f;
    else z = zig_atanf(fabsf(y / x));
    switch (m) {
        case 0: return z;
        case 1: return -z;
        case 2: return pi - (z - pi_lo);
        default: return (z - pi_lo) - pi;
    }
}

static float zl_sindf(double x) {               /* trig.zig __sindf */
    const double S1 = -0x15555554cbac77.0p-55, S2 = 0x111110896efbb2.0p-59;
    const double S3 = -0x1a00f9e2cae774.0p-65, S4 = 0x16cd878c3b46a7.0p-71;
    double z = x * x, w = z * z, r = S3 + z * S4, s = z * x;
    return (float)((x + s * (S1 + z * S2)) + s * w * r);
}

static float zl_cosdf(double x) {               /* trig.zig __cosdf */
    const double C0 = -0x1ffffffd0c5e81.0p-54, C1 = 0x155553e1053a42.0p-57;
    const double C2 = -0x16c087e80f1e27.0p-62, C3 = 0x199342e0ee5069.0p-68;
    double z = x * x, w = z * z, r = C2 + z * C3;
    return (float)(((1.0 + z * C0) + w * C1) + (w * z) * r);
}

static int zl_rem_pio2f(float x, double* y) {   /* rem_pio2f.zig, medium size */
    const double toint = 1.5 / 2.220446049250313080847e-16, pio4 = 0x1.921fb6p-1;
    const double invpio2 = 6.36619772367581382433e-01, pio2_1 = 1.57079631090164184570e+00;
    const double pio2_1t = 1.58932547735281966916e-08;
    double fn = (double)x * invpio2 + toint - toint;
    int n = (int)fn;
    *y = x - fn * pio2_1 - fn * pio2_1t;
    if (*y < -pio4) { n--; fn--; *y = x - fn * pio2_1 - fn * pio2_1t; }
    else if (*y > pio4) { n++; fn++; *y = x - fn * pio2_1 - fn * pio2_1t; }
    return n;
}

static float zig_sinf(float x) {                /* sin.zig sinf */
    const double p1 = 1 * 1.57079632679489661923, p2 = 2 * 1.57079632679489661923;
    const double p3 = 3 * 1.57079632679489661923, p4 = 4 * 1.57079632679489661923;
    uint32_t ix = zl_u(x), sign = ix >> 31;
    double y;
    int n;
    ix &= 0x7FFFFFFFu;
    if (ix <= 0x3F490FDAu) {
        if (ix < 0x39800000u) return x;
        return zl_sindf(x);
    }
    if (ix <= 0x407B53D1u) {
        if (ix <= 0x4016CBE3u) return sign ? -zl_cosdf(x + p1) : zl_cosdf(x - p1);
        return zl_sindf(sign ? -(x + p2) : -(x - p2));
    }
    if (ix <= 0x40E231D5u) {
        if (ix <= 0x40AFEDDFu) return sign ? zl_cosdf(x + p3) : -zl_cosdf(x - p3);
        return zl_sindf(sign ? x + p4 : x - p4);
    }
    if (ix >= 0x7F800000u) return x - x;
    if (ix >= 0x4DC90FDBu) return zl_nan();  /* __rem_pio2_large: outside every scene's range */
    n = zl_rem_pio2f(x, &y);
    switch (n & 3) {
        case 0: return zl_sindf(y);
        case 1: return zl_cosdf(y);
        case 2: return zl_sindf(-y);
        default: return -zl_cosdf(y);
    }
}

static float zig_logf(float x) {                /* log.zig logf */
    const float ln2_hi = 6.9313812256e-01f, ln2_lo = 9.0580006145e-06f;
    const float Lg1 = 0xaaaaaa.0p-24f, Lg2 = 0xccce13.0p-25f, Lg3 = 0x91e9ee.0p-25f, Lg4 = 0xf89e26.0p-26f;
    uint32_t ix = zl_u(x);
    int k = 0;
    float f, s, z, w, t1, t2, R, hfsq, dk;
    if (ix < 0x00800000u || (ix >> 31)) {
        if ((ix << 1) == 0) return -INFINITY;
        if (ix >> 31) return zl_nan();
        k -= 25;
        x *= 0x1.0p25f;
        ix = zl_u(x);
    } else if (ix >= 0x7F800000u) {
        return x;
    } else if (ix == 0x3F800000u) {
        return 0;
    }
    ix += 0x3F800000u - 0x3F3504F3u;
    k += (int)(ix >> 23) - 0x7F;
    ix = (ix & 0x007FFFFFu) + 0x3F3504F3u;
    x = zl_f(ix);
    f = x - 1.0f;
    s = f / (2.0f + f);
    z = s * s;
    w = z * z;
    t1 = w * (Lg2 + w * Lg4);
    t2 = z * (Lg1 + w * Lg3);
    R = t2 + t1;
    hfsq = 0.5f * f * f;
    dk = (float)k;
    return s * (hfsq + R) + dk * ln2_lo - hfsq + f + dk * ln2_hi;
}
#endif
