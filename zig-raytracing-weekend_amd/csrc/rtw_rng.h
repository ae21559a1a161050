// rtw_rng.h -- counter-based RNG replacing std.crypto.random (src/rtweekend.zig:14-27).
//
// The reference draws every random number from Zig's thread-local, OS-seeded
// CSPRNG; it cannot be seeded.  This product keys a SplitMix64 stream by
// (seed, domain, a, b):
//     key  = mix64(mix64(seed + domain * G) ^ (a << 32 | b))
//     draw = mix64(state += G)                    G = 0x9E3779B97F4A7C15
// domain 0 = render samples (a = pixel linear index, b = 0-based sample index),
// 1 = scene generation, 2 = BVH build axes, 3 = Perlin tables (a = table id).
// Every draw is mapped to f32 exactly like Zig's std.Random.float(f32).
// Identical (seed, pixel, sample) -> identical draws on any device, batch or
// shard.  Single-sourced for host (BVH build) and device (render kernel).
#pragma once
#include <stdint.h>
#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#endif

#if defined(__HIPCC__)
#define RTW_HD __host__ __device__ __forceinline__
#else
#define RTW_HD static inline
#endif

#define RTW_GOLDEN 0x9E3779B97F4A7C15ull

RTW_HD uint64_t rtw_mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
}

struct rtw_rng {
    uint64_t s;
};

RTW_HD rtw_rng rtw_rng_stream(uint64_t seed, uint64_t domain, uint32_t a, uint32_t b) {
    rtw_rng r;
    r.s = rtw_mix64(rtw_mix64(seed + domain * RTW_GOLDEN) ^ (((uint64_t)a << 32) | (uint64_t)b));
    return r;
}

RTW_HD uint64_t rtw_rng_next(rtw_rng& r) {
    r.s += RTW_GOLDEN;
#if defined(RTW_ABLATE_RNG) && defined(__HIP_DEVICE_COMPILE__)
    // timing ablation only (wrong numbers): 32-bit multiply-free hash
    uint32_t lo = (uint32_t)r.s, hi = (uint32_t)(r.s >> 32);
    lo ^= lo << 13; lo ^= lo >> 17; lo ^= lo << 5; hi ^= lo; hi ^= hi << 7; hi ^= hi >> 9;
    return ((uint64_t)hi << 32) | lo;
#else
    return rtw_mix64(r.s);
#endif
}

RTW_HD int rtw_clz64(uint64_t x) {
#if defined(__HIP_DEVICE_COMPILE__)
    return x ? __clzll((long long)x) : 64;
#else
    return x ? __builtin_clzll(x) : 64;
#endif
}

RTW_HD int rtw_clz32(uint32_t x) {
#if defined(__HIP_DEVICE_COMPILE__)
    return x ? __clz((int)x) : 32;
#else
    return x ? __builtin_clz(x) : 32;
#endif
}

// Zig std.Random.float(f32): mantissa = low 23 bits, exponent 126 - clz(draw).
RTW_HD float rtw_rng_float(rtw_rng& r) {
    uint64_t x = rtw_rng_next(r);
    int lz = rtw_clz64(x);
    if (lz >= 41) {
        lz = 41 + rtw_clz64(rtw_rng_next(r));
        if (lz == 41 + 64) lz += rtw_clz32((uint32_t)rtw_rng_next(r) | 0x7FFu);
    }
    uint32_t bits = ((uint32_t)(126 - lz) << 23) | (uint32_t)(x & 0x7FFFFFu);
    union { uint32_t u; float f; } cv;
    cv.u = bits;
    return cv.f;
}

// rtweekend.zig:18-20
RTW_HD float rtw_rng_range(rtw_rng& r, float mn, float mx) { return mn + (mx - mn) * rtw_rng_float(r); }

// Render-domain draws (camera jitter, defocus disk, ray time, every scatter draw):
// the path's state takes the same Weyl step, and a 32-bit finalizer (lowbias32,
// C. Wellons' hash-prospector: two 32-bit multiplies instead of SplitMix64's two
// 64-bit ones, a third of the cost per draw on gfx950) mixes hi ^ lo of it into a
// 24-bit uniform in [0, 1): k * 2^-24.  Keys stay mix64 (rtw_rng_stream), so
// paths are independent streams; the scene / BVH / Perlin domains keep
// rtw_rng_float (Zig's float(f32) mapping).
RTW_HD uint32_t rtw_lowbias32(uint32_t x) {
    x ^= x >> 16;
    x *= 0x7feb352du;
    x ^= x >> 15;
    x *= 0x846ca68bu;
    x ^= x >> 16;
    return x;
}
RTW_HD float rtw_path_float(rtw_rng& r) {
    r.s += RTW_GOLDEN;
#if defined(RTW_ABLATE_RNG) && defined(__HIP_DEVICE_COMPILE__)
    // timing ablation only (wrong numbers): multiply-free xorshift finalizer
    uint32_t h = (uint32_t)(r.s >> 32) ^ (uint32_t)r.s;
    h ^= h << 13; h ^= h >> 17; h ^= h << 5;
#else
    const uint32_t h = rtw_lowbias32((uint32_t)(r.s >> 32) ^ (uint32_t)r.s);
#endif
    return (float)(h >> 8) * 5.9604644775390625e-08f;  // exact: (h >> 8) < 2^24
}
RTW_HD float rtw_path_range(rtw_rng& r, float mn, float mx) { return mn + (mx - mn) * rtw_path_float(r); }

// ConstantMedium.hit's one draw (objects.zig:484), keyed instead of sequential so
// it does not depend on the order the BVH visits leaves: a float from the stream
// started at mix64(path_state ^ K * (medium + 1)), path_state = the path's RNG
// state at the traversal.
RTW_HD float rtw_medium_u(uint64_t path_state, uint32_t medium) {
    rtw_rng r;
    r.s = rtw_mix64(path_state ^ (0xD1B54A32D192ED03ull * (uint64_t)(medium + 1)));
    return rtw_rng_float(r);
}
