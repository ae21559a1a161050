// rtw_device.h -- device-side building blocks of the path tracer, shared by
// the megakernels (rtw_kernels.hip) and the wavefront kernels (rtw_wavefront.hip).
//
// The per-pixel sample loop Camera.render -> rayColor -> BVHNode.hit / Aabb.hit ->
// Sphere.hit -> Material.scatter -> Texture.value (src/camera.zig:93-208).
//
// Arithmetic contract: compiled with -ffp-contract=off (Zig's strict float
// mode never fuses), correctly rounded fp32 div/sqrt (hipcc default), fp32
// denormals kept.  Every geometric quantity (ray, t, p, normal, scatter
// direction) is evaluated with the same IEEE-754 operations in the same order
// as the Zig source, so paths are bit-identical to the CPU restatement under
// the same RNG key.  The radiance of a path is accumulated iteratively
// (L += T*e; T *= a) instead of the reference's recursive e0 + a0*(e1 + ...),
// a re-association bounded by max_depth * 2^-24 relative.
#pragma once
#include <hip/hip_runtime.h>

#include <cmath>

#include "../../include/rtw_gpu.h"
#include "rtw_internal.h"
#include "rtw_layout.h"
#include "rtw_libm.h"
#include "rtw_rng.h"

#pragma clang fp contract(off)

#ifndef RTW_STEPS
#define RTW_STEPS 1  // the persistent megakernel's node steps per readiness check (rtw_kernels.hip)
#endif


#if defined(RTW_ABLATE_MATH) && defined(__HIP_DEVICE_COMPILE__)
// timing ablation only (not IEEE): hardware sqrt / reciprocal
#define __builtin_sqrtf(x) __builtin_amdgcn_sqrtf(x)
#define RTW_DIV(a, b) ((a) * __builtin_amdgcn_rcpf(b))
#else
#define RTW_DIV(a, b) ((a) / (b))
#endif

// Every building block below is host + device (RTW_DHD): the CPU backend (rtw_cpu.hip) runs
// the same per-sample path (sample_radiance) as the GPU's v0 kernel.  The hardware estimates
// (v_rcp_f32 / v_sqrt_f32) exist only on the device; on the host they are never consulted --
// a host context has fast_reject = fast_box = 0 and no compact nodes.
#define RTW_DHD __host__ __device__ __forceinline__
#if defined(__HIP_DEVICE_COMPILE__)
#define RTW_RCP_EST(x) __builtin_amdgcn_rcpf(x)
#define RTW_SQRT_EST(x) __builtin_amdgcn_sqrtf(x)
#else
#define RTW_RCP_EST(x) (1.0f / (x))
#define RTW_SQRT_EST(x) __builtin_sqrtf(x)
#endif

namespace {

constexpr float kPi = 3.1415926535897932385f;  // rtweekend.zig:4
constexpr float kInf = __builtin_inff();

struct f3 {
    float x, y, z;
};
RTW_DHD f3 mk(float x, float y, float z) { return f3{x, y, z}; }
RTW_DHD f3 operator+(f3 a, f3 b) { return f3{a.x + b.x, a.y + b.y, a.z + b.z}; }
RTW_DHD f3 operator-(f3 a, f3 b) { return f3{a.x - b.x, a.y - b.y, a.z - b.z}; }
RTW_DHD f3 operator*(f3 a, f3 b) { return f3{a.x * b.x, a.y * b.y, a.z * b.z}; }
RTW_DHD f3 operator-(f3 a) { return f3{-a.x, -a.y, -a.z}; }
RTW_DHD f3 splat(float s) { return f3{s, s, s}; }
RTW_DHD float rcp_refined(float d, float y0);
RTW_DHD float div_shared(float x, float d, float y);
RTW_DHD float sqrt_refined(float x, float s);
#if defined(RTW_ABLATE_SHADE_MATH) && defined(__HIP_DEVICE_COMPILE__)
// timing ablation only (not IEEE): hardware reciprocal / sqrt in divs and unit_vector (shading), the walk unchanged
RTW_DHD f3 divs(f3 a, float s) {
    const float y = __builtin_amdgcn_rcpf(s);
    return f3{a.x * y, a.y * y, a.z * y};
}
RTW_DHD float unit_len(float ls) { return __builtin_amdgcn_sqrtf(ls); }
#else
// a / s per component, correctly rounded.  Device: one refined reciprocal of s shared by three div_shared
// (the compiler's IEEE division sequence without its range scaling and special-case fix-up, below) when s
// and every component lie in [2^-40, 2^40] in magnitude -- unscaled operands, normal quotients, no zero
// (whose sign div_shared would not keep) and no inf / NaN, checked on the magnitude bits; otherwise, and on
// the host, IEEE division.  (Hit normals (p - center) / radius, unit vectors.)
RTW_DHD f3 divs(f3 a, float s) {
#if defined(__HIP_DEVICE_COMPILE__) && !defined(RTW_ABLATE_MATH)
    const uint32_t ax = __builtin_bit_cast(uint32_t, a.x) & 0x7FFFFFFFu, ay = __builtin_bit_cast(uint32_t, a.y) & 0x7FFFFFFFu,
                   az = __builtin_bit_cast(uint32_t, a.z) & 0x7FFFFFFFu, as = __builtin_bit_cast(uint32_t, s) & 0x7FFFFFFFu;
    const uint32_t mx = __builtin_elementwise_max(__builtin_elementwise_max(ax, ay), __builtin_elementwise_max(az, as)),
                   mn = __builtin_elementwise_min(__builtin_elementwise_min(ax, ay), __builtin_elementwise_min(az, as));
    if (mn >= 0x2B800000u && mx <= 0x53800000u) {  // 2^-40, 2^40
        const float y = rcp_refined(s, RTW_RCP_EST(s));
        return f3{div_shared(a.x, s, y), div_shared(a.y, s, y), div_shared(a.z, s, y)};
    }
#endif
    return f3{RTW_DIV(a.x, s), RTW_DIV(a.y, s), RTW_DIV(a.z, s)};
}
// sqrt(lengthSquared) of unit_vector, correctly rounded: sqrt_refined on [2^-96, 2^128) on the device
RTW_DHD float unit_len(float ls) {
#if defined(__HIP_DEVICE_COMPILE__) && !defined(RTW_ABLATE_MATH)
    if (ls >= 0x1p-96f && ls <= 0x1.fffffep127f) return sqrt_refined(ls, RTW_SQRT_EST(ls));
#endif
    return __builtin_sqrtf(ls);
}
#endif
RTW_DHD float dot(f3 u, f3 v) { return u.x * v.x + u.y * v.y + u.z * v.z; }
RTW_DHD f3 cross(f3 u, f3 v) {  // vec3.zig:31-33
    return f3{u.y * v.z - u.z * v.y, u.z * v.x - u.x * v.z, u.x * v.y - u.y * v.x};
}
RTW_DHD float length_squared(f3 u) { return u.x * u.x + u.y * u.y + u.z * u.z; }
RTW_DHD f3 unit_vector(f3 v) { return divs(v, unit_len(length_squared(v))); }
RTW_DHD f3 ld3(const float* p) { return f3{p[0], p[1], p[2]}; }
RTW_DHD bool near_zero(f3 u) {  // vec3.zig:19-22
    const float s = 1e-8f;
    return __builtin_fabsf(u.x) < s && __builtin_fabsf(u.y) < s && __builtin_fabsf(u.z) < s;
}
RTW_DHD f3 reflect(f3 v, f3 n) { return v - n * splat(dot(v, n) * 2); }  // vec3.zig:77-79
RTW_DHD f3 refract(f3 uv, f3 n, float e) {                             // vec3.zig:81-86
    float c = dot(-uv, n);
    float cos_theta = c < 1.0f ? c : 1.0f;
    f3 perp = splat(e) * (uv + n * splat(cos_theta));
    f3 par = n * splat(-__builtin_sqrtf(__builtin_fabsf(1.0f - length_squared(perp))));
    return perp + par;
}
RTW_DHD uint32_t fbits(float f) { return __builtin_bit_cast(uint32_t, f); }
RTW_DHD float ubits(uint32_t u) { return __builtin_bit_cast(float, u); }

// ---- RNG helpers (rtweekend.zig / vec3.zig samplers) ----
RTW_DHD float rnd(rtw_rng& r) { return rtw_path_float(r); }  // render-domain draw
RTW_DHD f3 random_unit_vector(rtw_rng& r) {  // vec3.zig:59-68
#if defined(RTW_ABLATE_REJECT)
    {   // timing ablation only: one candidate, no rejection loop (wrong distribution)
        float x = rtw_path_range(r, -1, 1), y = rtw_path_range(r, -1, 1), z = rtw_path_range(r, -1, 1);
        return unit_vector(mk(x, y, z + 1e-3f));
    }
#endif
    for (;;) {
        float x = rtw_path_range(r, -1, 1);
        float y = rtw_path_range(r, -1, 1);
        float z = rtw_path_range(r, -1, 1);
        f3 p = mk(x, y, z);
        if (length_squared(p) < 1) return unit_vector(p);
    }
}

// Zig std.math.pow(f32, x, 5) via frexp-significand square-and-multiply +
// scalbn (restated; identical fp32 operations to the CPU restatement).
RTW_DHD float scalbn_f(float x, int n) {
    float y = x;
    if (n > 127) {
        y *= 1.7014118346046923e38f; n -= 127;
        if (n > 127) { y *= 1.7014118346046923e38f; n -= 127; if (n > 127) n = 127; }
    } else if (n < -126) {
        y *= 1.1754943508222875e-38f * 16777216.0f; n += 126 - 24;
        if (n < -126) { y *= 1.1754943508222875e-38f * 16777216.0f; n += 126 - 24; if (n < -126) n = -126; }
    }
    return y * ubits((uint32_t)(0x7f + n) << 23);
}
RTW_DHD float frexp_sig(float x, int* e) {
    uint32_t u = fbits(x);
    int ee = (int)((u >> 23) & 0xFF);
    int extra = 0;
    if (ee == 0) {
        if (x == 0) { *e = 0; return x; }
        x = x * 18446744073709551616.0f;
        u = fbits(x);
        ee = (int)((u >> 23) & 0xFF);
        extra = -64;
    }
    *e = ee - 126 + extra;
    return ubits((u & 0x807FFFFFu) | 0x3F000000u);
}
RTW_DHD float pow5(float x) {
    if (x == 1) return 1;
    if (x == 0) return x;  // pow(+-0, odd int > 0) = +-0
    if (!(x == x)) return x;
    int xe;
    float x1 = frexp_sig(x, &xe);
    float a1 = 1.0f;
    int ae = 0;
    // i = 5 = 0b101
    a1 *= x1; ae += xe;
    x1 *= x1; xe <<= 1; if (x1 < 0.5f) { x1 += x1; xe -= 1; }
    x1 *= x1; xe <<= 1; if (x1 < 0.5f) { x1 += x1; xe -= 1; }
    a1 *= x1; ae += xe;
    return scalbn_f(a1, ae);
}
RTW_DHD float reflectance(float cosine, float ref_idx) {  // material.zig:101-106
    float r0 = (1 - ref_idx) / (1 + ref_idx);
    r0 = r0 * r0;
    return r0 + (1 - r0) * pow5(1 - cosine);
}

struct Ray {
    f3 o, d;
    float time;
};

// Camera.getRay (camera.zig:156-180)
RTW_DHD Ray get_ray(const rtw_launch& L, uint32_t i, uint32_t j, rtw_rng& rng) {
    const f3 du = ld3(L.du), dv = ld3(L.dv);
    f3 pixel_center = (ld3(L.pixel00) + du * splat((float)i)) + dv * splat((float)j);
    float px = -0.5f + rnd(rng);
    float py = -0.5f + rnd(rng);
    f3 pixel_sample = pixel_center + (splat(px) * du + splat(py) * dv);
    f3 origin;
    if (L.defocus_angle <= 0) {
        origin = ld3(L.center);
    } else {
        float dx, dy;
        for (;;) {  // vec3.randomInUnitDisk (vec3.zig:40-45)
            dx = rtw_path_range(rng, -1, 1);
            dy = rtw_path_range(rng, -1, 1);
            if (dx * dx + dy * dy + 0.0f * 0.0f < 1) break;
        }
        origin = (ld3(L.center) + ld3(L.disk_u) * splat(dx)) + ld3(L.disk_v) * splat(dy);
    }
    Ray r;
    r.o = origin;
    r.d = pixel_sample - origin;
    r.time = rnd(rng);
    return r;
}

// Texture.value (textures.zig:22-123)
__host__ __device__ float perlin_noise(const float4* tab, f3 p) {  // perlin.zig:117-162 + perlin_interp 30-53
    const uint32_t* perm = reinterpret_cast<const uint32_t*>(tab + 256);
    float u = p.x - __builtin_floorf(p.x);
    float v = p.y - __builtin_floorf(p.y);
    float w = p.z - __builtin_floorf(p.z);
    int i = (int)__builtin_floorf(p.x);
    int j = (int)__builtin_floorf(p.y);
    int k = (int)__builtin_floorf(p.z);
    float uu = u * u * (3 - 2 * u);
    float vv = v * v * (3 - 2 * v);
    float ww = w * w * (3 - 2 * w);
    // perlin_interp's weights i*uu + (1-i)*(1-uu) for i in {0, 1}: with uu, vv, ww finite in
    // [0, 1] (u in [0, 1)), 0*uu = +0 and 1*x = x exactly, and +0 + x = x for x >= 0, so the
    // weight IS (1 - uu) for i = 0 and uu for i = 1, bit for bit: the folded form below does
    // the same rounded operations as perlin.zig:42-50 without the multiplications by 0 and 1
    // the compiler must keep (it cannot assume uu finite).
    const float wx[2] = {1 - uu, uu}, wy[2] = {1 - vv, vv}, wz[2] = {1 - ww, ww};
    const uint32_t px[2] = {perm[i & 255], perm[(i + 1) & 255]};
    const uint32_t py[2] = {perm[256 + (j & 255)], perm[256 + ((j + 1) & 255)]};
    const uint32_t pz[2] = {perm[512 + (k & 255)], perm[512 + ((k + 1) & 255)]};
    float accum = 0;
#pragma unroll
    for (int di = 0; di < 2; di++)
#pragma unroll
        for (int dj = 0; dj < 2; dj++)
#pragma unroll
            for (int dk = 0; dk < 2; dk++) {
                const uint32_t idx = px[di] ^ py[dj] ^ pz[dk];
                const float4 c = tab[idx & 255];
                // (u - i, v - j, w - k): u - 0 = u exactly
                const f3 wv = mk(di ? u - 1.0f : u, dj ? v - 1.0f : v, dk ? w - 1.0f : w);
                accum += wx[di] * wy[dj] * wz[dk] * dot(mk(c.x, c.y, c.z), wv);
            }
    return accum;
}

RTW_DHD void sphere_uv(f3 p, float& u, float& v) {  // objects.zig:101-114
    float theta = rtw_acosf(-p.y);  // std.math.acos / atan2 as Zig computes them (rtw_libm.h)
    float phi = rtw_atan2f(-p.z, p.x) + kPi;
    u = phi / (2 * kPi);
    v = theta / kPi;
}

// (u, v) of a hit: sphere hits derive it from the outward normal (getSphereUV,
// objects.zig:101-114, only when an image texture needs it); quads / instance
// members / media carry it explicitly.
struct HitUV {
    f3 outward;
    float u, v;
    bool set;
};

template <uint32_t FEAT>
__host__ __device__ f3 texture_value(const rtw_launch& L, uint32_t ti, const HitUV& uv, f3 p) {
    const rtw_dev_texture& t = L.texs[ti];
    const uint32_t kind = t.kind;
    if constexpr ((FEAT & RTW_F_CHECKER) != 0) {
        if (kind == RTW_TEX_CHECKER) {  // textures.zig:60-72
            int xi = (int)__builtin_floorf(t.scale * p.x);
            int yi = (int)__builtin_floorf(t.scale * p.y);
            int zi = (int)__builtin_floorf(t.scale * p.z);
            return ((xi + yi + zi) % 2 == 0) ? ld3(t.even) : ld3(t.odd);
        }
    }
    if constexpr ((FEAT & RTW_F_IMAGE) != 0) {
        if (kind == RTW_TEX_IMAGE) {  // textures.zig:85-104, rtw_image.zig:37-62
            const rtw_dev_image im = L.img_info[t.image];
            if (im.height <= 0) return mk(0, 1, 1);
            float u = uv.u, v = uv.v;
            if (!uv.set) sphere_uv(uv.outward, u, v);
            float nu = u < 0 ? 0 : (u > 1 ? 1 : u);
            float nv = 1.0f - (v < 0 ? 0 : (v > 1 ? 1 : v));
            uint32_t i = (uint32_t)__builtin_floorf(nu * (float)im.width);
            uint32_t j = (uint32_t)__builtin_floorf(nv * (float)im.height);
            uint32_t x = i < im.width ? i : im.width - 1;
            uint32_t y = j < im.height ? j : im.height - 1;
            const uchar4 px =
                *reinterpret_cast<const uchar4*>(L.images + im.offset + (uint64_t)y * im.bytes_per_row + 4ull * x);
            const float cs = 1.0f / 255.0f;
            return mk(cs * (float)px.x, cs * (float)px.y, cs * (float)px.z);
        }
    }
    if constexpr ((FEAT & RTW_F_NOISE) != 0) {
        if (kind == RTW_TEX_NOISE) {  // textures.zig:118-123, perlin.zig:103-115
            const float4* tab = L.perlin + (size_t)t.perlin * (RTW_PERLIN_BYTES / 16);
            f3 s = splat(t.scale) * p;
            float accum = 0, weight = 1.0f;
            f3 tp = s;
            for (int k = 0; k < 7; k++) {
                accum += weight * perlin_noise(tab, tp);
                weight *= 0.5f;
                tp = tp * splat(2);
            }
            float turb = __builtin_fabsf(accum);
            return splat(0.5f * (1 + rtw_sinf(s.z + 10 * turb)));  // @sin: rtw_libm.h
        }
    }
    return ld3(t.even);  // RTW_TEX_SOLID (textures.zig:43-45)
}

// Correctly rounded fp32 division and square root on operands known to be in range:
// the exact instruction sequences of the compiler's IEEE expansions with their
// range scaling and special-value fix-ups left out.  With v_div_scale leaving its
// operands unscaled (numerator and denominator normal, |exponent difference| < 96,
// quotient and 1/d normal) and v_div_fixup passing the quotient through, x / d is
//   y0 = rcp(d); e = fma(-d, y0, 1); y = fma(e, y0, y0)           (rcp_refined)
//   q0 = x * y; r0 = fma(-d, q0, x); q1 = fma(r0, y, q0);
//   r1 = fma(-d, q1, x); q = fma(r1, y, q1)                        (div_shared)
// so several divisions by one d (a ray's |d|^2, a sphere radius, a vector length)
// share y.  sqrt_refined: for x in [2^-96, 2^128) finite, the compiler's IEEE sqrt
// is v_sqrt_f32 then a +-1 ulp correction by the signs of fma residuals.
RTW_DHD float rcp_refined(float d, float y0) {
    const float e = __builtin_fmaf(-d, y0, 1.0f);
    return __builtin_fmaf(e, y0, y0);
}
RTW_DHD float div_shared(float x, float d, float y) {
    const float q0 = x * y;
    const float r0 = __builtin_fmaf(-d, q0, x);
    const float q1 = __builtin_fmaf(r0, y, q0);
    const float r1 = __builtin_fmaf(-d, q1, x);
    return __builtin_fmaf(r1, y, q1);
}
RTW_DHD float sqrt_refined(float x, float s /* v_sqrt_f32(x) */) {
    const float sdn = ubits(fbits(s) - 1u), sup = ubits(fbits(s) + 1u);
    const float rdn = __builtin_fmaf(-sdn, s, x), rup = __builtin_fmaf(-sup, s, x);
    const float r = (rdn <= 0.0f) ? sdn : s;
    return (rup > 0.0f) ? sup : r;
}

struct Counters {
    uint32_t rays = 0, nodes = 0, leaves = 0, nans = 0, tail_rays = 0;
#if defined(RTW_DIAG_WALK)
    uint32_t dsteps = 0, dleaves = 0;  // diagnostic build: steps / sphere tests of this lane's last compact walk
#endif
};

#if defined(RTW_DIAG_WALK) && defined(__HIP_DEVICE_COMPILE__)
// Diagnostic build only (make diag -> build/rtw_diag.so; tools/diag_walk.py): how the wave steps of the
// compact walk split into box / sphere-test / exact-root work.  w*: wave steps (counted once per wave by
// the lowest active lane), l*: lane steps.  Summed per launch into rtw_diag_walk (rtw_wavefront.hip).
struct WalkDiag {
    uint32_t wsteps = 0, wleaf = 0, wexact = 0, lsteps = 0, lleaf = 0, lexact = 0, lexact_hit = 0, walks = 0;
};
#define RTW_DG_PARAM , WalkDiag* dg = nullptr
#define RTW_DG_ARG(x) , x
__device__ __forceinline__ bool dg_leader() { return __lane_id() == (uint32_t)__builtin_ctzll(__ballot(1)); }
#else
#define RTW_DG_PARAM
#define RTW_DG_ARG(x)
#endif

// Per-ray constants of the traversal.
struct RayTrav {
    f3 inv;      // 1 / d per axis (aabb.zig:87); fast box: clamped hardware reciprocal
    f3 oinv;     // fast box only: -o * inv
    float a;     // lengthSquared(d) (objects.zig:124)
    float rcp_a; // hardware 1/a estimate for the sphere fast-reject (0 disables it)
    float ya;    // rcp_refined(a) for div_shared (0: a outside [2^-40, 2^40], IEEE division)
    float tk;    // a * tmin (sphere_may_hit)
    float ktk;   // 2^-20 * tk
    float gk;    // 1 - 2^-20 where the sphere filter applies (a in [2^-40, 2^40]), else 0
    float nk;    // -2^-20 in a VGPR: as an SGPR operand (gfx9 VOP3 has no literal) its FMAs would take 4
                 // clocks instead of dual-issuing at 2 (profiles/r4_valu_peak/)
};
RTW_DHD RayTrav ray_trav(const Ray& r, bool fast_box) {
    RayTrav t;
    if (fast_box) {
        // |inv| <= 1e30 keeps every product finite (no inf*0 / inf-inf); a zero
        // component gives slabs of +-1e30 * (P - o), i.e. still +-"infinite"
        // given the >= E*2^-19 box pad
        auto ci = [](float d) {
            return __builtin_fmaxf(__builtin_fminf(RTW_RCP_EST(d), 1e30f), -1e30f);
        };
        t.inv = mk(ci(r.d.x), ci(r.d.y), ci(r.d.z));
        t.oinv = mk(-(r.o.x * t.inv.x), -(r.o.y * t.inv.y), -(r.o.z * t.inv.z));
    } else {
        t.inv = mk(RTW_DIV(1.0f, r.d.x), RTW_DIV(1.0f, r.d.y), RTW_DIV(1.0f, r.d.z));
        t.oinv = mk(0, 0, 0);
    }
    t.a = length_squared(r.d);
    // fast-reject only where every intermediate below stays normal and finite
    t.rcp_a = (t.a > 1e-30f && t.a < 1e30f) ? RTW_RCP_EST(t.a) : 0.0f;
    t.ya = (t.a >= 0x1p-40f && t.a <= 0x1p40f) ? rcp_refined(t.a, t.rcp_a) : 0.0f;
    t.tk = t.a * 0.001f;  // kTmin (camera.zig:187)
    t.ktk = t.tk * 9.5367432e-07f;
    t.gk = (t.a >= 0x1p-40f && t.a <= 0x1p40f) ? 0.99999905f : 0.0f;  // 1 - 2^-20
    t.nk = -9.5367432e-07f;
#if defined(__HIP_DEVICE_COMPILE__)
    asm volatile("" : "+v"(t.nk));  // keep it a per-lane register
#endif
    return t;
}

constexpr float kTmin = 0.001f;  // camera.zig:187

// The sphere fast-reject of sphere_leaf (derivation there and in DESIGN.md §4): false only if no root of
// Sphere.hit's exact IEEE arithmetic (objects.zig:127-136) can lie in (tmin, closest).  tk = fl(a * tmin),
// ktk = 2^-20 * tk, gk = 1 - 2^-20 (0: no filtering, every disc >= 0 passes).  Host and device run the same
// fp32 operations (FMAs are correctly rounded on both), so tests/test_filter.py checks it on the host.
// nk = -2^-20 (RayTrav::nk: a VGPR on the device).
RTW_DHD bool sphere_may_hit(float hb, float disc, float a, float closest, float tk, float ktk, float gk,
                            float nk = -9.5367432e-07f) {
    const float xb = hb + tk;                                // X = hb + a tmin
    const float yb = __builtin_fmaf(-a, closest, -hb);       // Y = -hb - a closest (one rounding; -inf for inf)
    const float lx = __builtin_fmaf(nk, __builtin_fabsf(xb), xb - ktk);
    const float ly = __builtin_fmaf(nk, __builtin_fabsf(yb), __builtin_fmaf(nk, __builtin_fabsf(hb), yb));
    const float b = __builtin_fmaxf(__builtin_fmaxf(lx, ly) * gk, 0.0f);  // maxNum: a NaN bound becomes 0
    return disc >= b * b;
}

// ---------------------------------------------------------------------------
// Non-sphere world objects (scenes with RTW_F_GEOM / RTW_F_MEDIUM): quads,
// Translate/RotateY instances of a HittableList, ConstantMedium.  Same fp32
// operations in the same order as objects.zig (and the CPU restatement).
// ---------------------------------------------------------------------------
RTW_DHD float4 ldg4(const float* p) { return *reinterpret_cast<const float4*>(p); }

// Sphere.hit t only (objects.zig:116-136), open interval (tmin, tmax)
RTW_DHD bool sphere_t(f3 center, float radius, const Ray& r, float tmin, float tmax, float& t) {
    const f3 oc = r.o - center;
    const float a = length_squared(r.d);
    const float half_b = dot(oc, r.d);
    const float c = length_squared(oc) - radius * radius;
    const float disc = half_b * half_b - a * c;
    if (disc < 0) return false;
    const float sq = __builtin_sqrtf(disc);
    float root = RTW_DIV(-half_b - sq, a);
    if (!(tmin < root && root < tmax)) {
        root = RTW_DIV(-half_b + sq, a);
        if (!(tmin < root && root < tmax)) return false;
    }
    t = root;
    return true;
}

template <uint32_t FEAT>
RTW_DHD f3 member_sphere_center(const rtw_launch& L, const rtw_dev_sphere& s, uint32_t idx,
                                                   float time) {
    f3 c = ld3(s.c1);
    if constexpr ((FEAT & RTW_F_MOVING) != 0) {
        if (s.moving) {  // Sphere.getCenter (objects.zig:94-98)
            const float4 cv = L.cvec[idx];
            c = c + splat(time) * mk(cv.x, cv.y, cv.z);
        }
    }
    return c;
}

// Quad.hit t only (objects.zig:222-255), closed interval [tmin, tmax]
#if defined(RTW_ABLATE_QUAD2) && defined(__HIP_DEVICE_COMPILE__)
RTW_DHD bool quad_t_once(const rtw_dev_quad& q, const Ray& r, float tmin, float tmax, float& t);
RTW_DHD bool quad_t(const rtw_dev_quad& q, const Ray& r, float tmin, float tmax, float& t) {
    // timing ablation only: every quad test twice (the second is the same test)
    float tm = tmax, t2 = 0.0f;
    asm volatile("" : "+v"(tm));
    const bool h2 = quad_t_once(q, r, tmin, tm, t2);
    const bool h = quad_t_once(q, r, tmin, tmax, t);
    if (h2 != h) t = t2;
    return h;
}
RTW_DHD bool quad_t_once(const rtw_dev_quad& q, const Ray& r, float tmin, float tmax, float& t) {
#else
RTW_DHD bool quad_t(const rtw_dev_quad& q, const Ray& r, float tmin, float tmax, float& t) {
#endif
    const f3 n = ld3(q.n);
    const float denom = dot(n, r.d);
    if (__builtin_fabsf(denom) < 1e-8f) return false;
    const float tt = RTW_DIV(q.d - dot(n, r.o), denom);
    if (!(tmin <= tt && tt <= tmax)) return false;
    const f3 planar = (r.o + splat(tt) * r.d) - ld3(q.q);
    const f3 w = ld3(q.w);
    const float alpha = dot(w, cross(planar, ld3(q.v)));
    const float beta = dot(w, cross(ld3(q.u), planar));
    if ((alpha < 0) || (1 < alpha) || (beta < 0) || (1 < beta)) return false;
    t = tt;
    return true;
}

// world ray -> object space of an instance: the outermost transform first
// (Translate.hit objects.zig:314-317, RotateY.hit :401-411)
RTW_DHD Ray inst_to_object(const rtw_dev_instance* __restrict__ in, Ray r) {
    for (int k = (int)in->n_xf - 1; k >= 0; k--) {
        const float4 x = ldg4(in->xf[k]);
        if (fbits(x.x) == RTW_XF_TRANSLATE) {
            r.o = r.o - mk(x.y, x.z, x.w);
        } else {
            const float s = x.y, c = x.z;
            const f3 o = r.o, d = r.d;
            r.o.x = c * o.x - s * o.z;
            r.o.z = s * o.x + c * o.z;
            r.d.x = c * d.x - s * d.z;
            r.d.z = s * d.x + c * d.z;
        }
    }
    return r;
}

// object-space point/normal -> world: innermost transform first (RotateY.hit :419-435, Translate.hit :325-326)
RTW_DHD void inst_to_world(const rtw_dev_instance* __restrict__ in, f3& p, f3& n) {
    for (uint32_t k = 0; k < in->n_xf; k++) {
        const float4 x = ldg4(in->xf[k]);
        if (fbits(x.x) == RTW_XF_TRANSLATE) {
            p = p + mk(x.y, x.z, x.w);
        } else {
            const float s = x.y, c = x.z;
            const f3 p0 = p, n0 = n;
            p.x = c * p0.x + s * p0.z;
            p.z = -s * p0.x + c * p0.z;
            n.x = c * n0.x + s * n0.z;
            n.z = -s * n0.x + c * n0.z;
        }
    }
}

// HittableList.hit over the members in object space (objects.zig:281-289)
template <uint32_t FEAT>
RTW_DHD bool list_t(const rtw_launch& L, const rtw_dev_instance* __restrict__ in, const Ray& ro,
                                       float tmin, float tmax, float& t, uint32_t& sub) {
    bool any = false;
    float closest = tmax;
    const uint32_t first = in->first, count = in->count;
    for (uint32_t m = 0; m < count; m++) {
        const uint32_t ref = L.members[first + m];
        const uint32_t idx = RTW_REF_INDEX(ref);
        float tt;
        bool h;
        if (RTW_REF_KIND(ref) == RTW_OBJ_SPHERE) {
            const rtw_dev_sphere s = L.sph[idx];
            h = sphere_t(member_sphere_center<FEAT>(L, s, idx, ro.time), s.radius, ro, tmin, closest, tt);
        } else {
            h = quad_t(L.quads[idx], ro, tmin, closest, tt);
        }
        if (h) {
            closest = tt;
            sub = m;
            any = true;
        }
    }
    t = closest;
    return any;
}

// Hittable.hit of a sphere / quad / instance reference (a medium boundary)
template <uint32_t FEAT>
RTW_DHD bool boundary_t(const rtw_launch& L, uint32_t ref, const Ray& r, float tmin, float tmax,
                                           float& t) {
    const uint32_t idx = RTW_REF_INDEX(ref);
    switch (RTW_REF_KIND(ref)) {
    case RTW_OBJ_SPHERE: {
        const rtw_dev_sphere s = L.sph[idx];
        return sphere_t(member_sphere_center<FEAT>(L, s, idx, r.time), s.radius, r, tmin, tmax, t);
    }
    case RTW_OBJ_QUAD: return quad_t(L.quads[idx], r, tmin, tmax, t);
    default: {
        const rtw_dev_instance* in = L.insts + idx;
        uint32_t sub;
        return list_t<FEAT>(L, in, inst_to_object(in, r), tmin, tmax, t, sub);
    }
    }
}

// ConstantMedium.hit (objects.zig:470-507); the draw is keyed by (mkey, medium)
template <uint32_t FEAT>
RTW_DHD bool medium_t(const rtw_launch& L, uint32_t idx, const Ray& r, float tmin, float tmax,
                                         uint64_t mkey, float& t) {
    const rtw_dev_medium m = L.media[idx];
    float t1, t2;
    if (RTW_REF_KIND(m.boundary) == RTW_OBJ_INSTANCE) {
        // both boundary queries see the same object-space ray: transform it once
        const rtw_dev_instance* in = L.insts + RTW_REF_INDEX(m.boundary);
        const Ray ro = inst_to_object(in, r);
        uint32_t sub;
        if (!list_t<FEAT>(L, in, ro, -kInf, kInf, t1, sub)) return false;  // intervals.universe
        if (!list_t<FEAT>(L, in, ro, t1 + 0.0001f, kInf, t2, sub)) return false;
    } else {
        if (!boundary_t<FEAT>(L, m.boundary, r, -kInf, kInf, t1)) return false;  // intervals.universe
        if (!boundary_t<FEAT>(L, m.boundary, r, t1 + 0.0001f, kInf, t2)) return false;
    }
    if (t1 < tmin) t1 = tmin;
    if (t2 > tmax) t2 = tmax;
    if (t1 >= t2) return false;
    if (t1 < 0) t1 = 0;
    const float ray_length = __builtin_sqrtf(length_squared(r.d));
    const float inside = (t2 - t1) * ray_length;
    const float hit_distance = m.neg_inv_density * rtw_logf(rtw_medium_u(mkey, idx));  // @log: rtw_libm.h
    if (hit_distance > inside) return false;
    t = t1 + RTW_DIV(hit_distance, ray_length);
    return true;
}

// The padded world box of an instance (rtw_build_bvh) met by the ray on [0.001, closest]: the fast slab
// test of box_next.  Every hit the instance's leaf (or a medium bounded by it) can accept lies in the box,
// so a miss skips the transforms and member tests with the same result.  Within a leaf the walk stays in
// step across the wave; the member loop runs when any lane meets the box.  (As a walk node of its own the
// same box cost Cornell 4.6 %: lanes that skipped it walked out of step with the others)
RTW_DHD bool inst_box_met(const rtw_launch& L, const rtw_dev_instance* __restrict__ in, const RayTrav& rt,
                                         float closest) {
    if (!(L.fast_box && L.inst_cull)) return true;
    const float4 A = ldg4(in->box[0]), B = ldg4(in->box[1]);
    const float t0x = __builtin_fmaf(A.x, rt.inv.x, rt.oinv.x), t1x = __builtin_fmaf(B.x, rt.inv.x, rt.oinv.x);
    const float t0y = __builtin_fmaf(A.y, rt.inv.y, rt.oinv.y), t1y = __builtin_fmaf(B.y, rt.inv.y, rt.oinv.y);
    const float t0z = __builtin_fmaf(A.z, rt.inv.z, rt.oinv.z), t1z = __builtin_fmaf(B.z, rt.inv.z, rt.oinv.z);
    const float lo = __builtin_fmaxf(__builtin_fmaxf(kTmin, __builtin_fminf(t0x, t1x)),
                                     __builtin_fmaxf(__builtin_fminf(t0y, t1y), __builtin_fminf(t0z, t1z)));
    const float hi = __builtin_fminf(__builtin_fminf(closest, __builtin_fmaxf(t0x, t1x)),
                                     __builtin_fminf(__builtin_fmaxf(t0y, t1y), __builtin_fmaxf(t0z, t1z)));
    return !(hi <= lo);
}

// A non-sphere leaf tested with (0.001, closest): updates closest / hit
// (hit = node | member << 24 for an instance's list member)
template <uint32_t FEAT>
RTW_DHD void object_leaf(const rtw_launch& L, const Ray& r, const RayTrav& rt, uint32_t kind, uint32_t idx,
                                         uint32_t node, float& closest, int& hit, uint64_t mkey) {
    float t;
    uint32_t sub = 0;
    bool h = false;
    if (kind == RTW_OBJ_QUAD) {
        h = quad_t(L.quads[idx], r, kTmin, closest, t);
    } else if (kind == RTW_OBJ_INSTANCE) {
        const rtw_dev_instance* in = L.insts + idx;
        if (inst_box_met(L, in, rt, closest)) h = list_t<FEAT>(L, in, inst_to_object(in, r), kTmin, closest, t, sub);
    } else if constexpr ((FEAT & RTW_F_MEDIUM) != 0) {
        const uint32_t b = L.media[idx].boundary;
        if (RTW_REF_KIND(b) != RTW_OBJ_INSTANCE || inst_box_met(L, L.insts + RTW_REF_INDEX(b), rt, closest))
            h = medium_t<FEAT>(L, idx, r, kTmin, closest, mkey, t);
    }
    if (h) {
        closest = t;
        hit = (int)(node | (sub << RTW_HIT_NODE_BITS));
    }
}

// Node i of the pre-order walk: two 16-B loads issued together (both halves are
// needed on either path; a split load would put a second memory round trip on
// the inner-node path).
RTW_DHD void load_node(const float4* __restrict__ nodes, uint32_t i, float4& A, float4& B) {
    A = nodes[2 * i];
    B = nodes[2 * i + 1];
#if defined(__HIP_DEVICE_COMPILE__)
    asm volatile("" ::"v"(A.x), "v"(A.y), "v"(A.z), "v"(A.w), "v"(B.x), "v"(B.y), "v"(B.z), "v"(B.w));
#endif
}

// Leaf: Sphere.hit (objects.zig:116-136) on the open interval (0.001, closest),
// no box test (bvh.zig:123-125).  Updates closest/hit.
// Sphere.hit (objects.zig:116-136) of a sphere at `center` with rr = radius * radius
// (the reference's product, evaluated by the caller or on the host) on (0.001, closest).
RTW_DHD void sphere_leaf(const rtw_launch& L, const Ray& r, const RayTrav& rt, f3 center, float rr,
                                            uint32_t i, float& closest, int& hit RTW_DG_PARAM) {
#if defined(__HIP_DEVICE_COMPILE__)
    // oc = o - center, dot(oc, d) and lengthSquared(oc) (objects.zig:123-126) with the x and y lanes as
    // packed pairs: the same IEEE operations per component in the same order (x + y first, then + z),
    // and the node's center.xy arrives as an aligned register pair (no moves before v_pk_add_f32)
    typedef float f2v __attribute__((ext_vector_type(2)));
    const f2v oxy = {r.o.x, r.o.y}, cxy = {center.x, center.y}, dxy = {r.d.x, r.d.y};
    const f2v ocxy = oxy - cxy;
    const float ocz = r.o.z - center.z;
    const f2v p = ocxy * dxy, q = ocxy * ocxy;
    const float half_b = (p.x + p.y) + ocz * r.d.z;
    const float c = ((q.x + q.y) + ocz * ocz) - rr;
#else
    const f3 oc = r.o - center;
    const float half_b = dot(oc, r.d);
    const float c = length_squared(oc) - rr;
#endif
    const float disc = half_b * half_b - rt.a * c;
    bool exact = disc >= 0;
#if !defined(RTW_ABLATE_MATH)
    // Exact fast-reject (round 4): no square root, no division.  A root of objects.zig:130-136 lies in
    // (tmin, closest) only if root2 > tmin and root1 < closest (root1 <= root2: a > 0 and the rounded
    // operations are monotone), and with s = sqrt(disc) those hold only if s > max(Lx, Ly) for
    //   Lx = X - 2.03u|X| - 2.04u T,   X = hb + T, T = a * tmin          (root2 > tmin)
    //   Ly = Y - 3.06u|Y| - 1.02u|hb|, Y = -hb - a * closest             (root1 < closest; -inf for inf)
    // (u = 2^-24; the slack covers the reference's roundings of sqrt, the numerators and the divisions,
    // and the roundings of X and Y here).  sphere_may_hit computes lower bounds of both with k = 2^-20 =
    // 16u margins, b = max(them) * (1 - 2^-20) clamped at 0, and accepts iff disc >= fl(b * b): s > b >= 0
    // gives disc = s^2 > fl(b^2), so a ray the exact test would accept is never rejected (derivation in
    // DESIGN.md §4; tests/test_filter.py checks it against the exact test on adversarial inputs).  The
    // bound needs T normal: the ray's guard factor rt.gk is 0 (every disc >= 0 goes exact) unless
    // fast_reject and a in [2^-40, 2^40].  Overflowing squares only reject rays the reference rejects.
    // Measured on gfx950 (profiles/r4_valu_peak/): the old filter's v_sqrt_f32 took 8 clocks per wave and
    // its SGPR compares 4; these adds, FMAs and maxes dual-issue at 2.
    exact = sphere_may_hit(half_b, disc, rt.a, closest, rt.tk, rt.ktk, L.fast_reject ? rt.gk : 0.0f, rt.nk);
#endif
#if defined(RTW_DIAG_WALK) && defined(__HIP_DEVICE_COMPILE__)
    const float closest_in = closest;
    if (dg) {
        const uint64_t m = __ballot(exact);
        if (dg_leader()) {
            dg->wexact += m ? 1u : 0u;
            dg->lexact += (uint32_t)__popcll(m);
        }
    }
#endif
    if (exact) {
        float sq, root, root2;
        bool quick = false;  // the exact roots by sqrt_refined / div_shared (operands in range)
#if !defined(RTW_ABLATE_MATH)
        // |-hb -+ sq| < 2^51 and disc >= 2^-96; with a in [2^-40, 2^40] (ya != 0) the divisions are
        // unscaled except for quotients below 2^-80, which kTmin rejects either way
        quick = L.fast_reject & (rt.ya != 0.0f) & (disc >= 0x1p-96f) & (disc < 1e30f) &
                (__builtin_fabsf(half_b) < 1e15f);
#endif
        if (quick) {
            sq = sqrt_refined(disc, RTW_SQRT_EST(disc));
            root = div_shared(-half_b - sq, rt.a, rt.ya);
            root2 = div_shared(-half_b + sq, rt.a, rt.ya);
        } else {
            sq = __builtin_sqrtf(disc);
            root = RTW_DIV(-half_b - sq, rt.a);
            root2 = RTW_DIV(-half_b + sq, rt.a);
        }
        bool ok = kTmin < root && root < closest;
        if (!ok) {
            root = root2;
            ok = kTmin < root && root < closest;
        }
        if (ok) {
            closest = root;
            hit = (int)i;
        }
    }
#if defined(RTW_DIAG_WALK) && defined(__HIP_DEVICE_COMPILE__)
    if (dg && closest != closest_in) dg->lexact_hit++;
#endif
}

template <uint32_t FEAT>
RTW_DHD void leaf_test(const rtw_launch& L, const Ray& r, const RayTrav& rt, float4 A, float4 B,
                                          uint32_t i, float& closest, int& hit, Counters& cnt, uint64_t mkey = 0) {
    cnt.leaves++;
    if constexpr ((FEAT & RTW_F_GEOM) != 0) {
        const uint32_t kind = RTW_LEAF_KIND(fbits(B.w));
        if (kind != RTW_OBJ_SPHERE) {
            object_leaf<FEAT>(L, r, rt, kind, fbits(B.z), i, closest, hit, mkey);
            return;
        }
    }
    f3 center = mk(A.x, A.y, A.z);
    if constexpr ((FEAT & RTW_F_MOVING) != 0) {
        if (fbits(B.w)) {  // Sphere.getCenter (objects.zig:94-98)
            const float4 cv = L.cvec[fbits(B.z)];
            center = center + splat(r.time) * mk(cv.x, cv.y, cv.z);
        }
    }
    sphere_leaf(L, r, rt, center, B.x * B.x, i, closest, hit);
}

// Inner node: Aabb.hit (aabb.zig:82-114) with [0.001, closest]; returns the next
// node (i + 1 = descend, skip = past the subtree).
//  exact: the reference arithmetic.  hi/lo use fmax/fmin: for the NaN slabs of a
//    zero direction component (0*inf) maxNum keeps the other operand exactly like
//    the reference's `if (t0 > min) min = t0`, and lo/hi only grow/shrink, so the
//    single final `hi <= lo` equals the per-axis early exit of aabb.zig:111.
//  fast (SAH trees): t = fma(P, inv, -o*inv) with min/max instead of swaps, on
//    boxes padded by E*2^-19 -- conservative (never rejects a box the exact test
//    on the unpadded box accepts), so the closest hit is unchanged.
RTW_DHD uint32_t box_next(const Ray& r, const RayTrav& rt, float4 A, float4 B, uint32_t i,
                                             float closest, bool fast) {
    const uint32_t w = fbits(A.w);
    if (fast) {
        const float t0x = __builtin_fmaf(A.x, rt.inv.x, rt.oinv.x), t1x = __builtin_fmaf(B.x, rt.inv.x, rt.oinv.x);
        const float t0y = __builtin_fmaf(A.y, rt.inv.y, rt.oinv.y), t1y = __builtin_fmaf(B.y, rt.inv.y, rt.oinv.y);
        const float t0z = __builtin_fmaf(A.z, rt.inv.z, rt.oinv.z), t1z = __builtin_fmaf(B.z, rt.inv.z, rt.oinv.z);
        const float lo = __builtin_fmaxf(__builtin_fmaxf(kTmin, __builtin_fminf(t0x, t1x)),
                                         __builtin_fmaxf(__builtin_fminf(t0y, t1y), __builtin_fminf(t0z, t1z)));
        const float hi = __builtin_fminf(__builtin_fminf(closest, __builtin_fmaxf(t0x, t1x)),
                                         __builtin_fminf(__builtin_fmaxf(t0y, t1y), __builtin_fmaxf(t0z, t1z)));
        return (hi <= lo) ? w : i + 1;
    }
    float t0x = (A.x - r.o.x) * rt.inv.x, t1x = (B.x - r.o.x) * rt.inv.x;
    float t0y = (A.y - r.o.y) * rt.inv.y, t1y = (B.y - r.o.y) * rt.inv.y;
    float t0z = (A.z - r.o.z) * rt.inv.z, t1z = (B.z - r.o.z) * rt.inv.z;
    if (rt.inv.x < 0) { float tt = t1x; t1x = t0x; t0x = tt; }
    if (rt.inv.y < 0) { float tt = t1y; t1y = t0y; t0y = tt; }
    if (rt.inv.z < 0) { float tt = t1z; t1z = t0z; t0z = tt; }
    const float lo = __builtin_fmaxf(__builtin_fmaxf(kTmin, t0x), __builtin_fmaxf(t0y, t0z));
    const float hi = __builtin_fminf(__builtin_fminf(closest, t1x), __builtin_fminf(t1y, t1z));
    return (hi <= lo) ? w : i + 1;
}

// One node of the stackless pre-order walk of the reference BVH
// (bvh.zig:122-136).  Returns the next node index.
template <uint32_t FEAT>
RTW_DHD uint32_t trav_step(const float4* __restrict__ nodes, const rtw_launch& L, const Ray& r,
                                              const RayTrav& rt, uint32_t i, float& closest, int& hit,
                                              Counters& cnt, uint64_t mkey = 0) {
    float4 A, B;
    load_node(nodes, i, A, B);
    const uint32_t w = fbits(A.w);
    if (w & RTW_LEAF_BIT) {
        leaf_test<FEAT>(L, r, rt, A, B, i, closest, hit, cnt, mkey);
        return w & RTW_SKIP_MASK;
    }
    cnt.nodes++;
    return box_next(r, rt, A, B, i, closest, L.fast_box != 0);
}

// World hit for one ray (whole walk).  Returns leaf node index or -1.
// The node array a ray walks: SAH sphere scenes keep 8 copies, children ordered
// front-to-back for each ray-direction octant (rtw_bvh.hip SahBuilder::build);
// each lane walks its own octant's copy (a per-wave majority octant measured
// slower: more node visits and no gain in coherence).  The copy is recorded in
// the hit id (bits 24..26; such scenes have no instance members there) so
// shading finds the leaf.
// 4 copies (round 5): ordered by the signs of x and z only -- the axes the Book-1 field spreads over
// (the spheres lie within [0, 2] in y) -- so the compact stage is half the size (rtw_compact_nodes); the
// walk then takes y's near/far per ray (traverse_compact<.., Y4>).
RTW_DHD uint32_t order_of(const rtw_launch& L, const Ray& r) {
    if (L.n_orders <= 1) return 0;
    if (L.n_orders == 4) return (r.d.x < 0 ? 1u : 0u) | (r.d.z < 0 ? 2u : 0u);
    return (r.d.x < 0 ? 1u : 0u) | (r.d.y < 0 ? 2u : 0u) | (r.d.z < 0 ? 4u : 0u);
}
// median of three (v_med3_f32 on the device); operands finite (the fast slab test's clamped reciprocals)
RTW_DHD float med3f(float a, float b, float c) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_amdgcn_fmed3f(a, b, c);
#else
    return std::fmax(std::fmin(a, b), std::fmin(std::fmax(a, b), c));
#endif
}
RTW_DHD const float4* order_base(const float4* nodes, const rtw_launch& L, uint32_t oct) {
    return nodes + (size_t)oct * 2u * L.n_nodes;
}
RTW_DHD int hit_with_order(int hit, uint32_t oct) {
    return hit < 0 ? hit : (int)((uint32_t)hit | (oct << RTW_HIT_NODE_BITS));
}

// The walk over the compact 16-B nodes (rtw_bvh.hip rtw_compact_nodes; static
// sphere SAH trees, FMA slab test): one load per step.  Inner boxes are fp16,
// rounded outward, consumed by v_fma_mix_f32 (exact f16->f32, one rounding:
// the same t = fma(P, inv, -o*inv) as box_next's fast test on a superset box);
// leaves carry center and radius^2.  Same visits-superset argument: same hit.
RTW_DHD float h_lo(uint32_t w) { return (float)__builtin_bit_cast(_Float16, (unsigned short)(w & 0xFFFFu)); }
RTW_DHD float h_hi(uint32_t w) { return (float)__builtin_bit_cast(_Float16, (unsigned short)(w >> 16)); }

#if defined(RTW_DIAG_WALK)
// [0..7] the compact walk (WalkDiag); [8] camera-ray list waves, [9] list candidates tested (per wave),
// [10] list waves over the cap (they walk), [11] list candidates tested with the exact path (per wave)
__device__ unsigned long long rtw_diag_walk[16];
#endif
#if defined(RTW_DIAG_WALK) && defined(__HIP_DEVICE_COMPILE__)
// sum the lanes' diag counters (the lanes that walked) and add them to rtw_diag_walk
__device__ __forceinline__ void rtw_diag_flush(const WalkDiag& d) {
    uint32_t v[8] = {d.wsteps, d.wleaf, d.wexact, d.lsteps, d.lleaf, d.lexact, d.lexact_hit, d.walks};
    const uint64_t act = __ballot(1);
    const bool lead = dg_leader();
    for (int k = 0; k < 8; k++) {
        uint32_t x = v[k];
        for (int o = 32; o > 0; o >>= 1) {
            const uint32_t y = __shfl_xor(x, o);
            x += (act >> (__lane_id() ^ o)) & 1ull ? y : 0u;
        }
        if (lead && x) atomicAdd(&rtw_diag_walk[k], (unsigned long long)x);
    }
}
#endif

// `base`: L.cnodes, or their copy in LDS
// The walk steps through BYTE offsets (rtw_compact_nodes stores an inner node's skip target that
// way), with no index -> address multiply per step; a sphere's hit id is its byte offset until the
// walk ends.  LDS: `base` is the LDS stage, whose inner nodes stage_cnodes rebased to absolute LDS
// addresses, so a step's address IS the offset (ds_read_b128 with no add); else the offsets are
// from `base` (global memory).
#if defined(__HIP_DEVICE_COMPILE__)
typedef __attribute__((address_space(3))) const uint4 lds_uint4;
#endif
// the LDS address of a pointer into this block's LDS (device only; the host never walks an LDS stage)
RTW_DHD uint32_t lds_addr(const void* p) {
#if defined(__HIP_DEVICE_COMPILE__)
    return (uint32_t)(uintptr_t)(__attribute__((address_space(3))) const void*)p;
#else
    (void)p;
    return 0;
#endif
}
// Y4: the 4-copy layout (L.n_orders == 4; rtw_compact_nodes): x and z stored (near, far) for the copy's
// signs, y as (min, max) in the near-y / far-y slots.  With ta, tb the two y slab distances, lo = max(X, min(ta,
// tb)) and hi = min(Y, max(ta, tb)) (X = max(tmin, tnx, tnz), Y = min(closest, tfx, tfz)); the walk uses
// lo' = med3(X, ta, tb) = min(lo, max(ta, tb)) and hi' = med3(Y, ta, tb) = max(hi, min(ta, tb)), and lo' < hi'
// exactly when lo < hi (lo' <= lo and hi' >= hi; if lo > max(ta, tb) then hi' <= max(ta, tb) = lo', and if
// hi < min(ta, tb) then lo' >= min(ta, tb) = hi').  Four min/max-class instructions per box, as the 8-copy
// walk's max3 + max and min3 + min: the same test at the same cost, with half the stage.
// F32 (with Y4; rtw_compact_nodes fp32): 32-B nodes with the padded fp32 boxes -- the x pair (near, far) and
// the y pair (min, max) sit in the first uint4 as (x near, y min, x far, y max), so two v_pk_fma_f32 give
// (tnx, ty0) and (tfx, ty1) with the ray's (inv.x, inv.y) / (oinv.x, oinv.y) register pairs, and z's two FMAs
// pair up on their own: the box step's six FMAs cost 4 + 4 + 2 x 2 clocks instead of six 4-clock
// v_fma_mix_f32 (profiles/r4_valu_peak/).  The same t = fma(P, inv, -o * inv) on the same fp32 boxes as
// box_next's fast test: the same visits as the 32-B walk of those boxes, a subset of the fp16 walk's.
template <bool COUNT, bool LDS = false, bool Y4 = false, bool F32 = false>
RTW_DHD int traverse_compact(const rtw_launch& L, const uint4* base, const Ray& r, float& t_out,
                                                Counters& cnt) {
    static_assert(!F32 || Y4, "the fp32 nodes are the 4-copy layout");
    const uint32_t oct = order_of(L, r);
    const char* __restrict__ cb = reinterpret_cast<const char*>(base);
    uint32_t a_base = 0;  // LDS: the stage's LDS address
#if defined(__HIP_DEVICE_COMPILE__)
    if constexpr (LDS) a_base = lds_addr(base);
#endif
    // The copy's boxes are stored (near, far) per axis for its octant (rtw_compact_nodes),
    // so min(t0, t1) = t(near) without a min/max pair: fma(P, inv, c) is monotone in P,
    // non-decreasing for inv >= 0.  The sign of inv must then follow the octant, which
    // tests d < 0: a -0.0 component (octant "positive", rcp = -inf) gets +1e30.
    RayTrav rt = ray_trav(r, true);
    if constexpr (Y4)  // y: either sign (med3 below is symmetric in the two y slabs)
        rt.inv = mk((oct & 1u) ? -__builtin_fabsf(rt.inv.x) : __builtin_fabsf(rt.inv.x), rt.inv.y,
                    (oct & 2u) ? -__builtin_fabsf(rt.inv.z) : __builtin_fabsf(rt.inv.z));
    else
        rt.inv = mk((oct & 1u) ? -__builtin_fabsf(rt.inv.x) : __builtin_fabsf(rt.inv.x),
                    (oct & 2u) ? -__builtin_fabsf(rt.inv.y) : __builtin_fabsf(rt.inv.y),
                    (oct & 4u) ? -__builtin_fabsf(rt.inv.z) : __builtin_fabsf(rt.inv.z));
    rt.oinv = mk(-(r.o.x * rt.inv.x), -(r.o.y * rt.inv.y), -(r.o.z * rt.inv.z));
    float closest = kInf;
    int hit = -1;  // the byte offset of the closest sphere's node
    constexpr uint32_t NB = F32 ? 32u : 16u;  // bytes per node
    const uint32_t a0 = a_base + oct * L.n_nodes * NB, end = a0 + L.n_nodes * NB;
    uint32_t i = a0;
    if constexpr (F32) {
#if defined(__HIP_DEVICE_COMPILE__)
        typedef float f2v __attribute__((ext_vector_type(2)));
#else
        struct f2v { float x, y; };
#endif
        const f2v inv_xy = {rt.inv.x, rt.inv.y}, oinv_xy = {rt.oinv.x, rt.oinv.y};
        while (i < end) {
            uint4 c0, c1;
#if defined(__HIP_DEVICE_COMPILE__)
            if constexpr (LDS) {
                c0 = *(lds_uint4*)(uintptr_t)i;
                c1 = *(lds_uint4*)(uintptr_t)(i + 16u);
            } else
#endif
            {
                c0 = *reinterpret_cast<const uint4*>(cb + i);
                c1 = *reinterpret_cast<const uint4*>(cb + i + 16u);
            }
#if defined(__HIP_DEVICE_COMPILE__)
            // both halves in one round trip: left to itself the compiler reads z's pair inside the box branch,
            // a second dependent LDS latency on every inner step
            asm volatile("" ::"v"(c1.x), "v"(c1.y), "v"(c1.z));
#endif
            if (c1.z & RTW_LEAF_BIT) {
                if constexpr (COUNT) cnt.leaves++;
                sphere_leaf(L, r, rt, mk(ubits(c0.x), ubits(c0.y), ubits(c0.z)), ubits(c0.w), i, closest, hit);
                i += 32u;
            } else {
                if constexpr (COUNT) cnt.nodes++;
                float tnx, ty0, tfx, ty1;
#if defined(__HIP_DEVICE_COMPILE__)
                const f2v pn = {ubits(c0.x), ubits(c0.y)}, pf = {ubits(c0.z), ubits(c0.w)};
                const f2v tn = __builtin_elementwise_fma(pn, inv_xy, oinv_xy);
                const f2v tf = __builtin_elementwise_fma(pf, inv_xy, oinv_xy);
                tnx = tn.x;
                ty0 = tn.y;
                tfx = tf.x;
                ty1 = tf.y;
#else
                tnx = std::fma(ubits(c0.x), inv_xy.x, oinv_xy.x);
                ty0 = std::fma(ubits(c0.y), inv_xy.y, oinv_xy.y);
                tfx = std::fma(ubits(c0.z), inv_xy.x, oinv_xy.x);
                ty1 = std::fma(ubits(c0.w), inv_xy.y, oinv_xy.y);
#endif
                const float tnz = __builtin_fmaf(ubits(c1.x), rt.inv.z, rt.oinv.z);
                const float tfz = __builtin_fmaf(ubits(c1.y), rt.inv.z, rt.oinv.z);
                const float lo = med3f(__builtin_fmaxf(__builtin_fmaxf(kTmin, tnx), tnz), ty0, ty1);
                const float hi = med3f(__builtin_fminf(__builtin_fminf(closest, tfx), tfz), ty0, ty1);
                i = (hi <= lo) ? c1.z : i + 32u;
            }
        }
        t_out = closest;
        return hit_with_order(hit < 0 ? hit : (int)(((uint32_t)hit - a0) >> 5), oct);
    }
#if defined(RTW_DIAG_WALK) && defined(__HIP_DEVICE_COMPILE__)
    WalkDiag dgv;
    WalkDiag* dg = &dgv;
    dgv.walks = 1;
#endif
    while (i < end) {
        uint4 c;
#if defined(__HIP_DEVICE_COMPILE__)
        if constexpr (LDS) c = *(lds_uint4*)(uintptr_t)i;
        else
#endif
            c = *reinterpret_cast<const uint4*>(cb + i);
#if defined(RTW_DIAG_WALK) && defined(__HIP_DEVICE_COMPILE__)
        {
            const uint64_t a = __ballot(1), lf = __ballot((c.w & RTW_LEAF_BIT) != 0);
            if (dg_leader()) {
                dg->wsteps++;
                dg->wleaf += lf ? 1u : 0u;
            }
            dg->lsteps++;
            dg->lleaf += (c.w & RTW_LEAF_BIT) ? 1u : 0u;
            (void)a;
        }
#endif
        if (c.w & RTW_LEAF_BIT) {
            if constexpr (COUNT) cnt.leaves++;
            sphere_leaf(L, r, rt, mk(ubits(c.x), ubits(c.y), ubits(c.z)),
                        ubits(c.w & ~RTW_LEAF_BIT), i, closest, hit RTW_DG_ARG(dg));
            i += 16u;
        } else {
            if constexpr (COUNT) cnt.nodes++;
            const float tnx = __builtin_fmaf(h_lo(c.x), rt.inv.x, rt.oinv.x);
            const float tny = __builtin_fmaf(h_hi(c.x), rt.inv.y, rt.oinv.y);
            const float tnz = __builtin_fmaf(h_lo(c.y), rt.inv.z, rt.oinv.z);
            const float tfx = __builtin_fmaf(h_hi(c.y), rt.inv.x, rt.oinv.x);
            const float tfy = __builtin_fmaf(h_lo(c.z), rt.inv.y, rt.oinv.y);
            const float tfz = __builtin_fmaf(h_hi(c.z), rt.inv.z, rt.oinv.z);
            float lo, hi;
            if constexpr (Y4) {  // tny / tfy: the y slabs of min / max y, in either order
                lo = med3f(__builtin_fmaxf(__builtin_fmaxf(kTmin, tnx), tnz), tny, tfy);
                hi = med3f(__builtin_fminf(__builtin_fminf(closest, tfx), tfz), tny, tfy);
            } else {
                lo = __builtin_fmaxf(__builtin_fmaxf(kTmin, tnx), __builtin_fmaxf(tny, tnz));
                hi = __builtin_fminf(__builtin_fminf(closest, tfx), __builtin_fminf(tfy, tfz));
            }
            i = (hi <= lo) ? c.w : i + 16u;
        }
    }
#if defined(RTW_DIAG_WALK) && defined(__HIP_DEVICE_COMPILE__)
    cnt.dsteps = dgv.lsteps;
    cnt.dleaves = dgv.lleaf;
    rtw_diag_flush(dgv);
#endif
    t_out = closest;
    return hit_with_order(hit < 0 ? hit : (int)(((uint32_t)hit - a0) >> 4), oct);
}

// mkey: the path's RNG state (keys ConstantMedium draws; unused without media).
// `nodes` is the base of the node arrays (the octant copy is picked here).
// COMPACT = false: walk `nodes` (e.g. their LDS stage) even where compact nodes exist.
template <uint32_t FEAT, bool COMPACT = true>
RTW_DHD int traverse(const float4* __restrict__ nodes, const rtw_launch& L, const Ray& r,
                                        float& t_out, Counters& cnt, uint64_t mkey = 0) {
    if constexpr (COMPACT && (FEAT & (RTW_F_GEOM | RTW_F_MEDIUM | RTW_F_MOVING)) == 0) {
        if (L.cnodes && L.fast_box) {  // per-step counters only in counted passes
            if (L.cnode32)
                return L.counters ? traverse_compact<true, false, true, true>(L, L.cnodes, r, t_out, cnt)
                                  : traverse_compact<false, false, true, true>(L, L.cnodes, r, t_out, cnt);
            if (L.n_orders == 4)
                return L.counters ? traverse_compact<true, false, true>(L, L.cnodes, r, t_out, cnt)
                                  : traverse_compact<false, false, true>(L, L.cnodes, r, t_out, cnt);
            return L.counters ? traverse_compact<true>(L, L.cnodes, r, t_out, cnt)
                              : traverse_compact<false>(L, L.cnodes, r, t_out, cnt);
        }
    }
    const uint32_t oct = order_of(L, r);
    nodes = order_base(nodes, L, oct);
    const RayTrav rt = ray_trav(r, L.fast_box != 0);
    float closest = kInf;
    int hit = -1;
    uint32_t i = 0;
    const uint32_t n = L.n_nodes;
    while (i < n) i = trav_step<FEAT>(nodes, L, r, rt, i, closest, hit, cnt, mkey);
    t_out = closest;
    return hit_with_order(hit, oct);
}

RTW_DHD f3 background(const rtw_launch& L, const Ray& r) {
    if (L.bg_mode == RTW_BG_GRADIENT) {  // camera.zig:204-206
        f3 ud = unit_vector(r.d);
        float a = 0.5f * (ud.y + 1.0f);
        return mk(1, 1, 1) * splat(1.0f - a) + mk(0.5f, 0.7f, 1.0f) * splat(a);
    }
    return ld3(L.background);  // camera.zig:207
}

// Hit record for the closest hit (objects.zig:139-145) + the material.
struct HitPrep {
    f3 p, normal;
    HitUV uv;
    bool front;
    rtw_dev_material m;
};

// hit record of a quad, in the frame of ray r (Quad.hit objects.zig:237-254)
RTW_DHD void quad_prep(const rtw_dev_quad& q, const Ray& r, float t, HitPrep& h) {
    h.p = r.o + splat(t) * r.d;
    const f3 planar = h.p - ld3(q.q);
    const f3 w = ld3(q.w);
    h.uv.u = dot(w, cross(planar, ld3(q.v)));
    h.uv.v = dot(w, cross(ld3(q.u), planar));
    h.uv.set = true;
    const f3 n = ld3(q.n);
    h.front = dot(r.d, n) < 0;  // setFaceNormal (objects.zig:30-36)
    h.normal = h.front ? n : -n;
    h.uv.outward = n;
}

template <uint32_t FEAT>
RTW_DHD HitPrep object_prep(const rtw_launch& L, const Ray& r, uint32_t kind, uint32_t idx,
                                            uint32_t sub, float t) {
    HitPrep h;
    if (kind == RTW_OBJ_QUAD) {
        const rtw_dev_quad q = L.quads[idx];
        quad_prep(q, r, t, h);
        h.m = L.mats[q.mat];
        return h;
    }
    if (kind == RTW_OBJ_INSTANCE) {
        const rtw_dev_instance* in = L.insts + idx;
        const Ray ro = inst_to_object(in, r);
        const uint32_t ref = L.members[in->first + sub];
        const uint32_t mi = RTW_REF_INDEX(ref);
        uint32_t mat;
        if (RTW_REF_KIND(ref) == RTW_OBJ_SPHERE) {  // Sphere.hit record (objects.zig:138-147)
            const rtw_dev_sphere s = L.sph[mi];
            const f3 center = member_sphere_center<FEAT>(L, s, mi, ro.time);
            h.p = ro.o + splat(t) * ro.d;
            const f3 outward = divs(h.p - center, s.radius);
            h.front = dot(ro.d, outward) < 0;
            h.normal = h.front ? outward : -outward;
            sphere_uv(outward, h.uv.u, h.uv.v);
            h.uv.set = true;
            h.uv.outward = outward;
            mat = s.mat;
        } else {
            const rtw_dev_quad q = L.quads[mi];
            quad_prep(q, ro, t, h);
            mat = q.mat;
        }
        inst_to_world(in, h.p, h.normal);
        h.m = L.mats[mat];
        return h;
    }
    // ConstantMedium record (objects.zig:494-500)
    h.p = r.o + splat(t) * r.d;
    h.normal = mk(1, 0, 0);
    h.front = true;
    h.uv.outward = h.normal;
    h.uv.u = 0;
    h.uv.v = 0;
    h.uv.set = true;
    h.m = L.mats[L.media[idx].mat];
    return h;
}

// The material kind of a walk's hit (the record hit_prep reads, without the hit record itself)
template <uint32_t FEAT>
RTW_DHD uint32_t hit_material_kind(const float4* __restrict__ nodes, const rtw_launch& L, int hit) {
    if (L.n_orders > 1) {
        nodes = order_base(nodes, L, (uint32_t)hit >> RTW_HIT_NODE_BITS);
        hit &= (1 << RTW_HIT_NODE_BITS) - 1;
    }
    const uint32_t node = (uint32_t)hit & ((1u << RTW_HIT_NODE_BITS) - 1u);
    const float4 B = nodes[2 * node + 1];
    uint32_t mat = fbits(B.y);  // sphere leaf
    if constexpr ((FEAT & RTW_F_GEOM) != 0) {
        const uint32_t kind = RTW_LEAF_KIND(fbits(B.w)), idx = fbits(B.z);
        if (kind == RTW_OBJ_QUAD) {
            mat = L.quads[idx].mat;
        } else if (kind == RTW_OBJ_INSTANCE) {
            const uint32_t ref = L.members[L.insts[idx].first + ((uint32_t)hit >> RTW_HIT_NODE_BITS)];
            const uint32_t mi = RTW_REF_INDEX(ref);
            mat = RTW_REF_KIND(ref) == RTW_OBJ_SPHERE ? L.sph[mi].mat : L.quads[mi].mat;
        } else if (kind != RTW_OBJ_SPHERE) {
            mat = L.media[idx].mat;
        }
    }
    return L.mats[mat].kind;
}

template <uint32_t FEAT>
RTW_DHD HitPrep hit_prep(const float4* __restrict__ nodes, const rtw_launch& L, const Ray& r,
                                            int hit, float t) {
    if (L.n_orders > 1) {  // sphere scenes only: the octant copy the walk used
        nodes = order_base(nodes, L, (uint32_t)hit >> RTW_HIT_NODE_BITS);
        hit &= (1 << RTW_HIT_NODE_BITS) - 1;
    }
    if constexpr ((FEAT & RTW_F_GEOM) != 0) {
        const uint32_t node = (uint32_t)hit & ((1u << RTW_HIT_NODE_BITS) - 1u);
        const float4 B = nodes[2 * node + 1];
        const uint32_t kind = RTW_LEAF_KIND(fbits(B.w));
        if (kind != RTW_OBJ_SPHERE) return object_prep<FEAT>(L, r, kind, fbits(B.z), (uint32_t)hit >> RTW_HIT_NODE_BITS, t);
    }
    const float4 A = nodes[2 * hit];
    const float4 B = nodes[2 * hit + 1];
    f3 center = mk(A.x, A.y, A.z);
    if constexpr ((FEAT & RTW_F_MOVING) != 0) {
        if (fbits(B.w)) {
            const float4 cv = L.cvec[fbits(B.z)];
            center = center + splat(r.time) * mk(cv.x, cv.y, cv.z);
        }
    }
    HitPrep h;
    h.p = r.o + splat(t) * r.d;
    h.uv.outward = divs(h.p - center, B.x);
    h.uv.set = false;
    h.uv.u = h.uv.v = 0;
    h.front = dot(r.d, h.uv.outward) < 0;
    h.normal = h.front ? h.uv.outward : -h.uv.outward;
    h.m = L.mats[fbits(B.y)];
    return h;
}

// Does Material.scatter start by drawing vec3.randomUnitVector?
// (Lambertian material.zig:44, Metal :67, Isotropic :140)
template <uint32_t FEAT>
RTW_DHD bool needs_unit_vector(uint32_t kind) {
    if (kind == RTW_MAT_LAMBERTIAN || kind == RTW_MAT_METAL) return true;
    if constexpr ((FEAT & RTW_F_LIGHT) != 0) return kind == RTW_MAT_ISOTROPIC;
    return false;
}

// Material.emitted/scatter (material.zig:18-144) given the hit and, for the
// materials that draw one, the random unit vector `ruv` (already drawn from rng).
// Adds thr*emission to acc; returns true with (att, sc) when the ray scatters.
template <uint32_t FEAT>
RTW_DHD bool scatter_finish(const rtw_launch& L, const Ray& r, const HitPrep& h, f3 ruv,
                                               rtw_rng& rng, f3 thr, f3& acc, f3& att, Ray& sc) {
    const rtw_dev_material& m = h.m;
    sc.o = h.p;
    sc.time = r.time;
    switch (m.kind) {
    case RTW_MAT_LAMBERTIAN: {  // material.zig:43-54
        f3 dir = h.normal + ruv;
        if (near_zero(dir)) dir = h.normal;
        sc.d = dir;
        att = texture_value<FEAT>(L, m.texture, h.uv, h.p);
        return true;
    }
    case RTW_MAT_METAL: {  // material.zig:65-70
        f3 refl = reflect(unit_vector(r.d), h.normal);
        sc.d = refl + splat(m.fuzz) * ruv;
        att = ld3(m.albedo);
        return dot(sc.d, h.normal) > 0;
    }
    case RTW_MAT_DIELECTRIC: {  // material.zig:80-98
        att = mk(1, 1, 1);
        const float ratio = h.front ? (1.0f / m.ir) : m.ir;
        const f3 ud = unit_vector(r.d);
        const float dd = dot(-ud, h.normal);
        const float cos_theta = dd < 1.0f ? dd : 1.0f;
        const float sin_theta = __builtin_sqrtf(1.0f - cos_theta * cos_theta);
        const bool cannot = ratio * sin_theta > 1.0f;
        if (cannot || reflectance(cos_theta, ratio) > rnd(rng))
            sc.d = reflect(ud, h.normal);
        else
            sc.d = refract(ud, h.normal, ratio);
        return true;
    }
    default:
        break;
    }
    if constexpr ((FEAT & RTW_F_LIGHT) != 0) {
        if (m.kind == RTW_MAT_DIFFUSE_LIGHT) {  // material.zig:119-125
            acc = acc + thr * texture_value<FEAT>(L, m.texture, h.uv, h.p);
            return false;
        }
        // RTW_MAT_ISOTROPIC (material.zig:139-143)
        sc.d = ruv;
        att = texture_value<FEAT>(L, m.texture, h.uv, h.p);
        return true;
    }
    return false;
}

// Sequential form (one lane at a time): used by v0 and the debug kernel.
template <uint32_t FEAT>
RTW_DHD bool shade(const float4* __restrict__ nodes, const rtw_launch& L, const Ray& r, int hit,
                                      float t, rtw_rng& rng, f3 thr, f3& acc, f3& att, Ray& sc) {
    const HitPrep h = hit_prep<FEAT>(nodes, L, r, hit, t);
    f3 ruv = mk(0, 0, 0);
    if (needs_unit_vector<FEAT>(h.m.kind)) ruv = random_unit_vector(rng);
    return scatter_finish<FEAT>(L, r, h, ruv, rng, thr, acc, att, sc);
}

// ---------------------------------------------------------------------------
// Rejection sampling of vec3.randomInUnitSphere (D = 3) / randomInUnitDisk
// (D = 2) (vec3.zig:40-45, 59-64): the reference's per-lane loop, each lane
// drawing from its own counter-based stream.  (The wavefront kernels of sphere
// scenes share the randomUnitVector loop between the lanes of a wave, wf_reject3:
// the same draws; the camera's disk loop measured no gain that way)
// ---------------------------------------------------------------------------
template <int D>
RTW_DHD void seq_reject(rtw_rng& rng, float (&out)[D]) {
    for (;;) {
        float w[D];
        float ls;
#pragma unroll
        for (int d = 0; d < D; d++) w[d] = rtw_path_range(rng, -1, 1);
        if constexpr (D == 3) ls = w[0] * w[0] + w[1] * w[1] + w[2] * w[2];
        else ls = w[0] * w[0] + w[1] * w[1];
        if (ls < 1.0f) {
#pragma unroll
            for (int d = 0; d < D; d++) out[d] = w[d];
            return;
        }
    }
}

// Camera.getRay for every lane of the wave (`active` lanes get a ray): the same
// draws in the same order as get_ray, the disk's rejection loop outside the
// per-lane branch (one loop for the wave).
RTW_DHD Ray get_ray_wave(const rtw_launch& L, bool active, uint32_t i, uint32_t j, rtw_rng& rng) {
    const f3 du = ld3(L.du), dv = ld3(L.dv);
    f3 pixel_sample = mk(0, 0, 0);
    if (active) {
        const f3 pixel_center = (ld3(L.pixel00) + du * splat((float)i)) + dv * splat((float)j);
        const float px = -0.5f + rnd(rng);
        const float py = -0.5f + rnd(rng);
        pixel_sample = pixel_center + (splat(px) * du + splat(py) * dv);
    }
    f3 origin = ld3(L.center);
    if (L.defocus_angle > 0) {
        float dsk[2] = {0.0f, 0.0f};
        if (active) seq_reject<2>(rng, dsk);
        origin = (origin + ld3(L.disk_u) * splat(dsk[0])) + ld3(L.disk_v) * splat(dsk[1]);
    }
    Ray r;
    r.o = origin;
    r.d = pixel_sample - origin;
    r.time = active ? rnd(rng) : 0.0f;
    return r;
}

// One sample's radiance: getRay + iterative rayColor (camera.zig:169-208).
template <uint32_t FEAT>
__host__ __device__ f3 sample_radiance(const float4* __restrict__ nodes, const rtw_launch& L, uint32_t pixel, uint32_t x,
                              uint32_t y, uint32_t s, Counters& cnt) {
    rtw_rng rng;
    rng.s = rtw_mix64(L.key0 ^ (((uint64_t)pixel << 32) | (uint64_t)s));
    Ray r = get_ray(L, x, y, rng);
    f3 acc = mk(0, 0, 0);
    f3 thr = mk(1, 1, 1);
    for (uint32_t depth = L.max_depth; depth > 0; depth--) {
        cnt.rays++;
        float t;
        const int hit = traverse<FEAT>(nodes, L, r, t, cnt, rng.s);
        if (hit < 0) {
            acc = acc + thr * background(L, r);
            break;
        }
        f3 att;
        Ray sc;
        if (!shade<FEAT>(nodes, L, r, hit, t, rng, thr, acc, att, sc)) break;
        thr = thr * att;
        r = sc;
    }
    return acc;
}

RTW_DHD bool map_row(const rtw_launch& L, uint32_t r, uint32_t& y) {
    if (L.n_shards) {
        y = rtw_shard_row(L.H, L.rpb, L.n_shards, L.shard, r);
    } else {
        y = r;
    }
    return y < L.H;
}

RTW_DHD void flush_counters(const rtw_launch& L, const Counters& c, uint32_t samples) {
    if (!L.counters) return;
    atomicAdd(&L.counters[RTW_STAT_RAYS], (unsigned long long)c.rays);
    atomicAdd(&L.counters[RTW_STAT_NODES], (unsigned long long)c.nodes);
    atomicAdd(&L.counters[RTW_STAT_LEAVES], (unsigned long long)c.leaves);
    atomicAdd(&L.counters[RTW_STAT_SAMPLES], (unsigned long long)samples);
    if (c.nans) atomicAdd(&L.counters[RTW_STAT_NAN], (unsigned long long)c.nans);
    if (c.tail_rays) atomicAdd(&L.counters[RTW_STAT_TAIL_RAYS], (unsigned long long)c.tail_rays);
}

RTW_DHD bool is_nan3(f3 c) { return !(c.x == c.x) || !(c.y == c.y) || !(c.z == c.z); }

}  // namespace
