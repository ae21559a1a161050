// rtw_kernels.hip -- gfx950 path-tracing kernels: the device side of the
// per-pixel sample loop Camera.render -> rayColor -> BVHNode.hit / Aabb.hit ->
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
#include <hip/hip_runtime.h>

#include "../../include/rtw_gpu.h"
#include "rtw_internal.h"
#include "rtw_layout.h"
#include "rtw_rng.h"

#pragma clang fp contract(off)

#ifndef RTW_STEPS
#define RTW_STEPS 1
#endif

#if defined(RTW_ABLATE_MATH)
// timing ablation only (not IEEE): hardware sqrt / reciprocal
#define __builtin_sqrtf(x) __builtin_amdgcn_sqrtf(x)
#define RTW_DIV(a, b) ((a) * __builtin_amdgcn_rcpf(b))
#else
#define RTW_DIV(a, b) ((a) / (b))
#endif

namespace {

constexpr float kPi = 3.1415926535897932385f;  // rtweekend.zig:4
constexpr float kInf = __builtin_inff();

struct f3 {
    float x, y, z;
};
__device__ __forceinline__ f3 mk(float x, float y, float z) { return f3{x, y, z}; }
__device__ __forceinline__ f3 operator+(f3 a, f3 b) { return f3{a.x + b.x, a.y + b.y, a.z + b.z}; }
__device__ __forceinline__ f3 operator-(f3 a, f3 b) { return f3{a.x - b.x, a.y - b.y, a.z - b.z}; }
__device__ __forceinline__ f3 operator*(f3 a, f3 b) { return f3{a.x * b.x, a.y * b.y, a.z * b.z}; }
__device__ __forceinline__ f3 operator-(f3 a) { return f3{-a.x, -a.y, -a.z}; }
__device__ __forceinline__ f3 splat(float s) { return f3{s, s, s}; }
__device__ __forceinline__ f3 divs(f3 a, float s) { return f3{RTW_DIV(a.x, s), RTW_DIV(a.y, s), RTW_DIV(a.z, s)}; }
__device__ __forceinline__ float dot(f3 u, f3 v) { return u.x * v.x + u.y * v.y + u.z * v.z; }
__device__ __forceinline__ float length_squared(f3 u) { return u.x * u.x + u.y * u.y + u.z * u.z; }
__device__ __forceinline__ f3 unit_vector(f3 v) { return divs(v, __builtin_sqrtf(length_squared(v))); }
__device__ __forceinline__ f3 ld3(const float* p) { return f3{p[0], p[1], p[2]}; }
__device__ __forceinline__ bool near_zero(f3 u) {  // vec3.zig:19-22
    const float s = 1e-8f;
    return __builtin_fabsf(u.x) < s && __builtin_fabsf(u.y) < s && __builtin_fabsf(u.z) < s;
}
__device__ __forceinline__ f3 reflect(f3 v, f3 n) { return v - n * splat(dot(v, n) * 2); }  // vec3.zig:77-79
__device__ __forceinline__ f3 refract(f3 uv, f3 n, float e) {                             // vec3.zig:81-86
    float c = dot(-uv, n);
    float cos_theta = c < 1.0f ? c : 1.0f;
    f3 perp = splat(e) * (uv + n * splat(cos_theta));
    f3 par = n * splat(-__builtin_sqrtf(__builtin_fabsf(1.0f - length_squared(perp))));
    return perp + par;
}
__device__ __forceinline__ uint32_t fbits(float f) { return __float_as_uint(f); }

// ---- RNG helpers (rtweekend.zig / vec3.zig samplers) ----
__device__ __forceinline__ float rnd(rtw_rng& r) { return rtw_rng_float(r); }
__device__ __forceinline__ f3 random_unit_vector(rtw_rng& r) {  // vec3.zig:59-68
#if defined(RTW_ABLATE_REJECT)
    {   // timing ablation only: one candidate, no rejection loop (wrong distribution)
        float x = rtw_rng_range(r, -1, 1), y = rtw_rng_range(r, -1, 1), z = rtw_rng_range(r, -1, 1);
        return unit_vector(mk(x, y, z + 1e-3f));
    }
#endif
    for (;;) {
        float x = rtw_rng_range(r, -1, 1);
        float y = rtw_rng_range(r, -1, 1);
        float z = rtw_rng_range(r, -1, 1);
        f3 p = mk(x, y, z);
        if (length_squared(p) < 1) return unit_vector(p);
    }
}

// Zig std.math.pow(f32, x, 5) via frexp-significand square-and-multiply +
// scalbn (restated; identical fp32 operations to the CPU restatement).
__device__ __forceinline__ float scalbn_f(float x, int n) {
    float y = x;
    if (n > 127) {
        y *= 1.7014118346046923e38f; n -= 127;
        if (n > 127) { y *= 1.7014118346046923e38f; n -= 127; if (n > 127) n = 127; }
    } else if (n < -126) {
        y *= 1.1754943508222875e-38f * 16777216.0f; n += 126 - 24;
        if (n < -126) { y *= 1.1754943508222875e-38f * 16777216.0f; n += 126 - 24; if (n < -126) n = -126; }
    }
    return y * __uint_as_float((uint32_t)(0x7f + n) << 23);
}
__device__ __forceinline__ float frexp_sig(float x, int* e) {
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
    return __uint_as_float((u & 0x807FFFFFu) | 0x3F000000u);
}
__device__ __forceinline__ float pow5(float x) {
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
__device__ __forceinline__ float reflectance(float cosine, float ref_idx) {  // material.zig:101-106
    float r0 = (1 - ref_idx) / (1 + ref_idx);
    r0 = r0 * r0;
    return r0 + (1 - r0) * pow5(1 - cosine);
}

struct Ray {
    f3 o, d;
    float time;
};

// Camera.getRay (camera.zig:156-180)
__device__ __forceinline__ Ray get_ray(const rtw_launch& L, uint32_t i, uint32_t j, rtw_rng& rng) {
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
            dx = rtw_rng_range(rng, -1, 1);
            dy = rtw_rng_range(rng, -1, 1);
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
__device__ float perlin_noise(const float4* tab, f3 p) {  // perlin.zig:117-162 + perlin_interp 30-53
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
    float accum = 0;
#pragma unroll
    for (int di = 0; di < 2; di++)
#pragma unroll
        for (int dj = 0; dj < 2; dj++)
#pragma unroll
            for (int dk = 0; dk < 2; dk++) {
                uint32_t idx = perm[(i + di) & 255] ^ perm[256 + ((j + dj) & 255)] ^ perm[512 + ((k + dk) & 255)];
                float4 c = tab[idx & 255];
                const float i_f = (float)di, j_f = (float)dj, k_f = (float)dk;
                f3 wv = mk(u - i_f, v - j_f, w - k_f);
                accum += (i_f * uu + (1 - i_f) * (1 - uu)) * (j_f * vv + (1 - j_f) * (1 - vv)) *
                         (k_f * ww + (1 - k_f) * (1 - ww)) * dot(mk(c.x, c.y, c.z), wv);
            }
    return accum;
}

__device__ __forceinline__ void sphere_uv(f3 p, float& u, float& v) {  // objects.zig:101-114
    float theta = acosf(-p.y);
    float phi = atan2f(-p.z, p.x) + kPi;
    u = phi / (2 * kPi);
    v = theta / kPi;
}

template <uint32_t FEAT>
__device__ f3 texture_value(const rtw_launch& L, uint32_t ti, f3 outward, f3 p) {
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
            float u, v;
            sphere_uv(outward, u, v);
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
            return splat(0.5f * (1 + sinf(s.z + 10 * turb)));
        }
    }
    return ld3(t.even);  // RTW_TEX_SOLID (textures.zig:43-45)
}

struct Counters {
    uint32_t rays = 0, nodes = 0, leaves = 0, nans = 0;
};

// Per-ray constants of the traversal.
struct RayTrav {
    f3 inv;      // 1 / d per axis (aabb.zig:87)
    float a;     // lengthSquared(d) (objects.zig:124)
    float rcp_a; // hardware 1/a estimate for the sphere fast-reject (0 disables it)
};
__device__ __forceinline__ RayTrav ray_trav(const Ray& r) {
    RayTrav t;
    t.inv = mk(RTW_DIV(1.0f, r.d.x), RTW_DIV(1.0f, r.d.y), RTW_DIV(1.0f, r.d.z));
    t.a = length_squared(r.d);
    // fast-reject only where every intermediate below stays normal and finite
    t.rcp_a = (t.a > 1e-30f && t.a < 1e30f) ? __builtin_amdgcn_rcpf(t.a) : 0.0f;
    return t;
}

constexpr float kTmin = 0.001f;  // camera.zig:187

// One node of the stackless pre-order walk of the reference BVH
// (bvh.zig:122-136): a leaf is tested without a box test (Sphere.hit,
// objects.zig:116-136, open interval (0.001, closest)); an inner node's box is
// tested with [0.001, closest] (Aabb.hit, aabb.zig:82-114).  Returns the next
// node index.  hi/lo use fmax/fmin: for the NaN slabs of a zero direction
// component (0*inf) maxNum keeps the other operand exactly like the
// reference's `if (t0 > min) min = t0`, and lo/hi only grow/shrink, so the
// single final `hi <= lo` equals the per-axis early exit of aabb.zig:111.
template <uint32_t FEAT>
__device__ __forceinline__ uint32_t trav_step(const float4* __restrict__ nodes, const rtw_launch& L, const Ray& r,
                                              const RayTrav& rt, uint32_t i, float& closest, int& hit,
                                              Counters& cnt) {
    const float4 A = nodes[2 * i];
    const float4 B = nodes[2 * i + 1];
    const uint32_t w = fbits(A.w);
    if (w & RTW_LEAF_BIT) {
        cnt.leaves++;
        f3 center = mk(A.x, A.y, A.z);
        if constexpr ((FEAT & RTW_F_MOVING) != 0) {
            if (fbits(B.w)) {  // Sphere.getCenter (objects.zig:94-98)
                const float4 cv = L.cvec[fbits(B.z)];
                center = center + splat(r.time) * mk(cv.x, cv.y, cv.z);
            }
        }
        const f3 oc = r.o - center;
        const float half_b = dot(oc, r.d);
        const float c = length_squared(oc) - B.x * B.x;
        const float disc = half_b * half_b - rt.a * c;
        bool exact = disc >= 0;
#if !defined(RTW_ABLATE_MATH)
        // Exact fast-reject: with hardware sqrt/rcp estimates (<= 1 ulp each) the
        // candidate roots q1, q2 are within (|hb| + sq) / a * 6e-7 of the correctly
        // rounded roots of objects.zig:130-136.  If neither can lie in
        // (tmin, closest) even with a 2^-18 relative margin, the exact test
        // would reject both: skip the IEEE sqrt and divisions.  Guards keep every
        // intermediate finite and normal; otherwise the exact path runs.
        // Written as ONE predicate (no nested branch): a nested-branch form was
        // miscompiled by hipcc 7.2 (numerator left undefined on the guard-false edge).
        {
            const float sa = __builtin_amdgcn_sqrtf(disc);
            const float e = (__builtin_fabsf(half_b) + sa) * rt.rcp_a * 3.8146973e-06f;
            const float q1 = (-half_b - sa) * rt.rcp_a;
            const float q2 = (-half_b + sa) * rt.rcp_a;
            const bool guard = L.fast_reject && rt.rcp_a != 0.0f && disc > 1e-30f && disc < 1e30f &&
                               __builtin_fabsf(half_b) < 1e15f;
            const bool plausible = (q1 + e > kTmin && q1 - e < closest) || (q2 + e > kTmin && q2 - e < closest);
            exact = exact && (plausible || !guard);
        }
#endif
        if (exact) {
            const float sq = __builtin_sqrtf(disc);
            float root = RTW_DIV(-half_b - sq, rt.a);
            bool ok = kTmin < root && root < closest;
            if (!ok) {
                root = RTW_DIV(-half_b + sq, rt.a);
                ok = kTmin < root && root < closest;
            }
            if (ok) {
                closest = root;
                hit = (int)i;
            }
        }
        return w & RTW_SKIP_MASK;
    }
    cnt.nodes++;
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

// World hit for one ray (whole walk).  Returns leaf node index or -1.
template <uint32_t FEAT>
__device__ __forceinline__ int traverse(const float4* __restrict__ nodes, const rtw_launch& L, const Ray& r,
                                        float& t_out, Counters& cnt) {
    const RayTrav rt = ray_trav(r);
    float closest = kInf;
    int hit = -1;
    uint32_t i = 0;
    const uint32_t n = L.n_nodes;
    while (i < n) i = trav_step<FEAT>(nodes, L, r, rt, i, closest, hit, cnt);
    t_out = closest;
    return hit;
}

__device__ __forceinline__ f3 background(const rtw_launch& L, const Ray& r) {
    if (L.bg_mode == RTW_BG_GRADIENT) {  // camera.zig:204-206
        f3 ud = unit_vector(r.d);
        float a = 0.5f * (ud.y + 1.0f);
        return mk(1, 1, 1) * splat(1.0f - a) + mk(0.5f, 0.7f, 1.0f) * splat(a);
    }
    return ld3(L.background);  // camera.zig:207
}

// Hit record for the closest hit (objects.zig:139-145) + the material.
struct HitPrep {
    f3 p, outward, normal;
    bool front;
    rtw_dev_material m;
};

template <uint32_t FEAT>
__device__ __forceinline__ HitPrep hit_prep(const float4* __restrict__ nodes, const rtw_launch& L, const Ray& r,
                                            int hit, float t) {
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
    h.outward = divs(h.p - center, B.x);
    h.front = dot(r.d, h.outward) < 0;
    h.normal = h.front ? h.outward : -h.outward;
    h.m = L.mats[fbits(B.y)];
    return h;
}

// Does Material.scatter start by drawing vec3.randomUnitVector?
// (Lambertian material.zig:44, Metal :67, Isotropic :140)
template <uint32_t FEAT>
__device__ __forceinline__ bool needs_unit_vector(uint32_t kind) {
    if (kind == RTW_MAT_LAMBERTIAN || kind == RTW_MAT_METAL) return true;
    if constexpr ((FEAT & RTW_F_LIGHT) != 0) return kind == RTW_MAT_ISOTROPIC;
    return false;
}

// Material.emitted/scatter (material.zig:18-144) given the hit and, for the
// materials that draw one, the random unit vector `ruv` (already drawn from rng).
// Adds thr*emission to acc; returns true with (att, sc) when the ray scatters.
template <uint32_t FEAT>
__device__ __forceinline__ bool scatter_finish(const rtw_launch& L, const Ray& r, const HitPrep& h, f3 ruv,
                                               rtw_rng& rng, f3 thr, f3& acc, f3& att, Ray& sc) {
    const rtw_dev_material& m = h.m;
    sc.o = h.p;
    sc.time = r.time;
    switch (m.kind) {
    case RTW_MAT_LAMBERTIAN: {  // material.zig:43-54
        f3 dir = h.normal + ruv;
        if (near_zero(dir)) dir = h.normal;
        sc.d = dir;
        att = texture_value<FEAT>(L, m.texture, h.outward, h.p);
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
            acc = acc + thr * texture_value<FEAT>(L, m.texture, h.outward, h.p);
            return false;
        }
        // RTW_MAT_ISOTROPIC (material.zig:139-143)
        sc.d = ruv;
        att = texture_value<FEAT>(L, m.texture, h.outward, h.p);
        return true;
    }
    return false;
}

// Sequential form (one lane at a time): used by v0 and the debug kernel.
template <uint32_t FEAT>
__device__ __forceinline__ bool shade(const float4* __restrict__ nodes, const rtw_launch& L, const Ray& r, int hit,
                                      float t, rtw_rng& rng, f3 thr, f3& acc, f3& att, Ray& sc) {
    const HitPrep h = hit_prep<FEAT>(nodes, L, r, hit, t);
    f3 ruv = mk(0, 0, 0);
    if (needs_unit_vector<FEAT>(h.m.kind)) ruv = random_unit_vector(rng);
    return scatter_finish<FEAT>(L, r, h, ruv, rng, thr, acc, att, sc);
}

// ---------------------------------------------------------------------------
// Wave-cooperative rejection sampling (vec3.randomInUnitSphere D=3 /
// randomInUnitDisk D=2, vec3.zig:40-45, 59-64).  The sequential loop runs until
// the slowest lane of the wave accepts (E[max] ~ 6 iterations for 48 lanes at
// p = 0.52).  The RNG is counter-based, so candidate j of a lane is simply draws
// j*D+1 .. j*D+D after its current state: every round, all 64 lanes evaluate
// candidates of the still-unresolved lanes (64/n helpers each, consecutive j),
// and each lane takes its FIRST accepted candidate -- exactly the sequential
// result and stream position.  A draw on Zig's rare extra-draw path
// (clz >= 41, p = 2^-41) would shift positions: such a lane falls back to the
// sequential loop from its start.  Must be called with every lane of the wave
// converged (helpers are idle lanes).
// ---------------------------------------------------------------------------
__device__ __forceinline__ float float_from_draw(uint64_t x, int lz) {
    const uint32_t bits = ((uint32_t)(126 - lz) << 23) | (uint32_t)(x & 0x7FFFFFu);
    return __uint_as_float(bits);
}

template <int D>
__device__ __forceinline__ void seq_reject(rtw_rng& rng, float (&out)[D]) {
    for (;;) {
        float w[D];
        float ls;
#pragma unroll
        for (int d = 0; d < D; d++) w[d] = rtw_rng_range(rng, -1, 1);
        if constexpr (D == 3) ls = w[0] * w[0] + w[1] * w[1] + w[2] * w[2];
        else ls = w[0] * w[0] + w[1] * w[1];
        if (ls < 1.0f) {
#pragma unroll
            for (int d = 0; d < D; d++) out[d] = w[d];
            return;
        }
    }
}

template <int D>
__device__ __forceinline__ void coop_reject(bool active, rtw_rng& rng, float (&out)[D], uint32_t* slot,
                                            bool coop = true) {
    if (!coop) {  // A/B knob (RTW_COOP=0): plain per-lane loop, same results
        if (active) seq_reject<D>(rng, out);
        return;
    }
    const uint32_t lane = __lane_id();
    const uint64_t lt = lane ? (~0ull >> (64 - lane)) : 0ull;
    uint64_t pend = __ballot(active);
    if (!pend) return;
    const uint64_t s0 = rng.s;
    uint32_t base = 0;
    bool done = !active, fall = false;
    while (pend) {
        const uint32_t n = (uint32_t)__popcll(pend);
        const uint32_t k = 64u / n;
        const bool me = (pend >> lane) & 1ull;
        const uint32_t rank = (uint32_t)__popcll(pend & lt);
        if (me) slot[rank] = lane;
        const uint32_t tr = lane / k;
        const bool helper = tr < n;
        const uint32_t tl = helper ? slot[tr] : lane;
        const uint32_t ts_lo = __shfl((uint32_t)s0, (int)tl), ts_hi = __shfl((uint32_t)(s0 >> 32), (int)tl);
        const uint32_t tj = (uint32_t)__shfl((int)base, (int)tl) + (lane - tr * k);
        float v[D];
        bool acc = false, rare = false;
        if (helper) {
            uint64_t st = (((uint64_t)ts_hi << 32) | ts_lo) + (uint64_t)(tj * (uint32_t)D) * RTW_GOLDEN;
            float ls = 0.0f;
#pragma unroll
            for (int d = 0; d < D; d++) {
                st += RTW_GOLDEN;
                const uint64_t x = rtw_mix64(st);
                const int lz = rtw_clz64(x);
                rare = rare || lz >= 41;
                v[d] = -1.0f + 2.0f * float_from_draw(x, lz);  // randomDoubleRange(-1, 1)
            }
            if constexpr (D == 3) ls = v[0] * v[0] + v[1] * v[1] + v[2] * v[2];
            else ls = v[0] * v[0] + v[1] * v[1];            // + 0*0 of the disk's z (exact)
            acc = !rare && ls < 1.0f;
        } else {
#pragma unroll
            for (int d = 0; d < D; d++) v[d] = 0.0f;
        }
        const uint64_t accb = __ballot(acc), rareb = __ballot(rare);
        const uint32_t off = me ? rank * k : 0u;
        const uint64_t m = (k >= 64u) ? ~0ull : ((1ull << k) - 1ull);
        const uint64_t a = me ? ((accb >> off) & m) : 0ull;
        const uint64_t q = me ? ((rareb >> off) & m) : 0ull;
        const uint32_t fa = a ? (uint32_t)__builtin_ctzll(a) : 64u;
        const uint32_t fq = q ? (uint32_t)__builtin_ctzll(q) : 64u;
        const int src = (int)((me && fa < 64u) ? off + fa : lane);
        float got[D];
#pragma unroll
        for (int d = 0; d < D; d++) got[d] = __shfl(v[d], src);
        if (me) {
            if (fq < 64u && fq <= fa) {
                fall = true;
            } else if (fa < 64u) {
#pragma unroll
                for (int d = 0; d < D; d++) out[d] = got[d];
                rng.s = s0 + (uint64_t)((base + fa + 1u) * (uint32_t)D) * RTW_GOLDEN;
                done = true;
            } else {
                base += k;
            }
        }
        pend = __ballot(!done && !fall);
    }
    if (fall) {  // exact sequential path (rare-draw safe)
        rng.s = s0;
        seq_reject<D>(rng, out);
    }
}

// One sample's radiance: getRay + iterative rayColor (camera.zig:169-208).
template <uint32_t FEAT>
__device__ f3 sample_radiance(const float4* __restrict__ nodes, const rtw_launch& L, uint32_t pixel, uint32_t x,
                              uint32_t y, uint32_t s, Counters& cnt) {
    rtw_rng rng;
    rng.s = rtw_mix64(L.key0 ^ (((uint64_t)pixel << 32) | (uint64_t)s));
    Ray r = get_ray(L, x, y, rng);
    f3 acc = mk(0, 0, 0);
    f3 thr = mk(1, 1, 1);
    for (uint32_t depth = L.max_depth; depth > 0; depth--) {
        cnt.rays++;
        float t;
        const int hit = traverse<FEAT>(nodes, L, r, t, cnt);
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

__device__ __forceinline__ bool map_row(const rtw_launch& L, uint32_t r, uint32_t& y) {
    if (L.n_shards) {
        const uint32_t blk = r / L.rpb;
        y = (blk * L.n_shards + L.shard) * L.rpb + r % L.rpb;
    } else {
        y = r;
    }
    return y < L.H;
}

__device__ __forceinline__ void flush_counters(const rtw_launch& L, const Counters& c, uint32_t samples) {
    if (!L.counters) return;
    atomicAdd(&L.counters[RTW_STAT_RAYS], (unsigned long long)c.rays);
    atomicAdd(&L.counters[RTW_STAT_NODES], (unsigned long long)c.nodes);
    atomicAdd(&L.counters[RTW_STAT_LEAVES], (unsigned long long)c.leaves);
    atomicAdd(&L.counters[RTW_STAT_SAMPLES], (unsigned long long)samples);
    if (c.nans) atomicAdd(&L.counters[RTW_STAT_NAN], (unsigned long long)c.nans);
}

__device__ __forceinline__ bool is_nan3(f3 c) { return !(c.x == c.x) || !(c.y == c.y) || !(c.z == c.z); }

// ---------------------------------------------------------------------------
// v0: one thread per pixel, each wave an 8x8 pixel tile, block = 32x8 pixels;
// samples [s0, s1) looped in order, accumulator read once / written once.
// Kept as the simple reference kernel (and the A/B baseline for v1).
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void render_pixels_v0(rtw_launch L) {
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint32_t x = blockIdx.x * 32 + wave * 8 + (lane & 7);
    const uint32_t r = L.row0 + blockIdx.y * 8 + (lane >> 3);
    if (x >= L.W || r >= L.row0 + L.n_rows) return;
    uint32_t y;
    if (!map_row(L, r, y)) return;
    const uint32_t pixel = y * L.W + x;
    if (!L.n_shards && (pixel < L.pix_begin || pixel >= L.pix_end)) return;
    float4* slot = L.accum + (size_t)r * L.W + x;
    float4 acc = *slot;
    Counters cnt;
    const uint32_t px = x + L.pixel_offset, py = y + L.pixel_offset;  // camera.zig:100-101
    for (uint32_t s = L.s0; s < L.s1; s++) {
        f3 c = sample_radiance<RTW_F_ALL>(L.nodes, L, pixel, px, py, s, cnt);
        if (is_nan3(c)) cnt.nans++;
        acc.x += c.x;
        acc.y += c.y;
        acc.z += c.z;
    }
    acc.w = (float)L.s1;  // writeColor: buffer[i][3] = number_of_samples (camera.zig:56)
    *slot = acc;
    flush_counters(L, cnt, L.s1 - L.s0);
}

// ---------------------------------------------------------------------------
// v1: persistent megakernel.
//  * grid = resident blocks only; each wave pulls 16x16 pixel tiles from a
//    global atomic work counter and hands pixels to its lanes one at a time
//    (ballot + mbcnt), so a lane that finishes its pixel immediately takes the
//    next one -- no lane waits for the slowest pixel of a fixed tile;
//  * a lane owns one pixel for all samples [s0, s1) and adds the sample
//    radiances in sample order (bit-identical sums to the reference order);
//  * per-lane path regeneration: when a lane's path ends it starts the next
//    sample at once (ST_NEWSAMPLE) instead of waiting for the wave;
//  * traversal runs node steps until >= shade_min lanes have finished their
//    walk (ballot popcount), then shades only those lanes: the wave's shading
//    pass is shared by many lanes instead of one;
//  * the BVH (<= RTW_LDS_NODES nodes) is staged once per block in LDS.
// ---------------------------------------------------------------------------
enum : uint32_t { ST_TRAV = 0, ST_SHADE = 1, ST_NEWSAMPLE = 2, ST_NEWPIXEL = 3, ST_DONE = 4 };

#if defined(RTW_STAMPS)
// diagnostic build only: per-wave cycle split of the persistent loop
#define STAMP(var)                                  \
    __builtin_amdgcn_sched_barrier(0);              \
    var = __builtin_amdgcn_s_memtime();             \
    __builtin_amdgcn_sched_barrier(0);
#define STAMP_ADD(acc, t0, t1) acc += (t1) - (t0);
#else
#define STAMP(var)
#define STAMP_ADD(acc, t0, t1)
#endif

__device__ __forceinline__ uint32_t popc64(uint64_t m) { return (uint32_t)__popcll(m); }

template <uint32_t FEAT, bool LDS, int WAVES>
__global__ __launch_bounds__(256, WAVES) void render_persistent_v1(rtw_launch L) {
    extern __shared__ float4 lds_nodes[];
    const float4* __restrict__ nodes;
    if constexpr (LDS) {
        const uint32_t n4 = 2 * L.n_nodes;
        for (uint32_t k = threadIdx.x; k < n4; k += blockDim.x) lds_nodes[k] = L.nodes[k];
        __syncthreads();
        nodes = lds_nodes;
    } else {
        nodes = L.nodes;
    }
    const uint32_t lane = __lane_id();
    const uint64_t lt_mask = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
    const uint32_t n_nodes = L.n_nodes;
    __shared__ uint32_t coop_slots[4][64];  // per-wave scratch of coop_reject (1 KiB, multiple of 16 B)
    uint32_t* const coop_slot = coop_slots[threadIdx.x >> 6];

    // wave-uniform queue state
    uint32_t q_cur = 0, q_end = 0;
    bool q_empty = false;

    uint32_t st = ST_NEWPIXEL;
    uint32_t pixel = 0, out_idx = 0, px = 0, py = 0, s = 0;
    f3 acc = mk(0, 0, 0), Ls = mk(0, 0, 0), thr = mk(1, 1, 1);
    rtw_rng rng;
    rng.s = 0;
    Ray ray;
    ray.o = ray.d = mk(0, 0, 0);
    ray.time = 0;
    RayTrav rt;
    rt.inv = mk(0, 0, 0);
    rt.a = 0;
    uint32_t depth = 0, ti = 0;
    float closest = kInf;
    int hit = -1;
    Counters cnt;
    uint32_t samples_done = 0;
#if defined(RTW_STAMPS)
    uint64_t c_assign = 0, c_gen = 0, c_trav = 0, c_shade = 0, c_steps = 0, c_passes = 0, t0, t1;
#endif

    for (;;) {
        STAMP(t0)
        // ---- 1. hand pixels to lanes that need one
        uint64_t need = __ballot(st == ST_NEWPIXEL);
        while (need) {
            if (q_cur >= q_end) {
                if (q_empty) {
                    if (st == ST_NEWPIXEL) st = ST_DONE;
                    break;
                }
                uint32_t t = 0;
                if (lane == 0) t = atomicAdd(L.work_counter, 1u);
                t = __builtin_amdgcn_readfirstlane(t);
                if (t >= L.n_tiles) {
                    q_empty = true;
                    continue;
                }
                // tiles are handed out last-row-first: the bottom of a frame (ground,
                // many bounces) is the expensive part, the top (sky) the cheap one, so
                // the end-of-launch tail is made of cheap pixels (order never changes
                // arithmetic: a pixel is always one lane's, samples in order)
                if (L.tile_order) t = L.n_tiles - 1 - t;
                q_cur = t * RTW_TILE;
                q_end = q_cur + RTW_TILE;
            }
            const uint32_t avail = q_end - q_cur;
            const uint32_t rank = popc64(need & lt_mask);
            if (st == ST_NEWPIXEL && rank < avail) {
                const uint32_t seq = q_cur + rank;
                const uint32_t tile = seq / RTW_TILE, k = seq % RTW_TILE;
                const uint32_t x = (tile % L.n_tiles_x) * RTW_TILE_W + k % RTW_TILE_W;
                const uint32_t r = L.row0 + (tile / L.n_tiles_x) * RTW_TILE_H + k / RTW_TILE_W;
                uint32_t y;
                if (x < L.W && r < L.row0 + L.n_rows && map_row(L, r, y)) {
                    const uint32_t pix = y * L.W + x;
                    if (L.n_shards || (pix >= L.pix_begin && pix < L.pix_end)) {
                        pixel = pix;
                        out_idx = r * L.W + x;
                        px = x + L.pixel_offset;  // camera.zig:100-101
                        py = y + L.pixel_offset;
                        s = L.s0;
                        const float4 a0 = L.accum[out_idx];
                        acc = mk(a0.x, a0.y, a0.z);
                        st = (s < L.s1) ? ST_NEWSAMPLE : ST_NEWPIXEL;
                    }
                }
            }
            const uint32_t cnt_need = popc64(need);
            q_cur += cnt_need < avail ? cnt_need : avail;
            need = __ballot(st == ST_NEWPIXEL);
        }
        const uint64_t live = __ballot(st != ST_DONE);
        if (!live) break;
        STAMP(t1) STAMP_ADD(c_assign, t0, t1)

        // ---- 2. start a new sample: getRay (camera.zig:169-180).  Jitter draws
        // per lane, the defocus-disk rejection loop wave-cooperatively, then time.
        {
            const bool starting = st == ST_NEWSAMPLE;
            f3 pixel_sample = mk(0, 0, 0);
            if (starting) {
                rng.s = rtw_mix64(L.key0 ^ (((uint64_t)pixel << 32) | (uint64_t)s));
                const f3 du = ld3(L.du), dv = ld3(L.dv);
                const f3 pixel_center = (ld3(L.pixel00) + du * splat((float)px)) + dv * splat((float)py);
                const float jx = -0.5f + rnd(rng);
                const float jy = -0.5f + rnd(rng);
                pixel_sample = pixel_center + (splat(jx) * du + splat(jy) * dv);
            }
            float dsk[2] = {0.0f, 0.0f};
            const bool defocus = L.defocus_angle > 0;
            if (defocus) coop_reject<2>(starting, rng, dsk, coop_slot, L.coop != 0);
            if (starting) {
                f3 origin = ld3(L.center);
                if (defocus) origin = (origin + ld3(L.disk_u) * splat(dsk[0])) + ld3(L.disk_v) * splat(dsk[1]);
                ray.o = origin;
                ray.d = pixel_sample - origin;
                ray.time = rnd(rng);
                thr = mk(1, 1, 1);
                Ls = mk(0, 0, 0);
                depth = L.max_depth;
                if (depth == 0) {
                    st = ST_SHADE;  // rayColor(r, 0) = 0: finishes below without tracing
                    hit = -2;
                } else {
                    rt = ray_trav(ray);
                    ti = 0;
                    closest = kInf;
                    hit = -1;
                    st = ST_TRAV;
                    cnt.rays++;
                }
            }
        }

        STAMP(t0) STAMP_ADD(c_gen, t1, t0)
        // ---- 3. traversal until enough lanes are ready to shade
        {
            const uint32_t n_live = popc64(live);
            const uint32_t want = L.shade_min < n_live ? L.shade_min : n_live;
            for (;;) {
                const uint64_t trav = __ballot(st == ST_TRAV);
                if (!trav) break;
                if (popc64(__ballot(st == ST_SHADE)) >= want) break;
                // RTW_STEPS node steps per readiness check (amortises the ballot/branch bookkeeping)
#pragma unroll
                for (int u = 0; u < RTW_STEPS; u++) {
                    if (st == ST_TRAV) {
                        ti = trav_step<FEAT>(nodes, L, ray, rt, ti, closest, hit, cnt);
                        if (ti >= n_nodes) st = ST_SHADE;
                    }
                }
#if defined(RTW_STAMPS)
                c_steps++;
#endif
            }
        }
        STAMP(t1) STAMP_ADD(c_trav, t0, t1)
#if defined(RTW_STAMPS)
        c_passes++;
#endif

        // ---- 4. shade lanes whose walk is complete: hit record per lane, the
        // randomUnitVector rejection loop wave-cooperatively, then the material.
        {
            const bool shading = st == ST_SHADE;
            HitPrep hp;
            bool need_uv = false;
            if (shading && hit >= 0) {
                hp = hit_prep<FEAT>(nodes, L, ray, hit, closest);
                need_uv = needs_unit_vector<FEAT>(hp.m.kind);
            }
            float ruv3[3] = {0.0f, 0.0f, 0.0f};
            coop_reject<3>(need_uv, rng, ruv3, coop_slot, L.coop != 0);
            if (shading) {
                bool cont = false;
                if (hit == -1) {
                    Ls = Ls + thr * background(L, ray);
                } else if (hit >= 0) {
                    f3 att;
                    Ray sc;
                    const f3 ruv = need_uv ? unit_vector(mk(ruv3[0], ruv3[1], ruv3[2])) : mk(0, 0, 0);
                    if (scatter_finish<FEAT>(L, ray, hp, ruv, rng, thr, Ls, att, sc) && depth > 1) {
                        thr = thr * att;
                        ray = sc;
                        depth--;
                        rt = ray_trav(ray);
                        ti = 0;
                        closest = kInf;
                        hit = -1;
                        st = ST_TRAV;
                        cnt.rays++;
                        cont = true;
                    }
                }
                if (!cont) {
                    if (is_nan3(Ls)) cnt.nans++;
                    acc = acc + Ls;
                    samples_done++;
                    s++;
                    if (s < L.s1) {
                        st = ST_NEWSAMPLE;
                    } else {
                        L.accum[out_idx] = make_float4(acc.x, acc.y, acc.z, (float)L.s1);  // camera.zig:55-56
                        st = ST_NEWPIXEL;
                    }
                }
            }
        }
        STAMP(t0) STAMP_ADD(c_shade, t1, t0)
    }
    flush_counters(L, cnt, samples_done);
#if defined(RTW_STAMPS)
    if (L.counters && lane == 0) {
        atomicAdd(&L.counters[8], (unsigned long long)c_assign);
        atomicAdd(&L.counters[9], (unsigned long long)c_gen);
        atomicAdd(&L.counters[10], (unsigned long long)c_trav);
        atomicAdd(&L.counters[11], (unsigned long long)c_shade);
        atomicAdd(&L.counters[12], (unsigned long long)c_steps);
        atomicAdd(&L.counters[13], (unsigned long long)c_passes);
    }
#endif
}

__global__ void debug_rng_kernel(uint64_t seed, uint32_t pixel, uint32_t sample, uint32_t n, float* out) {
    if (threadIdx.x | blockIdx.x) return;
    rtw_rng r;
    r.s = rtw_mix64(rtw_mix64(seed) ^ (((uint64_t)pixel << 32) | (uint64_t)sample));
    for (uint32_t k = 0; k < n; k++) out[k] = rtw_rng_float(r);
}

// Diagnostic: for every bounce of one sample, brute-force all leaves with the
// exact test and with the fast-reject filter; record the first leaf the filter
// would wrongly reject (out[8..]).
__device__ void debug_filter_check(const rtw_launch& L, const Ray& r, float* out) {
    const RayTrav rt = ray_trav(r);
    for (uint32_t i = 0; i < L.n_nodes; i++) {
        const float4 A = L.nodes[2 * i];
        const float4 B = L.nodes[2 * i + 1];
        if (!(fbits(A.w) & RTW_LEAF_BIT)) continue;
        const f3 oc = r.o - mk(A.x, A.y, A.z);
        const float half_b = dot(oc, r.d);
        const float c = length_squared(oc) - B.x * B.x;
        const float disc = half_b * half_b - rt.a * c;
        if (!(disc >= 0)) continue;
        const float sq = __builtin_sqrtf(disc);
        const float r1 = (-half_b - sq) / rt.a, r2 = (-half_b + sq) / rt.a;
        const bool acc_exact = (kTmin < r1) || (kTmin < r2);
        const float sa = __builtin_amdgcn_sqrtf(disc);
        const float e = (__builtin_fabsf(half_b) + sa) * rt.rcp_a * 3.8146973e-06f;
        const float q1 = (-half_b - sa) * rt.rcp_a, q2 = (-half_b + sa) * rt.rcp_a;
        const bool acc_fast = (q1 + e > kTmin) || (q2 + e > kTmin);
        if (acc_exact && !acc_fast && out[8] == 0) {
            out[8] = 1; out[9] = (float)i; out[10] = half_b; out[11] = c; out[12] = disc; out[13] = sq; out[14] = sa;
            out[15] = rt.a; out[16] = rt.rcp_a; out[17] = r1; out[18] = r2; out[19] = q1; out[20] = q2; out[21] = e;
        }
    }
}

__global__ void debug_sample_kernel(rtw_launch L, uint32_t pixel, uint32_t sample, float* out) {
    if (threadIdx.x | blockIdx.x) return;
    for (int k = 0; k < 32; k++) out[k] = 0;
    Counters cnt;
    const uint32_t x = pixel % L.W, y = pixel / L.W;
    f3 c = sample_radiance<RTW_F_ALL>(L.nodes, L, pixel, x + L.pixel_offset, y + L.pixel_offset, sample, cnt);
    out[0] = c.x;
    out[1] = c.y;
    out[2] = c.z;
    out[3] = (float)cnt.rays;
    out[4] = (float)cnt.nodes;
    out[5] = (float)cnt.leaves;
    // replay the path to run the filter check on every bounce ray
    rtw_rng rng;
    rng.s = rtw_mix64(L.key0 ^ (((uint64_t)pixel << 32) | (uint64_t)sample));
    Ray r = get_ray(L, x + L.pixel_offset, y + L.pixel_offset, rng);
    f3 acc = mk(0, 0, 0), thr = mk(1, 1, 1);
    int bounce = 0;
    for (uint32_t depth = L.max_depth; depth > 0; depth--, bounce++) {
        debug_filter_check(L, r, out);
        float t;
        const int hit = traverse<RTW_F_ALL>(L.nodes, L, r, t, cnt);
        // brute-force exact closest over all leaves
        {
            const RayTrav rt = ray_trav(r);
            float best = kInf;
            int besti = -1;
            for (uint32_t i = 0; i < L.n_nodes; i++) {
                const float4 A = L.nodes[2 * i];
                const float4 B = L.nodes[2 * i + 1];
                if (!(fbits(A.w) & RTW_LEAF_BIT)) continue;
                const f3 oc = r.o - mk(A.x, A.y, A.z);
                const float half_b = dot(oc, r.d);
                const float c = length_squared(oc) - B.x * B.x;
                const float disc = half_b * half_b - rt.a * c;
                if (!(disc >= 0)) continue;
                const float sq = __builtin_sqrtf(disc);
                float root = (-half_b - sq) / rt.a;
                if (!(kTmin < root)) root = (-half_b + sq) / rt.a;
                if (kTmin < root && root < best) { best = root; besti = (int)i; }
            }
            if ((besti != hit || (hit >= 0 && best != t)) && out[22] == 0) {
                out[22] = 1; out[23] = (float)bounce; out[24] = (float)hit; out[25] = t; out[26] = (float)besti;
                out[27] = best; out[28] = r.o.x; out[29] = r.o.y; out[30] = r.o.z;
            }
        }
        if (hit < 0) break;
        f3 att;
        Ray sc;
        if (!shade<RTW_F_ALL>(L.nodes, L, r, hit, t, rng, thr, acc, att, sc)) break;
        r = sc;
    }
}

template <uint32_t FEAT, bool LDS, int WAVES>
void launch_v1(const rtw_launch& L, hipStream_t stream, int grid) {
    const size_t lds = LDS ? (size_t)L.n_nodes * 32 : 0;
    hipLaunchKernelGGL((render_persistent_v1<FEAT, LDS, WAVES>), dim3(grid), dim3(256), lds, stream, L);
}

template <uint32_t FEAT, bool LDS, int WAVES>
int occupancy_v1(size_t lds_bytes) {
    int b = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, render_persistent_v1<FEAT, LDS, WAVES>, 256,
                                                     LDS ? lds_bytes : 0) != hipSuccess)
        b = 1;
    return b < 1 ? 1 : b;
}

// waves-per-SIMD launch-bound variants (RTW_WAVES): 1 = compiler's choice, 6, 8
uint32_t pick_feat(uint32_t f) {
    if ((f & ~RTW_F_CHECKER) == 0) return f ? RTW_F_CHECKER : 0u;
    return RTW_F_ALL;
}


template <uint32_t FEAT, bool LDS>
void launch_waves(const rtw_launch& L, hipStream_t st, int grid, int waves) {
    if (waves >= 8) launch_v1<FEAT, LDS, 8>(L, st, grid);
    else if (waves >= 6) launch_v1<FEAT, LDS, 6>(L, st, grid);
    else launch_v1<FEAT, LDS, 1>(L, st, grid);
}
template <uint32_t FEAT, bool LDS>
int occ_waves(size_t lds, int waves) {
    if (waves >= 8) return occupancy_v1<FEAT, LDS, 8>(lds);
    if (waves >= 6) return occupancy_v1<FEAT, LDS, 6>(lds);
    return occupancy_v1<FEAT, LDS, 1>(lds);
}

}  // namespace

void rtw_launch_render(const rtw_launch& L, void* stream, int variant, int grid) {
    hipStream_t st = (hipStream_t)stream;
    if (variant == 0) {
        dim3 block(256);
        dim3 g((L.W + 31) / 32, (L.n_rows + 7) / 8);
        hipLaunchKernelGGL(render_pixels_v0, g, block, 0, st, L);
        return;
    }
    const bool lds = L.n_nodes <= RTW_LDS_NODES && L.use_lds;
    const int w = (int)L.waves;
    switch (pick_feat(L.feat)) {
    case 0u:
        lds ? launch_waves<0u, true>(L, st, grid, w) : launch_waves<0u, false>(L, st, grid, w);
        break;
    case RTW_F_CHECKER:
        lds ? launch_waves<RTW_F_CHECKER, true>(L, st, grid, w) : launch_waves<RTW_F_CHECKER, false>(L, st, grid, w);
        break;
    default:
        lds ? launch_waves<RTW_F_ALL, true>(L, st, grid, w) : launch_waves<RTW_F_ALL, false>(L, st, grid, w);
        break;
    }
}

int rtw_persistent_grid(uint32_t feat, uint32_t n_nodes, int waves, bool use_lds) {
    int dev = 0, n_cu = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev);
    if (n_cu <= 0) n_cu = 256;
    const bool lds = n_nodes <= RTW_LDS_NODES && use_lds;
    const size_t bytes = (size_t)n_nodes * 32;
    int b;
    switch (pick_feat(feat)) {
    case 0u: b = lds ? occ_waves<0u, true>(bytes, waves) : occ_waves<0u, false>(bytes, waves); break;
    case RTW_F_CHECKER:
        b = lds ? occ_waves<RTW_F_CHECKER, true>(bytes, waves) : occ_waves<RTW_F_CHECKER, false>(bytes, waves);
        break;
    default: b = lds ? occ_waves<RTW_F_ALL, true>(bytes, waves) : occ_waves<RTW_F_ALL, false>(bytes, waves); break;
    }
    return n_cu * b;
}

void rtw_launch_debug_rng(uint64_t seed, uint32_t pixel, uint32_t sample, uint32_t n, float* d_out, void* stream) {
    hipLaunchKernelGGL(debug_rng_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, seed, pixel, sample, n, d_out);
}

void rtw_launch_debug_sample(const rtw_launch& L, uint32_t pixel, uint32_t sample, float* d_out, void* stream) {
    hipLaunchKernelGGL(debug_sample_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, L, pixel, sample, d_out);
}
