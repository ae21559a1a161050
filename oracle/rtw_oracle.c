/*
 * rtw_oracle.c -- TEST INFRASTRUCTURE ONLY (see rtw_oracle.h).
 *
 * Faithful CPU restatement of the reference hot path, structured like the Zig
 * code it follows: recursive rayColor, pointer BVH in the reference topology
 * (random axis, heap sort, median split; leaves tested without a box test),
 * tagged-union material/texture dispatch, per-sample writeColor/toGamma2,
 * samples-outer / pixels-inner loop over contiguous Task chunks.
 *
 * Build with -ffp-contract=off and no fast-math: Zig's default float mode is
 * strict (no FMA contraction), so every +,-,*,/,sqrt here is one IEEE-754 fp32
 * operation in the same order as the Zig source.
 */
#include "rtw_oracle.h"

#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

#include "zig_libm.h"  /* std.math.acos/atan2, @sin, @log as the Zig toolchain computes them */

#define GOLDEN 0x9E3779B97F4A7C15ULL
#define PI_F 3.1415926535897932385f                 /* rtweekend.zig:4 */
#define INF_F (__builtin_inff())

/* ------------------------------------------------------------------------- */
/* RNG: counter-based replacement for std.crypto.random (rtweekend.zig:14-16) */
/* ------------------------------------------------------------------------- */
uint64_t oracle_mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
    return z ^ (z >> 31);
}

typedef struct { uint64_t s; } rng_t;

static rng_t rng_stream(uint64_t seed, uint64_t domain, uint32_t a, uint32_t b) {
    rng_t r;
    uint64_t k = oracle_mix64(seed + domain * GOLDEN);
    r.s = oracle_mix64(k ^ (((uint64_t)a << 32) | (uint64_t)b));
    return r;
}

static inline uint64_t rng_next(rng_t* r) {
    r->s += GOLDEN;
    return oracle_mix64(r->s);
}

static inline int clz64(uint64_t x) { return x ? __builtin_clzll(x) : 64; }

/* Zig std.Random.float(f32): 23 low bits -> mantissa, exponent from the
 * leading-zero count of the 64-bit draw (exponentially biased, covers every
 * representable value of [0,1)). */
static inline float rnd(rng_t* r) {
    uint64_t x = rng_next(r);
    int lz = clz64(x);
    if (lz >= 41) {
        lz = 41 + clz64(rng_next(r));
        if (lz == 41 + 64) lz += __builtin_clz((uint32_t)rng_next(r) | 0x7FFu);
    }
    uint32_t bits = ((uint32_t)(126 - lz) << 23) | (uint32_t)(x & 0x7FFFFFu);
    float f;
    memcpy(&f, &bits, 4);
    return f;
}

/* rtweekend.zig:18-20 */
static inline float rnd_range(rng_t* r, float mn, float mx) { return mn + (mx - mn) * rnd(r); }

/* Render-domain draws (camera, scatter): the same Weyl step, a lowbias32 finalizer
 * on hi ^ lo, 24-bit float k * 2^-24 (csrc/rtw_rng.h rtw_path_float, DESIGN.md RNG). */
static inline uint32_t lowbias32(uint32_t x) {
    x ^= x >> 16;
    x *= 0x7feb352du;
    x ^= x >> 15;
    x *= 0x846ca68bu;
    x ^= x >> 16;
    return x;
}
static inline float rndp(rng_t* r) {
    r->s += GOLDEN;
    uint32_t h = lowbias32((uint32_t)(r->s >> 32) ^ (uint32_t)r->s);
    return (float)(h >> 8) * 5.9604644775390625e-08f;
}
static inline float rndp_range(rng_t* r, float mn, float mx) { return mn + (mx - mn) * rndp(r); }

/* rtweekend.zig:23-27 (biased: returns up to max+1) */
static inline uint32_t rnd_int_range(rng_t* r, uint32_t mn, uint32_t mx) {
    float mn_f = (float)mn, mx_f = (float)(mx + 1);
    return (uint32_t)roundf(rnd_range(r, mn_f, mx_f));
}

void oracle_rng_floats(uint64_t seed, uint64_t domain, uint32_t a, uint32_t b, uint32_t n, float* out) {
    rng_t r = rng_stream(seed, domain, a, b);
    for (uint32_t i = 0; i < n; i++) out[i] = rnd(&r);
}

void oracle_path_floats(uint64_t seed, uint32_t a, uint32_t b, uint32_t n, float* out) {
    rng_t r = rng_stream(seed, 0, a, b);
    for (uint32_t i = 0; i < n; i++) out[i] = rndp(&r);
}

void oracle_rng_u64(uint64_t seed, uint64_t domain, uint32_t a, uint32_t b, uint32_t n, uint64_t* out) {
    rng_t r = rng_stream(seed, domain, a, b);
    for (uint32_t i = 0; i < n; i++) out[i] = rng_next(&r);
}

/* ------------------------------------------------------------------------- */
/* Instrumentation                                                           */
/* ------------------------------------------------------------------------- */
static int g_count = 0;
typedef struct { uint64_t rays, nodes, leaves, texels, noise, samples; } counters_t;
static __thread counters_t t_cnt;
static counters_t g_cnt;
static pthread_mutex_t g_cnt_mu = PTHREAD_MUTEX_INITIALIZER;

void oracle_counters_enable(int on) { g_count = on; }
void oracle_counters_reset(void) {
    pthread_mutex_lock(&g_cnt_mu);
    memset(&g_cnt, 0, sizeof g_cnt);
    memset(&t_cnt, 0, sizeof t_cnt);
    pthread_mutex_unlock(&g_cnt_mu);
}
static void counters_flush(void) {
    if (!g_count) return;
    pthread_mutex_lock(&g_cnt_mu);
    g_cnt.rays += t_cnt.rays; g_cnt.nodes += t_cnt.nodes; g_cnt.leaves += t_cnt.leaves;
    g_cnt.texels += t_cnt.texels; g_cnt.noise += t_cnt.noise; g_cnt.samples += t_cnt.samples;
    memset(&t_cnt, 0, sizeof t_cnt);
    pthread_mutex_unlock(&g_cnt_mu);
}
void oracle_counters_get(uint64_t out[6]) {
    counters_flush();
    out[0] = g_cnt.rays; out[1] = g_cnt.nodes; out[2] = g_cnt.leaves;
    out[3] = g_cnt.texels; out[4] = g_cnt.noise; out[5] = g_cnt.samples;
}
#define COUNT(field) do { if (g_count) t_cnt.field++; } while (0)

/* ------------------------------------------------------------------------- */
/* vec3.zig                                                                  */
/* ------------------------------------------------------------------------- */
typedef struct { float e[3]; } v3;
static inline v3 V(float x, float y, float z) { v3 r = {{x, y, z}}; return r; }
static inline v3 vload(const float* p) { return V(p[0], p[1], p[2]); }
static inline v3 add(v3 a, v3 b) { return V(a.e[0] + b.e[0], a.e[1] + b.e[1], a.e[2] + b.e[2]); }
static inline v3 sub(v3 a, v3 b) { return V(a.e[0] - b.e[0], a.e[1] - b.e[1], a.e[2] - b.e[2]); }
static inline v3 mul(v3 a, v3 b) { return V(a.e[0] * b.e[0], a.e[1] * b.e[1], a.e[2] * b.e[2]); }
static inline v3 vdiv(v3 a, v3 b) { return V(a.e[0] / b.e[0], a.e[1] / b.e[1], a.e[2] / b.e[2]); }
static inline v3 neg(v3 a) { return V(-a.e[0], -a.e[1], -a.e[2]); }
static inline v3 splat(float s) { return V(s, s, s); }
static inline float length_squared(v3 u) { return u.e[0] * u.e[0] + u.e[1] * u.e[1] + u.e[2] * u.e[2]; }
static inline float vlength(v3 u) { return sqrtf(length_squared(u)); }
static inline int near_zero(v3 u) {
    const float s = 1e-8f;
    return fabsf(u.e[0]) < s && fabsf(u.e[1]) < s && fabsf(u.e[2]) < s;
}
static inline float dot(v3 u, v3 v) { return u.e[0] * v.e[0] + u.e[1] * v.e[1] + u.e[2] * v.e[2]; }
static inline v3 cross(v3 u, v3 v) {
    return V(u.e[1] * v.e[2] - u.e[2] * v.e[1], u.e[2] * v.e[0] - u.e[0] * v.e[2], u.e[0] * v.e[1] - u.e[1] * v.e[0]);
}
static inline v3 unit_vector(v3 v) { return vdiv(v, splat(vlength(v))); }

/* vec3.zig:40-45 */
static inline v3 random_in_unit_disk(rng_t* r) {
    for (;;) {
        float x = rndp_range(r, -1, 1);
        float y = rndp_range(r, -1, 1);
        v3 p = V(x, y, 0);
        if (length_squared(p) < 1) return p;
    }
}
/* vec3.zig:47-49 */
static inline v3 random_v(rng_t* r) {
    float x = rnd(r), y = rnd(r), z = rnd(r);
    return V(x, y, z);
}
/* vec3.zig:51-57 */
static inline v3 random_range_v(rng_t* r, float mn, float mx) {
    float x = rnd_range(r, mn, mx), y = rnd_range(r, mn, mx), z = rnd_range(r, mn, mx);
    return V(x, y, z);
}
/* vec3.zig:59-64 */
static inline v3 random_in_unit_sphere(rng_t* r) {
    for (;;) {
        float x = rndp_range(r, -1, 1), y = rndp_range(r, -1, 1), z = rndp_range(r, -1, 1);
        v3 p = V(x, y, z);
        if (length_squared(p) < 1) return p;
    }
}
/* vec3.zig:66-68 */
static inline v3 random_unit_vector(rng_t* r) { return unit_vector(random_in_unit_sphere(r)); }
/* vec3.zig:77-79 */
static inline v3 reflect(v3 v, v3 n) { return sub(v, mul(n, splat(dot(v, n) * 2))); }
/* vec3.zig:81-86 */
static inline v3 refract(v3 uv, v3 n, float etai_over_etat) {
    float c = dot(neg(uv), n);
    float cos_theta = c < 1.0f ? c : 1.0f;
    v3 r_out_perp = mul(splat(etai_over_etat), add(uv, mul(n, splat(cos_theta))));
    v3 r_out_parallel = mul(n, splat(-sqrtf(fabsf(1.0f - length_squared(r_out_perp)))));
    return add(r_out_perp, r_out_parallel);
}

/* ------------------------------------------------------------------------- */
/* Zig std.math.pow(f32, x, y) for the Schlick term (material.zig:105).      */
/* Restated: integer-exponent path = square-and-multiply on the frexp        */
/* significand, then scalbn (Zig std/math/pow.zig, 0.12).                    */
/* ------------------------------------------------------------------------- */
static float frexp_sig(float x, int* e) {
    uint32_t u; memcpy(&u, &x, 4);
    int ee = (int)((u >> 23) & 0xFF);
    if (ee == 0) {                              /* subnormal or zero */
        if (x == 0) { *e = 0; return x; }
        float y = x * 18446744073709551616.0f;  /* 2^64 */
        float s = frexp_sig(y, e);
        *e -= 64;
        return s;
    }
    if (ee == 0xFF) { *e = 0; return x; }
    *e = ee - 126;
    u = (u & 0x807FFFFFu) | 0x3F000000u;
    memcpy(&x, &u, 4);
    return x;
}
static float scalbn_f(float x, int n) {          /* correctly rounded x * 2^n */
    float y = x;
    if (n > 127) {
        y *= 1.7014118346046923e38f; n -= 127;   /* 0x1p127 */
        if (n > 127) { y *= 1.7014118346046923e38f; n -= 127; if (n > 127) n = 127; }
    } else if (n < -126) {
        y *= 1.1754943508222875e-38f * 16777216.0f; n += 126 - 24;
        if (n < -126) { y *= 1.1754943508222875e-38f * 16777216.0f; n += 126 - 24; if (n < -126) n = -126; }
    }
    uint32_t b = (uint32_t)(0x7f + n) << 23; float s; memcpy(&s, &b, 4);
    return y * s;
}
float oracle_pow(float x, float y) {
    if (y == 0 || x == 1) return 1;
    if (isnan(x) || isnan(y)) return NAN;
    if (x == 0) {
        /* pow(+-0, y>0 odd int) = +-0 ; other y>0 -> +0 (schlick never takes y<0) */
        float yi = truncf(y);
        if (y > 0) return (yi == y && fmodf(y, 2) != 0) ? x : 0.0f;
        return INF_F;
    }
    if (y == 0.5f) return sqrtf(x);
    if (y == -0.5f) return 1 / sqrtf(x);
    float ay = fabsf(y);
    float yi = truncf(ay), yf = ay - yi;
    if (yf != 0 && x < 0) return NAN;
    if (yi >= 2147483648.0f) return expf(y * logf(x));
    float a1 = 1.0f; int ae = 0;
    if (yf != 0) {
        if (yf > 0.5f) { yf -= 1; yi += 1; }
        a1 = expf(yf * logf(x));
    }
    int xe; float x1 = frexp_sig(x, &xe);
    int32_t i = (int32_t)yi;
    while (i != 0) {
        if (xe < -(1 << 9) || (1 << 9) < xe) {   /* overflow guard (never hit for Schlick) */
            ae += xe; break;
        }
        if (i & 1) { a1 *= x1; ae += xe; }
        x1 *= x1;
        xe <<= 1;
        if (x1 < 0.5f) { x1 += x1; xe -= 1; }
        i >>= 1;
    }
    if (y < 0) { a1 = 1 / a1; ae = -ae; }
    return scalbn_f(a1, ae);
}

/* ------------------------------------------------------------------------- */
/* ray.zig, interval.zig                                                     */
/* ------------------------------------------------------------------------- */
typedef struct { v3 origin, direction; float time; } ray3;
static inline v3 ray_at(const ray3* r, float t) { return add(r->origin, mul(splat(t), r->direction)); }
typedef struct { float min, max; } interval_t;
static inline int surrounds(interval_t i, float x) { return i.min < x && x < i.max; }  /* interval.zig:12-14 */
static inline float clampi(interval_t i, float x) {                                   /* interval.zig:16-20 */
    if (x < i.min) return i.min;
    if (x > i.max) return i.max;
    return x;
}

/* ------------------------------------------------------------------------- */
/* aabb.zig                                                                  */
/* ------------------------------------------------------------------------- */
typedef struct { interval_t ax[3]; } aabb_t;
static aabb_t aabb_from_points(v3 a, v3 b) {  /* aabb.zig:18-26 */
    aabb_t r;
    for (int i = 0; i < 3; i++) {
        r.ax[i].min = a.e[i] < b.e[i] ? a.e[i] : b.e[i];
        r.ax[i].max = a.e[i] > b.e[i] ? a.e[i] : b.e[i];
    }
    return r;
}
static aabb_t aabb_from_boxes(aabb_t a, aabb_t b) {  /* aabb.zig:28-34, interval.zig:42-44 */
    aabb_t r;
    for (int i = 0; i < 3; i++) {
        r.ax[i].min = a.ax[i].min < b.ax[i].min ? a.ax[i].min : b.ax[i].min;
        r.ax[i].max = a.ax[i].max > b.ax[i].max ? a.ax[i].max : b.ax[i].max;
    }
    return r;
}
/* aabb.zig:82-114 */
static int aabb_hit(const aabb_t* b, const ray3* r, interval_t ray_t) {
    float ray_t_min = ray_t.min, ray_t_max = ray_t.max;
    for (int a = 0; a < 3; a++) {
        float invD = 1 / r->direction.e[a];
        float orig = r->origin.e[a];
        float t0 = (b->ax[a].min - orig) * invD;
        float t1 = (b->ax[a].max - orig) * invD;
        if (invD < 0) { float tmp = t1; t1 = t0; t0 = tmp; }
        if (t0 > ray_t_min) ray_t_min = t0;
        if (t1 < ray_t_max) ray_t_max = t1;
        if (ray_t_max <= ray_t_min) return 0;
    }
    return 1;
}
int oracle_aabb_hit(const float box[6], const float origin[3], const float dir[3], float tmin, float tmax) {
    aabb_t b;
    for (int i = 0; i < 3; i++) { b.ax[i].min = box[i]; b.ax[i].max = box[3 + i]; }
    ray3 r = {vload(origin), vload(dir), 0};
    interval_t it = {tmin, tmax};
    return aabb_hit(&b, &r, it);
}

/* ------------------------------------------------------------------------- */
/* objects.zig: HitRecord, Sphere                                            */
/* ------------------------------------------------------------------------- */
typedef struct {
    v3 p, normal;
    uint32_t mat;
    float t, u, v;
    int front_face;
} hit_record_t;

static inline void set_face_normal(hit_record_t* rec, const ray3* r, v3 outward) {  /* objects.zig:30-36 */
    rec->front_face = dot(r->direction, outward) < 0;
    rec->normal = rec->front_face ? outward : neg(outward);
}

/* objects.zig:101-114 */
static void get_sphere_uv(v3 p, float* u, float* v) {
    float theta = zig_acosf(-p.e[1]);
    float phi = zig_atan2f(-p.e[2], p.e[0]) + PI_F;
    *u = phi / (2 * PI_F);
    *v = theta / PI_F;
}
void oracle_sphere_uv(const float p[3], float uv[2]) { get_sphere_uv(vload(p), &uv[0], &uv[1]); }
/* the restated transcendentals over arrays (tests): fn 0 acos, 1 atan2(y = a, x = b), 2 sin, 3 log, 4 atan */
void oracle_libm(int fn, const float* a, const float* b, float* out, uint64_t n) {
    for (uint64_t i = 0; i < n; i++) {
        switch (fn) {
            case 0: out[i] = zig_acosf(a[i]); break;
            case 1: out[i] = zig_atan2f(a[i], b[i]); break;
            case 2: out[i] = zig_sinf(a[i]); break;
            case 3: out[i] = zig_logf(a[i]); break;
            default: out[i] = zig_atanf(a[i]); break;
        }
    }
}

typedef struct {
    v3 center1, center_vec;
    float radius;
    int is_moving;
    uint32_t mat;
    uint32_t orig;             /* index in the scene description (dump/tests only) */
    aabb_t bbox;
} sphere_t;

static inline v3 sphere_center(const sphere_t* s, float time) {       /* objects.zig:94-98 */
    return add(s->center1, mul(splat(time), s->center_vec));
}

/* objects.zig:116-148 */
static int sphere_hit(const sphere_t* s, const ray3* r, interval_t ray_t, hit_record_t* rec) {
    v3 center = s->is_moving ? sphere_center(s, r->time) : s->center1;
    v3 oc = sub(r->origin, center);
    float a = length_squared(r->direction);
    float half_b = dot(oc, r->direction);
    float c = length_squared(oc) - s->radius * s->radius;
    float discriminant = half_b * half_b - a * c;
    if (discriminant < 0) return 0;
    float sqrtd = sqrtf(discriminant);
    float root = (-half_b - sqrtd) / a;
    if (!surrounds(ray_t, root)) {
        root = (-half_b + sqrtd) / a;
        if (!surrounds(ray_t, root)) return 0;
    }
    rec->t = root;
    rec->p = ray_at(r, rec->t);
    v3 outward = vdiv(sub(rec->p, center), splat(s->radius));
    set_face_normal(rec, r, outward);
    get_sphere_uv(outward, &rec->u, &rec->v);
    rec->mat = s->mat;
    return 1;
}

static void sphere_from_desc(const o_sphere* d, sphere_t* s) {     /* objects.zig:80-92 */
    s->center1 = vload(d->center1);
    s->radius = d->radius;
    s->mat = d->material;
    v3 rvec = V(d->radius, d->radius, d->radius);
    if (d->is_moving) {
        v3 c2 = vload(d->center2);                 /* initMoving: center_vec = center2 - center1 */
        s->center_vec = sub(c2, s->center1);
        s->is_moving = 1;
        aabb_t b1 = aabb_from_points(sub(s->center1, rvec), add(s->center1, rvec));
        aabb_t b2 = aabb_from_points(sub(c2, rvec), add(c2, rvec));
        s->bbox = aabb_from_boxes(b1, b2);
    } else {
        s->center_vec = V(0, 0, 0);
        s->is_moving = 0;
        s->bbox = aabb_from_points(sub(s->center1, rvec), add(s->center1, rvec));
    }
}

int oracle_sphere_hit(const o_sphere* d, const float origin[3], const float dir[3], float time,
                      float tmin, float tmax, float out[8]) {
    sphere_t s; sphere_from_desc(d, &s);
    ray3 r = {vload(origin), vload(dir), time};
    interval_t it = {tmin, tmax};
    hit_record_t rec;
    if (!sphere_hit(&s, &r, it, &rec)) return 0;
    out[0] = rec.t;
    for (int i = 0; i < 3; i++) { out[1 + i] = rec.p.e[i]; out[4 + i] = rec.normal.e[i]; }
    out[7] = (float)rec.front_face;
    return 1;
}

/* ------------------------------------------------------------------------- */
/* perlin.zig                                                                */
/* ------------------------------------------------------------------------- */
/* perlin.zig:30-53 */
static float perlin_interp(v3 c[2][2][2], float u, float v, float w) {
    float uu = u * u * (3 - 2 * u);
    float vv = v * v * (3 - 2 * v);
    float ww = w * w * (3 - 2 * w);
    float accum = 0;
    for (int i = 0; i < 2; i++)
        for (int j = 0; j < 2; j++)
            for (int k = 0; k < 2; k++) {
                float i_f = (float)i, j_f = (float)j, k_f = (float)k;
                v3 weight_v = V(u - i_f, v - j_f, w - k_f);
                accum += (i_f * uu + (1 - i_f) * (1 - uu)) *
                         (j_f * vv + (1 - j_f) * (1 - vv)) *
                         (k_f * ww + (1 - k_f) * (1 - ww)) * dot(c[i][j][k], weight_v);
            }
    return accum;
}
/* perlin.zig:117-162 */
float oracle_perlin_noise(const o_perlin* pl, const float pp[3]) {
    float u = pp[0] - floorf(pp[0]);
    float v = pp[1] - floorf(pp[1]);
    float w = pp[2] - floorf(pp[2]);
    int32_t i = (int32_t)floorf(pp[0]);
    int32_t j = (int32_t)floorf(pp[1]);
    int32_t k = (int32_t)floorf(pp[2]);
    v3 c[2][2][2];
    for (int di = 0; di < 2; di++)
        for (int dj = 0; dj < 2; dj++)
            for (int dk = 0; dk < 2; dk++) {
                uint32_t idi = (uint32_t)((i + di) & 255);
                uint32_t idj = (uint32_t)((j + dj) & 255);
                uint32_t idk = (uint32_t)((k + dk) & 255);
                uint32_t idx = (uint32_t)(pl->perm_x[idi] ^ pl->perm_y[idj] ^ pl->perm_z[idk]);
                c[di][dj][dk] = vload(pl->ranvec[idx & 255]);
            }
    return perlin_interp(c, u, v, w);
}
/* perlin.zig:103-115 */
float oracle_perlin_turb(const o_perlin* pl, const float pp[3], int depth) {
    float accum = 0;
    v3 temp_p = vload(pp);
    float weight = 1.0f;
    for (int i = 0; i < depth; i++) {
        accum += weight * oracle_perlin_noise(pl, temp_p.e);
        weight *= 0.5f;
        temp_p = mul(temp_p, splat(2));
    }
    return fabsf(accum);
}

/* perlin.zig:8-28, 83-101 restated on the seeded stream.  permute's
 * randomIntRange(0,i) can return i+1; at i=255 that indexes p[256] (UB in the
 * reference) -- clamped to 255 here (documented deviation). */
static void permute(rng_t* r, uint16_t* p, uint16_t n) {
    for (uint16_t i = n - 1; i > 0; i--) {
        uint32_t target = rnd_int_range(r, 0, i);
        if (target > 255) target = 255;
        uint16_t tmp = p[i];
        p[i] = p[target];
        p[target] = tmp;
    }
}
int oracle_gen_perlin(uint64_t seed, uint32_t id, o_perlin* out) {
    rng_t r = rng_stream(seed, 3, id, 0);
    for (int i = 0; i < 256; i++) {
        v3 v = unit_vector(random_range_v(&r, -1, 1));
        out->ranvec[i][0] = v.e[0]; out->ranvec[i][1] = v.e[1]; out->ranvec[i][2] = v.e[2];
    }
    uint16_t* tabs[3] = {out->perm_x, out->perm_y, out->perm_z};
    for (int t = 0; t < 3; t++) {
        for (int i = 0; i < 256; i++) tabs[t][i] = (uint16_t)i;
        permute(&r, tabs[t], 256);
    }
    return 0;
}

/* ------------------------------------------------------------------------- */
/* textures.zig, rtw_image.zig                                               */
/* ------------------------------------------------------------------------- */
static uint32_t img_clamp(uint32_t x, uint32_t low, uint32_t high) {  /* rtw_image.zig:37-45 */
    if (x < low) return low;
    if (x < high) return x;
    return high - 1;
}

static v3 texture_value(const o_scene_desc* d, uint32_t ti, float u, float v, v3 p) {
    const o_texture* t = &d->textures[ti];
    switch (t->kind) {
    case O_TEX_SOLID:                                          /* textures.zig:43-45 */
        return vload(t->even);
    case O_TEX_CHECKER: {                                      /* textures.zig:60-72 */
        int32_t xi = (int32_t)floorf(t->scale * p.e[0]);
        int32_t yi = (int32_t)floorf(t->scale * p.e[1]);
        int32_t zi = (int32_t)floorf(t->scale * p.e[2]);
        int is_even = ((xi + yi + zi) % 2) == 0;
        return is_even ? vload(t->even) : vload(t->odd);
    }
    case O_TEX_IMAGE: {                                        /* textures.zig:85-104 */
        const o_image* im = &d->images[t->image];
        if (im->height <= 0) return V(0, 1, 1);
        interval_t unit = {0, 1};
        float new_u = clampi(unit, u);
        float new_v = 1.0f - clampi(unit, v);
        float u_p = new_u * (float)im->width;
        float v_p = new_v * (float)im->height;
        uint32_t i = (uint32_t)floorf(u_p);
        uint32_t j = (uint32_t)floorf(v_p);
        uint32_t x = img_clamp(i, 0, im->width), y = img_clamp(j, 0, im->height);  /* rtw_image.zig:51-62 */
        uint32_t start = y * im->bytes_per_row + x * 4;
        const uint8_t* px = im->data + start;
        COUNT(texels);
        const float color_scale = 1.0f / 255.0f;
        return V(color_scale * (float)px[0], color_scale * (float)px[1], color_scale * (float)px[2]);
    }
    case O_TEX_NOISE: {                                        /* textures.zig:118-123 */
        const o_perlin* pl = &d->perlins[t->perlin];
        v3 s = mul(splat(t->scale), p);
        COUNT(noise);
        return splat(0.5f * (1 + zig_sinf(s.e[2] + 10 * oracle_perlin_turb(pl, s.e, 7))));
    }
    }
    return V(0, 0, 0);
}
void oracle_texture_value(const o_scene_desc* d, uint32_t tex, float u, float v, const float p[3], float out[3]) {
    v3 r = texture_value(d, tex, u, v, vload(p));
    out[0] = r.e[0]; out[1] = r.e[1]; out[2] = r.e[2];
}

/* ------------------------------------------------------------------------- */
/* material.zig                                                              */
/* ------------------------------------------------------------------------- */
float oracle_reflectance(float cosine, float ref_idx) {          /* material.zig:101-106 */
    float r0 = (1 - ref_idx) / (1 + ref_idx);
    r0 = r0 * r0;
    return r0 + (1 - r0) * oracle_pow(1 - cosine, 5);
}
void oracle_reflect(const float v[3], const float n[3], float out[3]) {
    v3 r = reflect(vload(v), vload(n)); memcpy(out, r.e, 12);
}
void oracle_refract(const float uv[3], const float n[3], float e, float out[3]) {
    v3 r = refract(vload(uv), vload(n), e); memcpy(out, r.e, 12);
}

/* material.zig:18-22 dispatch */
static int scatter(const o_scene_desc* d, const ray3* r_in, const hit_record_t* rec, v3* attenuation,
                   ray3* scattered, rng_t* rng) {
    const o_material* m = &d->materials[rec->mat];
    switch (m->kind) {
    case O_MAT_LAMBERTIAN: {                                   /* material.zig:43-54 */
        v3 dir = add(rec->normal, random_unit_vector(rng));
        if (near_zero(dir)) dir = rec->normal;
        scattered->origin = rec->p; scattered->direction = dir; scattered->time = r_in->time;
        *attenuation = texture_value(d, m->texture, rec->u, rec->v, rec->p);
        return 1;
    }
    case O_MAT_METAL: {                                        /* material.zig:65-70 */
        v3 reflected = reflect(unit_vector(r_in->direction), rec->normal);
        scattered->origin = rec->p;
        scattered->direction = add(reflected, mul(splat(m->fuzz), random_unit_vector(rng)));
        scattered->time = r_in->time;
        *attenuation = vload(m->albedo);
        return dot(scattered->direction, rec->normal) > 0;
    }
    case O_MAT_DIELECTRIC: {                                   /* material.zig:80-98 */
        *attenuation = V(1, 1, 1);
        float refraction_ratio = rec->front_face ? (1.0f / m->ir) : m->ir;
        v3 unit_direction = unit_vector(r_in->direction);
        float dd = dot(neg(unit_direction), rec->normal);
        float cos_theta = dd < 1.0f ? dd : 1.0f;
        float sin_theta = sqrtf(1.0f - cos_theta * cos_theta);
        int cannot_refract = refraction_ratio * sin_theta > 1.0f;
        v3 direction;
        if (cannot_refract || oracle_reflectance(cos_theta, refraction_ratio) > rndp(rng))
            direction = reflect(unit_direction, rec->normal);
        else
            direction = refract(unit_direction, rec->normal, refraction_ratio);
        scattered->origin = rec->p; scattered->direction = direction; scattered->time = r_in->time;
        return 1;
    }
    case O_MAT_DIFFUSE_LIGHT:                                  /* material.zig:119-121 */
        return 0;
    case O_MAT_ISOTROPIC: {                                    /* material.zig:139-143 */
        scattered->origin = rec->p; scattered->direction = random_unit_vector(rng); scattered->time = r_in->time;
        *attenuation = texture_value(d, m->texture, rec->u, rec->v, rec->p);
        return 1;
    }
    }
    return 0;
}
/* material.zig:24-29 */
static v3 emitted(const o_scene_desc* d, uint32_t mat, float u, float v, v3 p) {
    const o_material* m = &d->materials[mat];
    if (m->kind == O_MAT_DIFFUSE_LIGHT) return texture_value(d, m->texture, u, v, p);
    return V(0, 0, 0);
}

/* ------------------------------------------------------------------------- */
/* objects.zig: Quad, HittableList, Translate, RotateY, ConstantMedium       */
/* ------------------------------------------------------------------------- */
/* Interval.contains (interval.zig:8-10) */
static inline int contains(interval_t i, float x) { return i.min <= x && x <= i.max; }

/* Aabb.pad (aabb.zig:36-43), Interval.expand (interval.zig:26-29) */
static aabb_t aabb_pad(aabb_t b) {
    const float delta = 0.0001f;
    for (int k = 0; k < 3; k++) {
        if (!(b.ax[k].max - b.ax[k].min >= delta)) {
            const float padding = delta / 2.0f;
            b.ax[k].min = b.ax[k].min - padding;
            b.ax[k].max = b.ax[k].max + padding;
        }
    }
    return b;
}

typedef struct {
    v3 q, u, v, normal, w;
    float d;
    uint32_t mat;
    aabb_t bbox;
} quad_t;

static void quad_from_desc(const o_quad* o, quad_t* q) {      /* objects.zig:201-210 */
    q->q = vload(o->q); q->u = vload(o->u); q->v = vload(o->v);
    q->mat = o->material;
    v3 n = cross(q->u, q->v);
    q->normal = unit_vector(n);
    q->d = dot(q->normal, q->q);
    q->w = vdiv(n, splat(dot(n, n)));
    q->bbox = aabb_pad(aabb_from_points(q->q, add(add(q->q, q->u), q->v)));
}

/* objects.zig:222-255 */
static int quad_hit(const quad_t* q, const ray3* r, interval_t ray_t, hit_record_t* rec) {
    float denom = dot(q->normal, r->direction);
    if (fabsf(denom) < 1e-8f) return 0;
    float t = (q->d - dot(q->normal, r->origin)) / denom;
    if (!contains(ray_t, t)) return 0;
    v3 intersection = ray_at(r, t);
    v3 planar = sub(intersection, q->q);
    float alpha = dot(q->w, cross(planar, q->v));
    float beta = dot(q->w, cross(q->u, planar));
    if ((alpha < 0) || (1 < alpha) || (beta < 0) || (1 < beta)) return 0;   /* isInterior :212-220 */
    rec->u = alpha;
    rec->v = beta;
    rec->t = t;
    rec->p = intersection;
    rec->mat = q->mat;
    set_face_normal(rec, r, q->normal);
    return 1;
}

int oracle_quad_hit(const o_quad* o, const float origin[3], const float dir[3], float tmin, float tmax,
                    float out[10]) {
    quad_t q; quad_from_desc(o, &q);
    ray3 r = {vload(origin), vload(dir), 0};
    interval_t it = {tmin, tmax};
    hit_record_t rec;
    if (!quad_hit(&q, &r, it, &rec)) return 0;
    out[0] = rec.t;
    for (int i = 0; i < 3; i++) { out[1 + i] = rec.p.e[i]; out[4 + i] = rec.normal.e[i]; }
    out[7] = (float)rec.front_face; out[8] = rec.u; out[9] = rec.v;
    return 1;
}

typedef struct {
    uint32_t kind;
    v3 offset;                   /* translate */
    float sin_theta, cos_theta;  /* rotate_y */
} xf_t;

typedef struct {
    uint32_t first, count, n_xf;
    xf_t xf[O_MAX_XF];
    aabb_t bbox;
} inst_t;

typedef struct {
    o_object boundary;
    float neg_inv_density;
    uint32_t mat;
    aabb_t bbox;
} medium_t;

/* BVH leaf = one world object */
typedef struct {
    uint32_t kind, index;
    uint32_t orig;             /* position in world_objects (dump/tests only) */
    aabb_t bbox;
} object_t;

typedef struct bvh_node {
    const object_t* leaf;
    const struct bvh_node *left, *right;
    aabb_t bbox;
} bvh_node_t;

typedef struct world {
    o_scene_desc desc;
    sphere_t* spheres;         /* every sphere record (world objects and list members) */
    quad_t* quads;
    inst_t* insts;
    medium_t* media;
    object_t* objects;         /* world_objects.items (reordered in place by the build) */
    uint32_t n;
    bvh_node_t* pool;
    uint32_t pool_used, pool_cap;
    const bvh_node_t* root;
    uint32_t axis_draws;
    rng_t build_rng;
} world_t;

/* RotateY.init (objects.zig:340-388): sin/cos and the rotated box */
static aabb_t rotate_y_box(aabb_t bbox, float sin_theta, float cos_theta) {
    const float inf = INF_F;
    v3 mn = V(inf, inf, inf), mx = V(-inf, -inf, -inf);
    for (int i = 0; i < 2; i++)
        for (int j = 0; j < 2; j++)
            for (int k = 0; k < 2; k++) {
                float i_f = (float)i, j_f = (float)j, k_f = (float)k;
                float x = i_f * bbox.ax[0].max + (1 - i_f) * bbox.ax[0].min;
                float y = j_f * bbox.ax[1].max + (1 - j_f) * bbox.ax[1].min;
                float z = k_f * bbox.ax[2].max + (1 - k_f) * bbox.ax[2].min;
                float newx = cos_theta * x + sin_theta * z;
                float newz = -sin_theta * x + cos_theta * z;
                v3 tester = V(newx, y, newz);
                for (int c = 0; c < 3; c++) {
                    mn.e[c] = fminf(mn.e[c], tester.e[c]);
                    mx.e[c] = fmaxf(mx.e[c], tester.e[c]);
                }
            }
    return aabb_from_points(mn, mx);
}

static aabb_t prim_box(const world_t* w, o_object ref) {
    return ref.kind == O_OBJ_SPHERE ? w->spheres[ref.index].bbox : w->quads[ref.index].bbox;
}

static void inst_from_desc(const world_t* w, const o_instance* o, inst_t* in) {
    in->first = o->first; in->count = o->count; in->n_xf = o->n_xf;
    aabb_t b;
    if (o->flags & O_INST_LIST) {                          /* HittableList.add (objects.zig:273-276) */
        memset(&b, 0, sizeof b);                           /* Aabb{} = [0,0]^3 */
        for (uint32_t m = 0; m < o->count; m++) b = aabb_from_boxes(b, prim_box(w, w->desc.members[o->first + m]));
    } else {
        b = prim_box(w, w->desc.members[o->first]);
    }
    for (uint32_t k = 0; k < o->n_xf; k++) {
        xf_t* x = &in->xf[k];
        x->kind = o->xf[k].kind;
        if (x->kind == O_XF_TRANSLATE) {                   /* Translate.init (objects.zig:299-304) */
            x->offset = vload(o->xf[k].v);
            for (int c = 0; c < 3; c++) {                  /* Aabb.add / Interval.add */
                b.ax[c].min = b.ax[c].min + x->offset.e[c];
                b.ax[c].max = b.ax[c].max + x->offset.e[c];
            }
        } else {
            float radians = o->xf[k].v[0] * PI_F / 180.0f; /* degreesToRadians (rtweekend.zig:10-12) */
            x->sin_theta = sinf(radians);
            x->cos_theta = cosf(radians);
            b = rotate_y_box(b, x->sin_theta, x->cos_theta);
        }
    }
    in->bbox = b;
}

static int object_hit(const world_t* w, o_object ref, const ray3* r, interval_t ray_t, hit_record_t* rec,
                      const rng_t* rng);

/* HittableList.hit (objects.zig:281-289) */
static int list_hit(const world_t* w, const inst_t* in, const ray3* r, interval_t ray_t, hit_record_t* rec) {
    int any = 0;
    float closest_so_far = ray_t.max;
    for (uint32_t m = 0; m < in->count; m++) {
        hit_record_t h;
        interval_t it = {ray_t.min, closest_so_far};
        if (object_hit(w, w->desc.members[in->first + m], r, it, &h, NULL)) {
            closest_so_far = h.t;
            *rec = h;
            any = 1;
        }
    }
    return any;
}

/* the transform chain xf[k] .. xf[0] around the list (Translate.hit :314-330, RotateY.hit :398-442) */
static int inst_hit_k(const world_t* w, const inst_t* in, int k, const ray3* r, interval_t ray_t,
                      hit_record_t* rec) {
    if (k < 0) return list_hit(w, in, r, ray_t, rec);
    const xf_t* x = &in->xf[k];
    if (x->kind == O_XF_TRANSLATE) {
        ray3 moved = {sub(r->origin, x->offset), r->direction, r->time};
        if (!inst_hit_k(w, in, k - 1, &moved, ray_t, rec)) return 0;
        rec->p = add(rec->p, x->offset);
        return 1;
    }
    const float s = x->sin_theta, c = x->cos_theta;
    ray3 rot = *r;
    rot.origin.e[0] = c * r->origin.e[0] - s * r->origin.e[2];
    rot.origin.e[2] = s * r->origin.e[0] + c * r->origin.e[2];
    rot.direction.e[0] = c * r->direction.e[0] - s * r->direction.e[2];
    rot.direction.e[2] = s * r->direction.e[0] + c * r->direction.e[2];
    if (!inst_hit_k(w, in, k - 1, &rot, ray_t, rec)) return 0;
    v3 p = rec->p, n = rec->normal;
    p.e[0] = c * rec->p.e[0] + s * rec->p.e[2];
    p.e[2] = -s * rec->p.e[0] + c * rec->p.e[2];
    n.e[0] = c * rec->normal.e[0] + s * rec->normal.e[2];
    n.e[2] = -s * rec->normal.e[0] + c * rec->normal.e[2];
    rec->p = p;
    rec->normal = n;
    return 1;
}

/* ConstantMedium's one random draw, keyed: u = float(mix64(state ^ K*(medium+1))) */
float oracle_medium_draw(uint64_t path_state, uint32_t medium) {
    rng_t r;
    r.s = oracle_mix64(path_state ^ (0xD1B54A32D192ED03ull * (uint64_t)(medium + 1)));
    return rnd(&r);
}

/* ConstantMedium.hit (objects.zig:470-507) */
static int medium_hit(const world_t* w, uint32_t mi, const ray3* r, interval_t ray_t, hit_record_t* rec,
                      const rng_t* rng) {
    const medium_t* m = &w->media[mi];
    const interval_t universe = {-INF_F, INF_F};
    hit_record_t rec_1, rec_2;
    if (!object_hit(w, m->boundary, r, universe, &rec_1, NULL)) return 0;
    interval_t second = {rec_1.t + 0.0001f, INF_F};
    if (!object_hit(w, m->boundary, r, second, &rec_2, NULL)) return 0;
    if (rec_1.t < ray_t.min) rec_1.t = ray_t.min;
    if (rec_2.t > ray_t.max) rec_2.t = ray_t.max;
    if (rec_1.t >= rec_2.t) return 0;
    if (rec_1.t < 0) rec_1.t = 0;
    float ray_length = vlength(r->direction);
    float distance_inside_boundary = (rec_2.t - rec_1.t) * ray_length;
    float hit_distance = m->neg_inv_density * zig_logf(oracle_medium_draw(rng ? rng->s : 0, mi));
    if (hit_distance > distance_inside_boundary) return 0;
    rec->t = rec_1.t + hit_distance / ray_length;
    rec->p = ray_at(r, rec->t);
    rec->normal = V(1, 0, 0);          /* arbitrary */
    rec->front_face = 1;               /* also arbitrary */
    rec->mat = m->mat;
    rec->u = 0;
    rec->v = 0;
    return 1;
}

/* Hittable.hit dispatch (objects.zig:49-53) */
static int object_hit(const world_t* w, o_object ref, const ray3* r, interval_t ray_t, hit_record_t* rec,
                      const rng_t* rng) {
    switch (ref.kind) {
    case O_OBJ_SPHERE: return sphere_hit(&w->spheres[ref.index], r, ray_t, rec);
    case O_OBJ_QUAD: return quad_hit(&w->quads[ref.index], r, ray_t, rec);
    case O_OBJ_INSTANCE: {
        const inst_t* in = &w->insts[ref.index];
        return inst_hit_k(w, in, (int)in->n_xf - 1, r, ray_t, rec);
    }
    case O_OBJ_MEDIUM: return medium_hit(w, ref.index, r, ray_t, rec, rng);
    }
    return 0;
}

static aabb_t object_box(const world_t* w, o_object ref) {
    switch (ref.kind) {
    case O_OBJ_SPHERE: return w->spheres[ref.index].bbox;
    case O_OBJ_QUAD: return w->quads[ref.index].bbox;
    case O_OBJ_INSTANCE: return w->insts[ref.index].bbox;
    default: return w->media[ref.index].bbox;
    }
}

/* ------------------------------------------------------------------------- */
/* bvh.zig                                                                   */
/* ------------------------------------------------------------------------- */
static bvh_node_t* make_node(world_t* w) { return &w->pool[w->pool_used++]; }

/* bvh.zig:95-103 */
static int box_comparator(uint32_t axis, const object_t* a, const object_t* b) {
    uint32_t ax = axis == 0 ? 0 : (axis == 1 ? 1 : 2);
    return a->bbox.ax[ax].min < b->bbox.ax[ax].min;
}

/* Zig std.sort.heap (0.12): heapContext + siftDown */
static void sift_down(object_t* it, size_t a, size_t target, size_t b, uint32_t axis) {
    size_t cur = target;
    for (;;) {
        size_t child = (cur - a) * 2 + a + 1;
        if (!(child < b)) break;
        size_t next_child = child + 1;
        if (next_child < b && box_comparator(axis, &it[child], &it[next_child])) child = next_child;
        if (box_comparator(axis, &it[child], &it[cur])) break;
        object_t tmp = it[cur]; it[cur] = it[child]; it[child] = tmp;
        cur = child;
    }
}
static void heap_sort(object_t* it, size_t a, size_t b, uint32_t axis) {
    size_t i = a + (b - a) / 2;
    while (i > a) { i -= 1; sift_down(it, a, i, b, axis); }
    i = b;
    while (i > a) {
        i -= 1;
        object_t tmp = it[a]; it[a] = it[i]; it[i] = tmp;
        sift_down(it, a, a, i, axis);
    }
}

static bvh_node_t* make_leaf(world_t* w, const object_t* s) {  /* bvh.zig:82-89 */
    bvh_node_t* n = make_node(w);
    n->leaf = s; n->left = n->right = NULL; n->bbox = s->bbox;
    return n;
}

/* bvh.zig:43-71 */
static bvh_node_t* construct_tree(world_t* w, size_t start, size_t end) {
    const bvh_node_t *left, *right;
    size_t obj_span = end - start;
    uint32_t axis = rnd_int_range(&w->build_rng, 0, 2);
    w->axis_draws++;
    if (obj_span == 1) return make_leaf(w, &w->objects[start]);
    if (obj_span == 2) {
        if (box_comparator(axis, &w->objects[start], &w->objects[start + 1])) {
            left = make_leaf(w, &w->objects[start]);
            right = make_leaf(w, &w->objects[start + 1]);
        } else {
            left = make_leaf(w, &w->objects[start + 1]);
            right = make_leaf(w, &w->objects[start]);
        }
    } else {
        heap_sort(w->objects, start, end, axis);
        size_t mid = start + obj_span / 2;
        left = construct_tree(w, start, mid);
        right = construct_tree(w, mid, end);
    }
    bvh_node_t* n = make_node(w);                                 /* bvh.zig:73-80 */
    n->left = left; n->right = right; n->leaf = NULL;
    n->bbox = aabb_from_boxes(left->bbox, right->bbox);
    return n;
}

/* bvh.zig:122-136 */
static int bvh_hit(const world_t* w, const bvh_node_t* node, const ray3* r, interval_t ray_t, hit_record_t* rec,
                   const rng_t* rng) {
    if (node->leaf) {
        COUNT(leaves);
        o_object ref = {node->leaf->kind, node->leaf->index};
        return object_hit(w, ref, r, ray_t, rec, rng);
    }
    COUNT(nodes);
    if (!aabb_hit(&node->bbox, r, ray_t)) return 0;
    hit_record_t left_rec, right_rec;
    int hl = bvh_hit(w, node->left, r, ray_t, &left_rec, rng);
    interval_t r_int = {ray_t.min, hl ? left_rec.t : ray_t.max};
    int hr = bvh_hit(w, node->right, r, r_int, &right_rec, rng);
    if (hr) { *rec = right_rec; return 1; }
    if (hl) { *rec = left_rec; return 1; }
    return 0;
}

void* oracle_world_create(const o_scene_desc* d) {
    if (!d) return NULL;
    const uint32_t n_obj = d->objects ? d->n_objects : d->n_spheres;
    if (n_obj == 0) return NULL;
    world_t* w = (world_t*)calloc(1, sizeof(world_t));
    w->desc = *d;
    w->spheres = (sphere_t*)calloc(d->n_spheres ? d->n_spheres : 1, sizeof(sphere_t));
    for (uint32_t i = 0; i < d->n_spheres; i++) { sphere_from_desc(&d->spheres[i], &w->spheres[i]); w->spheres[i].orig = i; }
    w->quads = (quad_t*)calloc(d->n_quads ? d->n_quads : 1, sizeof(quad_t));
    for (uint32_t i = 0; i < d->n_quads; i++) quad_from_desc(&d->quads[i], &w->quads[i]);
    w->insts = (inst_t*)calloc(d->n_instances ? d->n_instances : 1, sizeof(inst_t));
    for (uint32_t i = 0; i < d->n_instances; i++) inst_from_desc(w, &d->instances[i], &w->insts[i]);
    w->media = (medium_t*)calloc(d->n_media ? d->n_media : 1, sizeof(medium_t));
    for (uint32_t i = 0; i < d->n_media; i++) {
        medium_t* m = &w->media[i];
        m->boundary = d->media[i].boundary;
        m->neg_inv_density = -1.0f / d->media[i].density;    /* objects.zig:451 */
        m->mat = d->media[i].material;
        m->bbox = object_box(w, m->boundary);
    }
    w->n = n_obj;
    w->objects = (object_t*)malloc(sizeof(object_t) * w->n);
    for (uint32_t i = 0; i < w->n; i++) {
        o_object ref = d->objects ? d->objects[i] : (o_object){O_OBJ_SPHERE, i};
        w->objects[i].kind = ref.kind;
        w->objects[i].index = ref.index;
        w->objects[i].orig = i;
        w->objects[i].bbox = object_box(w, ref);
    }
    w->pool_cap = 2 * w->n;
    w->pool = (bvh_node_t*)calloc(w->pool_cap, sizeof(bvh_node_t));
    w->build_rng = rng_stream(d->bvh_seed, 2, 0, 0);
    w->root = construct_tree(w, 0, w->n);
    return w;
}

void oracle_world_destroy(void* p) {
    world_t* w = (world_t*)p;
    if (!w) return;
    free(w->spheres); free(w->quads); free(w->insts); free(w->media);
    free(w->objects); free(w->pool); free(w);
}

static uint32_t tree_depth(const bvh_node_t* n) {
    if (!n || n->leaf) return 1;
    uint32_t a = tree_depth(n->left), b = tree_depth(n->right);
    return 1 + (a > b ? a : b);
}
int oracle_world_stats(void* p, uint32_t out[4]) {
    world_t* w = (world_t*)p;
    out[0] = w->pool_used; out[1] = w->n; out[2] = tree_depth(w->root); out[3] = w->axis_draws;
    return 0;
}

static uint32_t dump_rec(const world_t* w, const bvh_node_t* n, float* out, uint32_t* k, uint32_t cap) {
    uint32_t me = (*k)++;
    if (me < cap) {
        float* o = out + 8 * me;
        for (int i = 0; i < 3; i++) { o[i] = n->bbox.ax[i].min; o[3 + i] = n->bbox.ax[i].max; }
        o[6] = n->leaf ? (float)n->leaf->orig : -1.0f;
    }
    uint32_t size = 1;
    if (!n->leaf) {
        size += dump_rec(w, n->left, out, k, cap);
        size += dump_rec(w, n->right, out, k, cap);
    }
    if (me < cap) out[8 * me + 7] = (float)size;
    return size;
}
int oracle_world_dump(void* p, float* out, uint32_t cap) {
    world_t* w = (world_t*)p;
    uint32_t k = 0;
    dump_rec(w, w->root, out, &k, cap);
    return (int)k;
}

/* ------------------------------------------------------------------------- */
/* camera.zig                                                                */
/* ------------------------------------------------------------------------- */
static inline float degrees_to_radians(float deg) { return deg * PI_F / 180.0f; }  /* rtweekend.zig:10-12 */

int oracle_camera_init(const o_camera_params* p, o_camera* c) {       /* camera.zig:118-154 */
    memset(c, 0, sizeof *c);
    uint32_t H = p->image_height;
    if (H == 0) H = (uint32_t)roundf((float)p->image_width / p->aspect_ratio);
    if (H < 1) H = 1;
    uint32_t W = p->image_width;
    c->image_width = W; c->image_height = H; c->size = W * H;
    c->samples_per_pixel = p->samples_per_pixel; c->max_depth = p->max_depth;
    c->background_mode = p->background_mode; c->pixel_offset = p->pixel_offset;
    memcpy(c->background, p->background, 12);
    v3 lookfrom = vload(p->lookfrom), lookat = vload(p->lookat), vup = vload(p->vup);
    v3 center = lookfrom;
    float theta = degrees_to_radians(p->vfov);
    float h = tanf(theta / 2.0f);
    float viewport_height = 2 * h * p->focus_dist;
    float viewport_width = viewport_height * ((float)W / (float)H);
    v3 w = unit_vector(sub(lookfrom, lookat));
    v3 u = unit_vector(cross(vup, w));
    v3 v = cross(w, u);
    v3 viewport_u = mul(splat(viewport_width), u);
    v3 viewport_v = mul(splat(viewport_height), neg(v));
    v3 du = vdiv(viewport_u, splat((float)W));
    v3 dv = vdiv(viewport_v, splat((float)H));
    v3 upper_left = sub(sub(sub(center, mul(splat(p->focus_dist), w)), vdiv(viewport_u, splat(2.0f))),
                        vdiv(viewport_v, splat(2.0f)));
    v3 p00 = add(upper_left, mul(splat(0.5f), add(du, dv)));
    float defocus_radius = p->focus_dist * tanf(degrees_to_radians(p->defocus_angle / 2.0f));
    v3 ddu = mul(u, splat(defocus_radius));
    v3 ddv = mul(v, splat(defocus_radius));
    memcpy(c->center, center.e, 12); memcpy(c->pixel00_loc, p00.e, 12);
    memcpy(c->pixel_delta_u, du.e, 12); memcpy(c->pixel_delta_v, dv.e, 12);
    memcpy(c->u, u.e, 12); memcpy(c->v, v.e, 12); memcpy(c->w, w.e, 12);
    memcpy(c->defocus_disk_u, ddu.e, 12); memcpy(c->defocus_disk_v, ddv.e, 12);
    c->defocus_angle = p->defocus_angle;
    return 0;
}

/* camera.zig:169-180 (+ pixelSampleSquare 162-167, defocusDiskSample 156-160) */
static ray3 get_ray(const o_camera* c, uint32_t i, uint32_t j, rng_t* rng) {
    v3 p00 = vload(c->pixel00_loc), du = vload(c->pixel_delta_u), dv = vload(c->pixel_delta_v);
    v3 pixel_center = add(add(p00, mul(du, splat((float)i))), mul(dv, splat((float)j)));
    float px = -0.5f + rndp(rng);
    float py = -0.5f + rndp(rng);
    v3 square = add(mul(splat(px), du), mul(splat(py), dv));
    v3 pixel_sample = add(pixel_center, square);
    v3 origin;
    if (c->defocus_angle <= 0) {
        origin = vload(c->center);
    } else {
        v3 p = random_in_unit_disk(rng);
        origin = add(add(vload(c->center), mul(vload(c->defocus_disk_u), splat(p.e[0]))),
                     mul(vload(c->defocus_disk_v), splat(p.e[1])));
    }
    ray3 r;
    r.origin = origin;
    r.direction = sub(pixel_sample, origin);
    r.time = rndp(rng);
    return r;
}

static v3 background(const o_camera* c, const ray3* r) {
    if (c->background_mode == O_BG_GRADIENT) {              /* camera.zig:204-206 */
        v3 unit_direction = unit_vector(r->direction);
        float a = 0.5f * (unit_direction.e[1] + 1.0f);
        return add(mul(V(1, 1, 1), splat(1.0f - a)), mul(V(0.5f, 0.7f, 1.0f), splat(a)));
    }
    return vload(c->background);                            /* camera.zig:207 */
}

/* camera.zig:182-208 */
static v3 ray_color(const world_t* w, const o_camera* c, const ray3* r, uint32_t depth, rng_t* rng) {
    if (depth <= 0) return V(0, 0, 0);
    interval_t ray_t = {0.001f, INF_F};
    hit_record_t rec;
    COUNT(rays);
    if (bvh_hit(w, w->root, r, ray_t, &rec, rng)) {
        ray3 scattered;
        v3 attenuation = V(0, 0, 0);
        v3 color_from_emission = emitted(&w->desc, rec.mat, rec.u, rec.v, rec.p);
        if (scatter(&w->desc, r, &rec, &attenuation, &scattered, rng)) {
            v3 color_from_scatter = mul(attenuation, ray_color(w, c, &scattered, depth - 1, rng));
            return add(color_from_emission, color_from_scatter);
        }
        return color_from_emission;
    }
    return background(c, r);
}

static v3 sample_color(const world_t* w, const o_camera* c, uint64_t k0, uint32_t i, uint32_t s) {
    rng_t rng;
    rng.s = oracle_mix64(k0 ^ (((uint64_t)i << 32) | (uint64_t)s));
    uint32_t x = i % c->image_width + c->pixel_offset;       /* camera.zig:100-101 */
    uint32_t y = i / c->image_width + c->pixel_offset;
    ray3 r = get_ray(c, x, y, &rng);
    COUNT(samples);
    return ray_color(w, c, &r, c->max_depth, &rng);
}

void oracle_sample(void* p, const o_camera* c, uint64_t seed, uint32_t pixel, uint32_t sample, float out[3]) {
    v3 col = sample_color((const world_t*)p, c, oracle_mix64(seed), pixel, sample);
    memcpy(out, col.e, 12);
}

/* color.zig:43-62 toGamma2 + camera.zig:58-65 texel */
void oracle_gamma2(const float px[4], uint8_t out[4]) {
    float scale = 1.0f / px[3];
    interval_t intensity = {0, 0.999f};
    for (int k = 0; k < 3; k++) {
        float x = px[k] * scale;
        x = sqrtf(x);
        float g = 256 * clampi(intensity, x);
        out[k] = (uint8_t)g;
    }
    out[3] = 255;
}

/* camera.zig:54-66 */
static inline void write_color(float* buffer, uint8_t* texture, size_t i, v3 col, uint64_t n) {
    float* b = buffer + 4 * i;
    b[0] += col.e[0]; b[1] += col.e[1]; b[2] += col.e[2];
    b[3] = (float)n;
    if (texture) oracle_gamma2(b, texture + 4 * i);
}

/* camera.zig:93-116 */
int oracle_render_task(void* p, const o_camera* c, uint64_t seed, uint32_t thread_idx, uint32_t chunk_size,
                       float* buffer, uint8_t* texture) {
    const world_t* w = (const world_t*)p;
    uint64_t k0 = oracle_mix64(seed);
    size_t start_at = (size_t)thread_idx * chunk_size;
    size_t end_before = start_at + chunk_size;
    for (uint32_t n = 1; n < c->samples_per_pixel + 1; n++) {
        for (size_t i = start_at; i < end_before; i++) {
            v3 col = sample_color(w, c, k0, (uint32_t)i, n - 1);
            write_color(buffer, texture, i, col, n);
        }
    }
    counters_flush();
    return 0;
}

typedef struct {
    void* w; const o_camera* c; uint64_t seed; uint32_t tid, chunk; float* buf; uint8_t* tex;
    const uint32_t* pix; uint32_t n, s0, s1;
} task_arg_t;

static void* task_thread(void* a) {
    task_arg_t* t = (task_arg_t*)a;
    oracle_render_task(t->w, t->c, t->seed, t->tid, t->chunk, t->buf, t->tex);
    return NULL;
}

/* main.zig:314-326 */
int oracle_render_threads(void* w, const o_camera* c, uint64_t seed, uint32_t n_threads,
                          float* buffer, uint8_t* texture) {
    if (n_threads < 1) n_threads = 1;
    uint32_t chunk = c->size / n_threads;
    pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * n_threads);
    task_arg_t* args = (task_arg_t*)calloc(n_threads, sizeof(task_arg_t));
    for (uint32_t t = 0; t < n_threads; t++) {
        args[t].w = w; args[t].c = c; args[t].seed = seed; args[t].tid = t; args[t].chunk = chunk;
        args[t].buf = buffer; args[t].tex = texture;
        pthread_create(&th[t], NULL, task_thread, &args[t]);
    }
    for (uint32_t t = 0; t < n_threads; t++) pthread_join(th[t], NULL);
    free(th); free(args);
    return 0;
}

static void* pixels_thread(void* a) {
    task_arg_t* t = (task_arg_t*)a;
    const world_t* w = (const world_t*)t->w;
    uint64_t k0 = oracle_mix64(t->seed);
    for (uint32_t s = t->s0; s < t->s1; s++) {                 /* samples outer */
        for (uint32_t k = 0; k < t->n; k++) {                   /* pixels inner */
            v3 col = sample_color(w, t->c, k0, t->pix[k], s);
            float* b = t->buf + 4 * (size_t)k;
            b[0] += col.e[0]; b[1] += col.e[1]; b[2] += col.e[2];
            b[3] = (float)(s + 1);
        }
    }
    counters_flush();
    return NULL;
}

int oracle_render_pixels(void* w, const o_camera* c, uint64_t seed, const uint32_t* pix, uint32_t n,
                         uint32_t spp_begin, uint32_t spp_end, float* out4, uint32_t n_threads) {
    if (n_threads < 1) n_threads = 1;
    if (n_threads > n) n_threads = n ? n : 1;
    pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * n_threads);
    task_arg_t* args = (task_arg_t*)calloc(n_threads, sizeof(task_arg_t));
    uint32_t base = 0;
    for (uint32_t t = 0; t < n_threads; t++) {
        uint32_t cnt = n / n_threads + (t < n % n_threads ? 1 : 0);
        args[t].w = w; args[t].c = c; args[t].seed = seed; args[t].pix = pix + base; args[t].n = cnt;
        args[t].buf = out4 + 4 * (size_t)base; args[t].s0 = spp_begin; args[t].s1 = spp_end;
        base += cnt;
        pthread_create(&th[t], NULL, pixels_thread, &args[t]);
    }
    for (uint32_t t = 0; t < n_threads; t++) pthread_join(th[t], NULL);
    free(th); free(args);
    return 0;
}

/* ------------------------------------------------------------------------- */
/* main.zig:253-312 generateWorld restated on the seeded scene stream.       */
/* variant 0 = "book1" (static spheres, solid grey ground, brown sphere),    */
/* variant 1 = "ref_head" (HEAD: checker ground, moving diffuse spheres,     */
/* earth image texture on the (-4,1,0) sphere, image index 0).               */
/* ------------------------------------------------------------------------- */
typedef struct {
    o_sphere* sp; o_material* mt; o_texture* tx; uint32_t cap, ns, nm, nt; int overflow;
} scene_out_t;

static uint32_t add_tex_solid(scene_out_t* o, v3 c) {
    if (o->nt >= o->cap) { o->overflow = 1; return 0; }
    o_texture* t = &o->tx[o->nt]; memset(t, 0, sizeof *t);
    t->kind = O_TEX_SOLID; memcpy(t->even, c.e, 12);
    return o->nt++;
}
static uint32_t add_mat(scene_out_t* o, uint32_t kind, uint32_t tex, v3 albedo, float fuzz, float ir) {
    if (o->nm >= o->cap) { o->overflow = 1; return 0; }
    o_material* m = &o->mt[o->nm]; memset(m, 0, sizeof *m);
    m->kind = kind; m->texture = tex; memcpy(m->albedo, albedo.e, 12); m->fuzz = fuzz; m->ir = ir;
    return o->nm++;
}
static void add_sphere(scene_out_t* o, v3 c1, float r, uint32_t mat, int moving, v3 c2) {
    if (o->ns >= o->cap) { o->overflow = 1; return; }
    o_sphere* s = &o->sp[o->ns++]; memset(s, 0, sizeof *s);
    memcpy(s->center1, c1.e, 12); s->radius = r; s->material = mat;
    if (moving) { memcpy(s->center2, c2.e, 12); s->is_moving = 1; }
}

int oracle_gen_book1(uint64_t seed, uint32_t variant, o_sphere* sp, o_material* mt, o_texture* tx,
                     uint32_t cap, uint32_t counts[3]) {
    scene_out_t o = {sp, mt, tx, cap, 0, 0, 0, 0};
    rng_t r = rng_stream(seed, 1, 0, 0);
    v3 zero = V(0, 0, 0);
    uint32_t gm;
    if (variant == 1) {
        if (o.nt >= cap) return -1;
        o_texture* t = &o.tx[o.nt]; memset(t, 0, sizeof *t);
        t->kind = O_TEX_CHECKER; t->scale = 1.0f / 0.32f;
        t->even[0] = 0.2f; t->even[1] = 0.3f; t->even[2] = 0.1f;
        t->odd[0] = 0.9f; t->odd[1] = 0.9f; t->odd[2] = 0.9f;
        gm = add_mat(&o, O_MAT_LAMBERTIAN, o.nt++, zero, 0, 0);
    } else {
        gm = add_mat(&o, O_MAT_LAMBERTIAN, add_tex_solid(&o, V(0.5f, 0.5f, 0.5f)), zero, 0, 0);
    }
    add_sphere(&o, V(0, -1000, 0), 1000, gm, 0, zero);
    for (float a = -11; a < 11; a += 1) {
        for (float b = -11; b < 11; b += 1) {
            float choose_mat = rnd(&r);
            float cx = a + 0.9f * rnd(&r);
            float cz = b + 0.9f * rnd(&r);
            v3 center = V(cx, 0.4f * choose_mat, cz);
            if (vlength(sub(center, V(4, 0.2f, 0))) > 0.9f) {
                if (choose_mat < 0.8f) {
                    v3 r1 = random_v(&r);
                    v3 r2 = random_v(&r);
                    v3 albedo = mul(r1, r2);
                    uint32_t m = add_mat(&o, O_MAT_LAMBERTIAN, add_tex_solid(&o, albedo), zero, 0, 0);
                    if (variant == 1) {
                        float d0 = rnd_range(&r, 0, 0.5f), d1 = rnd_range(&r, 0, 0.5f), d2 = rnd_range(&r, 0, 0.5f);
                        v3 center2 = add(center, V(d0, d1, d2));
                        add_sphere(&o, center, 0.4f * choose_mat, m, 1, center2);
                    } else {
                        add_sphere(&o, center, 0.4f * choose_mat, m, 0, zero);
                    }
                } else if (choose_mat < 0.95f) {
                    v3 albedo = random_range_v(&r, 0.5f, 1);
                    float fuzz = rnd_range(&r, 0, 0.5f);
                    uint32_t m = add_mat(&o, O_MAT_METAL, 0, albedo, fuzz < 1 ? fuzz : 1, 0);
                    add_sphere(&o, center, 0.5f * choose_mat, m, 0, zero);
                } else {
                    float ir = rnd_range(&r, 1, 2);
                    uint32_t m = add_mat(&o, O_MAT_DIELECTRIC, 0, zero, 0, ir);
                    add_sphere(&o, center, 0.3f * choose_mat, m, 0, zero);
                }
            }
        }
    }
    add_sphere(&o, V(0, 1, 0), 1.0f, add_mat(&o, O_MAT_DIELECTRIC, 0, zero, 0, 1.5f), 0, zero);
    if (variant == 1) {
        if (o.nt >= cap) return -1;
        o_texture* t = &o.tx[o.nt]; memset(t, 0, sizeof *t);
        t->kind = O_TEX_IMAGE; t->image = 0;
        add_sphere(&o, V(-4, 1, 0), 1.0f, add_mat(&o, O_MAT_LAMBERTIAN, o.nt++, zero, 0, 0), 0, zero);
    } else {
        add_sphere(&o, V(-4, 1, 0), 1.0f,
                   add_mat(&o, O_MAT_LAMBERTIAN, add_tex_solid(&o, V(0.4f, 0.2f, 0.1f)), zero, 0, 0), 0, zero);
    }
    add_sphere(&o, V(4, 1, 0), 1.0f, add_mat(&o, O_MAT_METAL, 0, V(0.7f, 0.6f, 0.5f), 0.1f, 0), 0, zero);
    counts[0] = o.ns; counts[1] = o.nm; counts[2] = o.nt;
    return o.overflow ? -1 : 0;
}
