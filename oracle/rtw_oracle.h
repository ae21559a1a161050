/*
 * rtw_oracle.h -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of dariooddenino/zig-raytracing-weekend's per-pixel sample loop
 * (src/camera.zig:93-208 -> bvh.zig -> aabb.zig -> objects.zig -> material.zig ->
 * textures.zig / perlin.zig / rtw_image.zig).  It is the parity checker for the
 * HIP path and the timed CPU baseline of bench.py ("cpu_baseline.kind": "port").
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it.
 * The product (zig-raytracing-weekend_amd/) never links, includes or calls it.
 *
 * Parity pinning: reference aabb test cases (src/aabb.zig:117-136), sphere-UV
 * table (src/objects.zig:105-107), the golden sky rows of the reference's own
 * image.ppm / image2.ppm (±1 LSB), and the stb_image decode hash of
 * content/earthmap.jpg.  The Zig reference cannot be built here (no Zig
 * toolchain, Dawn fetched by URL, RoundBox.hit incomplete) and its RNG is the
 * unseedable std.crypto.random, so the RNG is replaced by the counter-based
 * stream documented in DESIGN.md §RNG (same definition, restated independently
 * in the HIP kernel).
 *
 * Wire layouts below are the neutral scene-description records of
 * include/rtw_gpu.h (same sizes and field order); they are restated here so the
 * oracle does not include product headers.
 */
#ifndef RTW_ORACLE_H
#define RTW_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct o_sphere {           /* 48 B */
    float center1[3];
    float radius;
    float center2[3];               /* initMoving's second centre (objects.zig:87-92) */
    uint32_t is_moving;
    uint32_t material;
    uint32_t _pad[3];
} o_sphere;

enum { O_MAT_LAMBERTIAN = 0, O_MAT_METAL = 1, O_MAT_DIELECTRIC = 2,
       O_MAT_DIFFUSE_LIGHT = 3, O_MAT_ISOTROPIC = 4 };
typedef struct o_material {         /* 32 B */
    uint32_t kind;
    uint32_t texture;
    float fuzz;
    float ir;
    float albedo[3];
    float _pad;
} o_material;

enum { O_TEX_SOLID = 0, O_TEX_CHECKER = 1, O_TEX_IMAGE = 2, O_TEX_NOISE = 3 };
typedef struct o_texture {          /* 48 B */
    uint32_t kind;
    uint32_t image;
    uint32_t perlin;
    float scale;                    /* checker: inv_scale; noise: scale */
    float even[3];                  /* solid: color_value */
    float _p0;
    float odd[3];
    float _p1;
} o_texture;

typedef struct o_image {
    const uint8_t* data;            /* RGBA8 (stb forced 4 comps) */
    uint32_t width, height, bytes_per_row, _pad;
} o_image;

typedef struct o_perlin {           /* 4608 B */
    float ranvec[256][3];
    uint16_t perm_x[256], perm_y[256], perm_z[256];
} o_perlin;

typedef struct o_quad {             /* 48 B: Quad.init(q, u, v, mat) (objects.zig:201-210) */
    float q[3];
    uint32_t material;
    float u[3];
    uint32_t _p0;
    float v[3];
    uint32_t _p1;
} o_quad;

enum { O_OBJ_SPHERE = 0, O_OBJ_QUAD = 1, O_OBJ_INSTANCE = 2, O_OBJ_MEDIUM = 3 };
typedef struct o_object { uint32_t kind, index; } o_object;

enum { O_XF_TRANSLATE = 0, O_XF_ROTATE_Y = 1 };
typedef struct o_transform { uint32_t kind; float v[3]; } o_transform;

#define O_MAX_XF 3
enum { O_INST_LIST = 1u };
typedef struct o_instance {         /* 64 B: xf[0] innermost .. xf[n_xf-1] outermost */
    uint32_t first, count, n_xf, flags;
    o_transform xf[O_MAX_XF];
} o_instance;

typedef struct o_medium {           /* 16 B: ConstantMedium (objects.zig:445-460) */
    o_object boundary;
    float density;
    uint32_t material;              /* the Isotropic phase function */
} o_medium;

typedef struct o_scene_desc {
    const o_sphere* spheres;   uint32_t n_spheres;
    const o_material* materials; uint32_t n_materials;
    const o_texture* textures; uint32_t n_textures;
    const o_image* images;     uint32_t n_images;
    const o_perlin* perlins;   uint32_t n_perlins;
    uint64_t bvh_seed;
    uint32_t bvh_mode;              /* ignored: the oracle always builds the reference topology */
    float order_dir[3];
    const o_quad* quads;       uint32_t n_quads;
    const o_object* members;   uint32_t n_members;
    const o_instance* instances; uint32_t n_instances;
    const o_medium* media;     uint32_t n_media;
    const o_object* objects;   uint32_t n_objects;  /* world_objects; NULL = every sphere */
} o_scene_desc;

enum { O_BG_CONSTANT = 0, O_BG_GRADIENT = 1 };
typedef struct o_camera_params {
    float aspect_ratio;
    uint32_t image_width;
    uint32_t image_height;          /* 0 -> derived from aspect (camera.zig:119-121) */
    uint32_t samples_per_pixel;
    uint32_t max_depth;
    uint32_t background_mode;
    float background[3];
    float vfov;
    float lookfrom[3];
    float lookat[3];
    float vup[3];
    float defocus_angle;
    float focus_dist;
    uint32_t pixel_offset;          /* +1 quirk of camera.zig:100-101 */
} o_camera_params;

typedef struct o_camera {
    uint32_t image_width, image_height, size, samples_per_pixel, max_depth;
    uint32_t background_mode, pixel_offset, _pad;
    float center[3], pixel00_loc[3], pixel_delta_u[3], pixel_delta_v[3];
    float u[3], v[3], w[3];
    float defocus_disk_u[3], defocus_disk_v[3];
    float defocus_angle;
    float background[3];
} o_camera;

/* RNG */
uint64_t oracle_mix64(uint64_t z);
void oracle_rng_floats(uint64_t seed, uint64_t domain, uint32_t a, uint32_t b, uint32_t n, float* out);
void oracle_rng_u64(uint64_t seed, uint64_t domain, uint32_t a, uint32_t b, uint32_t n, uint64_t* out);
/* render-domain draws of path (a = pixel, b = sample): rtw_rng.h rtw_path_float */
void oracle_path_floats(uint64_t seed, uint32_t a, uint32_t b, uint32_t n, float* out);

/* Known-answer hooks */
int oracle_aabb_hit(const float box[6], const float origin[3], const float dir[3], float tmin, float tmax);
void oracle_sphere_uv(const float p[3], float uv[2]);
void oracle_libm(int fn, const float* a, const float* b, float* out, uint64_t n);
float oracle_pow(float x, float y);
void oracle_reflect(const float v[3], const float n[3], float out[3]);
void oracle_refract(const float uv[3], const float n[3], float e, float out[3]);
float oracle_reflectance(float cosine, float ref_idx);
int oracle_sphere_hit(const o_sphere* s, const float origin[3], const float dir[3], float time,
                      float tmin, float tmax, float out[8]); /* t,p3,n3,front */
void oracle_texture_value(const o_scene_desc* d, uint32_t tex, float u, float v, const float p[3], float out[3]);
float oracle_perlin_noise(const o_perlin* pl, const float p[3]);
float oracle_perlin_turb(const o_perlin* pl, const float p[3], int depth);
void oracle_gamma2(const float px[4], uint8_t out[4]);

/* Scenes (src/main.zig builders restated with the seeded stream) */
int oracle_gen_perlin(uint64_t seed, uint32_t id, o_perlin* out);
int oracle_gen_book1(uint64_t seed, uint32_t variant, o_sphere* sp, o_material* mt, o_texture* tx,
                     uint32_t cap, uint32_t counts[3]);

/* Camera.init (camera.zig:118-154) */
int oracle_camera_init(const o_camera_params* p, o_camera* c);

/* Quad.hit (objects.zig:222-255): out t, p3, n3, front, u, v */
int oracle_quad_hit(const o_quad* q, const float origin[3], const float dir[3], float tmin, float tmax,
                    float out[10]);
/* the keyed draw of ConstantMedium.hit (domain "medium") */
float oracle_medium_draw(uint64_t path_state, uint32_t medium);

/* World = BVHTree over world_objects (bvh.zig:22-104) */
void* oracle_world_create(const o_scene_desc* d);
void oracle_world_destroy(void* w);
int oracle_world_stats(void* w, uint32_t out[4]); /* nodes, leaves, depth, axis draws */
/* preorder dump of the pointer tree: per node 8 floats (box min3,max3, leaf object idx or -1, subtree size);
 * the leaf index is the position in world_objects (= sphere index when objects is NULL) */
int oracle_world_dump(void* w, float* out, uint32_t cap);

/* Hot loop.  Camera.render (camera.zig:93-116) for one Task: samples outer,
 * pixels inner over [thread_idx*chunk, (thread_idx+1)*chunk). buffer: float4 per
 * pixel (camera.zig:21-66), texture: u8x4 per pixel (may be NULL). */
int oracle_render_task(void* w, const o_camera* c, uint64_t seed, uint32_t thread_idx, uint32_t chunk_size,
                       float* buffer, uint8_t* texture);
/* startRender (main.zig:314-326): n_threads workers, chunk = size / n_threads */
int oracle_render_threads(void* w, const o_camera* c, uint64_t seed, uint32_t n_threads,
                          float* buffer, uint8_t* texture);
/* Arbitrary pixel subset, samples [spp_begin, spp_end) (0-based sample index),
 * same per-pixel arithmetic; writes float4 accumulators (rgb += , w = spp_end).
 * n_threads > 1 splits the pixel list into contiguous chunks. */
int oracle_render_pixels(void* w, const o_camera* c, uint64_t seed, const uint32_t* pix, uint32_t n,
                         uint32_t spp_begin, uint32_t spp_end, float* out4, uint32_t n_threads);
/* One sample's radiance */
void oracle_sample(void* w, const o_camera* c, uint64_t seed, uint32_t pixel, uint32_t sample, float out[3]);

/* Instrumentation for algorithmic bytes */
void oracle_counters_enable(int on);
void oracle_counters_reset(void);
/* rays, inner nodes visited (box tests), leaves/spheres tested, texel fetches, noise evals, samples */
void oracle_counters_get(uint64_t out[6]);

#ifdef __cplusplus
}
#endif
#endif
