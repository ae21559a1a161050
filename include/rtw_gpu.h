/*
 * rtw_gpu.h -- C ABI of the MI355X-native path-tracing hot path.
 *
 * Drop-in boundary for dariooddenino/zig-raytracing-weekend's per-pixel sample
 * loop.  The reference's only entry point into the loop is
 *
 *     pub fn render(self: *Camera, raytrace: *RayTraceState, context: Task) !void
 *                                                        (src/camera.zig:93)
 *
 * called by RenderThread.renderFn (src/main.zig:66-68) for each of 8 Tasks
 * spawned by startRender (src/main.zig:314-326).  It reads the Camera fields
 * derived by Camera.init (src/camera.zig:118-154), the world (a BVHTree of
 * Spheres, src/bvh.zig:17-104, src/objects.zig:68-148), and writes the
 * SharedStateImageWriter float4 buffer (src/camera.zig:21-66).  The entry
 * points below replace exactly that: a host (Zig via @cImport, C++, or Python
 * via ctypes) describes the scene once (rtw_scene_create, replaces the
 * pointer graph of Hittable/Material/Texture unions), derives the camera
 * (rtw_camera_init, replaces Camera.init) and calls rtw_render for a pixel
 * range and a sample range (replaces Camera.render for one Task).
 *
 * Plain C types only; no HIP or torch types cross the boundary (streams and
 * device buffers are passed as void*).  Every function returns an RTW_* status;
 * rtw_last_error() returns a thread-local message for the last failure.
 * No exceptions cross the ABI.  The library never frees caller memory.
 *
 * Threading: render calls on one rtw_ctx may come from several threads at once
 * (the reference's 8 RenderThreads, src/main.zig:314-326): they are serialised
 * per context, and a device-API call on another stream than the previous call
 * waits for that call's work on the device.  rtw_scene_destroy must not race a
 * render on the same context.
 */
#ifndef RTW_GPU_H
#define RTW_GPU_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RTW_ABI_VERSION 8

enum rtw_status {
    RTW_OK = 0,
    RTW_E_INVALID = -1,     /* bad argument / inconsistent scene */
    RTW_E_HIP = -2,         /* HIP runtime error (message in rtw_last_error) */
    RTW_E_OOM = -3,         /* device or host allocation failed */
    RTW_E_CANCELLED = -4,   /* cancel flag observed between sample batches */
    RTW_E_NODEVICE = -5     /* no gfx950 device visible */
};

/* ---------------------------------------------------------------------------
 * Scene description (host memory, caller-owned, read once by rtw_scene_create)
 * ------------------------------------------------------------------------- */

/* Sphere.init / Sphere.initMoving (src/objects.zig:80-92).  48 bytes. */
typedef struct rtw_sphere {
    float center1[3];
    float radius;
    float center2[3];          /* used iff is_moving: center_vec = center2 - center1 */
    uint32_t is_moving;
    uint32_t material;         /* index into materials[] */
    uint32_t _pad[3];
} rtw_sphere;

/* Material union (src/material.zig:11-144).  32 bytes. */
enum rtw_material_kind {
    RTW_MAT_LAMBERTIAN = 0,    /* albedo = textures[texture] */
    RTW_MAT_METAL = 1,         /* albedo[3], fuzz (already clamped <= 1 as Metal.fromColor does) */
    RTW_MAT_DIELECTRIC = 2,    /* ir */
    RTW_MAT_DIFFUSE_LIGHT = 3, /* emit = textures[texture] */
    RTW_MAT_ISOTROPIC = 4      /* albedo = textures[texture] (needs ConstantMedium; not in the sphere path) */
};
typedef struct rtw_material {
    uint32_t kind;
    uint32_t texture;
    float fuzz;
    float ir;
    float albedo[3];
    float _pad;
} rtw_material;

/* Texture union (src/textures.zig:10-124).  48 bytes. */
enum rtw_texture_kind {
    RTW_TEX_SOLID = 0,         /* even[] = color_value */
    RTW_TEX_CHECKER = 1,       /* scale = inv_scale, even[], odd[] */
    RTW_TEX_IMAGE = 2,         /* image = index into images[] */
    RTW_TEX_NOISE = 3          /* perlin = index into perlins[], scale */
};
typedef struct rtw_texture {
    uint32_t kind;
    uint32_t image;
    uint32_t perlin;
    float scale;
    float even[3];
    float _p0;
    float odd[3];
    float _p1;
} rtw_texture;

/* zstbi.Image as used by RtwImage (src/rtw_image.zig:5-62): RGBA8, 4 B/texel. */
typedef struct rtw_image {
    const uint8_t* data;
    uint32_t width, height, bytes_per_row, _pad;
} rtw_image;

/* Perlin tables (src/perlin.zig:76-101).  4608 bytes. */
typedef struct rtw_perlin {
    float ranvec[256][3];
    uint16_t perm_x[256], perm_y[256], perm_z[256];
} rtw_perlin;

/* Quad.init (src/objects.zig:193-210): corner q, edges u, v.  The library derives
 * normal = unitVector(cross(u, v)), d = dot(normal, q), w = n / dot(n, n) and the
 * box fromPoints(q, q + u + v).pad() exactly as Quad.init does.  48 bytes. */
typedef struct rtw_quad {
    float q[3];
    uint32_t material;
    float u[3];
    uint32_t _p0;
    float v[3];
    uint32_t _p1;
} rtw_quad;

/* A Hittable (src/objects.zig:39-48) by kind + index into its array. */
enum rtw_object_kind {
    RTW_OBJ_SPHERE = 0,        /* spheres[index] */
    RTW_OBJ_QUAD = 1,          /* quads[index] */
    RTW_OBJ_INSTANCE = 2,      /* instances[index] */
    RTW_OBJ_MEDIUM = 3         /* media[index] */
};
typedef struct rtw_object {
    uint32_t kind;
    uint32_t index;
} rtw_object;

/* Translate / RotateY (src/objects.zig:292-443). */
enum rtw_transform_kind {
    RTW_XF_TRANSLATE = 0,      /* v = offset */
    RTW_XF_ROTATE_Y = 1        /* v[0] = angle in degrees (sin/cos as RotateY.init) */
};
typedef struct rtw_transform {
    uint32_t kind;
    float v[3];
} rtw_transform;

#define RTW_MAX_XF 3
enum { RTW_INST_LIST = 1u };   /* rtw_instance.flags: the members form a HittableList (its box
                                  starts from the zero Aabb{}, objects.zig:264-279); else one primitive */
/* A HittableList (createBox, src/objects.zig:264-290, 510-532) of members[first ..
 * first + count) -- spheres or quads -- wrapped in xf[0] (innermost) .. xf[n_xf-1]
 * (outermost), e.g. Translate(RotateY(createBox(...))) = {ROTATE_Y, TRANSLATE}.  64 bytes. */
typedef struct rtw_instance {
    uint32_t first, count, n_xf, flags;
    rtw_transform xf[RTW_MAX_XF];
} rtw_instance;

/* ConstantMedium.initFromColor/initFromTexture (src/objects.zig:445-460): boundary is
 * a sphere, quad or instance; material = the Isotropic phase function
 * (RTW_MAT_ISOTROPIC).  The one random draw of ConstantMedium.hit (objects.zig:484)
 * is keyed by (path RNG state at the traversal, medium index), not taken from the
 * path's sequential stream, so the result does not depend on the BVH topology. */
typedef struct rtw_medium {
    rtw_object boundary;
    float density;
    uint32_t material;
} rtw_medium;

enum rtw_bvh_mode {
    RTW_BVH_REFERENCE = 0,     /* BVHTree.constructTree (src/bvh.zig:43-71): random axis from the
                                  seeded build stream, std.sort.heap by box min, median split */
    RTW_BVH_SAH = 1            /* binned SAH, single-sphere leaves, children ordered front-to-back
                                  along order_dir.  Same closest hit (topology-independent). */
};

typedef struct rtw_scene_desc {
    const rtw_sphere* spheres;     uint32_t n_spheres;
    const rtw_material* materials; uint32_t n_materials;
    const rtw_texture* textures;   uint32_t n_textures;
    const rtw_image* images;       uint32_t n_images;
    const rtw_perlin* perlins;     uint32_t n_perlins;
    uint64_t bvh_seed;
    uint32_t bvh_mode;
    float order_dir[3];        /* RTW_BVH_SAH child order hint (e.g. camera forward); 0 = (0,-1,0) */
    /* ABI 2: the rest of the Hittable union.  objects = world_objects in order (the
     * BVH leaves); NULL/0 = every sphere in order (ABI 1 behaviour). */
    const rtw_quad* quads;         uint32_t n_quads;
    const rtw_object* members;     uint32_t n_members;     /* instance list entries: spheres/quads */
    const rtw_instance* instances; uint32_t n_instances;
    const rtw_medium* media;       uint32_t n_media;
    const rtw_object* objects;     uint32_t n_objects;
} rtw_scene_desc;

/* ---------------------------------------------------------------------------
 * Camera (src/camera.zig:69-91 fields; rtw_camera_init restates Camera.init)
 * ------------------------------------------------------------------------- */
enum rtw_background_mode {
    RTW_BG_CONSTANT = 0,       /* Camera.background (camera.zig:80, 207); HEAD default black */
    RTW_BG_GRADIENT = 1        /* Book-1 sky, the commented camera.zig:204-206 */
};

typedef struct rtw_camera_params {
    float aspect_ratio;
    uint32_t image_width;
    uint32_t image_height;     /* 0 -> round(width / aspect) (camera.zig:119-121) */
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
    uint32_t pixel_offset;     /* 1 reproduces camera.zig:100-101 (x = i%W + 1, y = i/W + 1) */
} rtw_camera_params;

typedef struct rtw_camera {
    uint32_t image_width, image_height, size, samples_per_pixel, max_depth;
    uint32_t background_mode, pixel_offset, _pad;
    float center[3], pixel00_loc[3], pixel_delta_u[3], pixel_delta_v[3];
    float u[3], v[3], w[3];
    float defocus_disk_u[3], defocus_disk_v[3];
    float defocus_angle;
    float background[3];
} rtw_camera;

/* ---------------------------------------------------------------------------
 * Entry points
 * ------------------------------------------------------------------------- */
typedef struct rtw_ctx rtw_ctx;

/* Progress callback: samples (pixel x spp) finished so far in this call.
 * Return non-zero to cancel (like RenderThread.stop, src/main.zig:58-60). */
typedef int (*rtw_progress_fn)(uint64_t samples_done, uint64_t samples_total, void* user);

/* Device time per kernel kind of one render call (rtw_render_opts.timing). */
enum { RTW_K_GEN = 0, RTW_K_TRACE = 1, RTW_K_SHADE = 2, RTW_K_TAIL = 3, RTW_K_REDUCE = 4, RTW_K_MEGA = 5,
       RTW_K_COUNT = 8 };
typedef struct rtw_kernel_timing {
    float ms[RTW_K_COUNT];         /* summed HIP-event time of the launches of each kind */
    uint32_t launches[RTW_K_COUNT];
} rtw_kernel_timing;

typedef struct rtw_render_opts {
    uint32_t spp_batch;        /* samples per kernel launch (cancel/progress granularity); 0 = auto */
    uint32_t flags;            /* RTW_RENDER_* */
    uint64_t* counters;        /* optional device-side stats out (RTW_STAT_COUNT u64) or NULL */
    rtw_kernel_timing* timing; /* optional host out: per-kernel device time (the call then synchronises) */
    /* ABI 5: stop and progress, polled before every spp batch and after each one (a call given any of
     * them synchronises after every batch).  Samples of the batches that finished stay in the buffer
     * and its .w is the last finished batch's end (camera.zig:56), so a stopped render can resume. */
    const volatile uint8_t* running; /* RenderThread.running (src/main.zig:50, a Zig `bool`; stop() clears
                                        it, main.zig:58-60; Camera.render polls it, camera.zig:107):
                                        0 = stop, non-zero = go on; NULL = not polled */
    const volatile int32_t* cancel;  /* non-zero = stop (rtw_render's flag); NULL = not polled */
    rtw_progress_fn progress;        /* samples finished so far in this call; non-zero return = stop */
    void* user;                      /* passed to progress */
} rtw_render_opts;

enum { RTW_RENDER_NO_SYNC = 1u };  /* rtw_render_device: do not synchronise the stream */
enum { RTW_STAT_RAYS = 0, RTW_STAT_NODES = 1, RTW_STAT_LEAVES = 2, RTW_STAT_SAMPLES = 3, RTW_STAT_NAN = 4,
       RTW_STAT_TAIL_RAYS = 5, /* rays traced by the wavefront tail kernel (subset of RAYS) */
       RTW_STAT_COUNT = 8 };

int rtw_version(void);
/* ABI 6: the library's build id, the first 16 hex digits of the sha256 of its sources (csrc/Makefile);
 * PMC passes under profiles/ record it, and bench.py derives no roofline from a pass of another build. */
const char* rtw_build_id(void);
const char* rtw_last_error(void);
int rtw_device_count(int* out);

/* Camera.init (src/camera.zig:118-154). Host-only arithmetic; shared by every caller. */
int rtw_camera_init(const rtw_camera_params* params, rtw_camera* out);

/* Builds the BVH (bvh_mode) on the host, flattens it to 32-byte depth-first
 * nodes with skip links, and uploads nodes / materials / textures / images /
 * perlin tables to `device`.  Replaces generateWorld's BVHTree.init
 * (src/main.zig:309, src/bvh.zig:22-29).
 * device = RTW_DEVICE_CPU makes a HOST context (no GPU needed): rtw_render on it runs the
 * same per-sample code as the GPU on host threads (bit-identical images); the device-buffer
 * and multi-GPU entry points refuse it (RTW_E_INVALID). */
#define RTW_DEVICE_CPU (-1)
int rtw_scene_create(const rtw_scene_desc* desc, int device, rtw_ctx** out);

/* Implementation choices of a context (ABI 3).  Every setting renders the SAME image,
 * bit for bit (each one is a different schedule of the same fp32
 * operations); they exist for A/B measurement and the invariance tests.  Start from
 * rtw_tuning_defaults() -- the product defaults -- and change fields. */
enum rtw_kernel_kind {
    RTW_KERNEL_WAVEFRONT = 0,  /* wavefront path tracer (rtw_wavefront.hip), the product path */
    RTW_KERNEL_PERSISTENT = 1, /* persistent megakernel (render_persistent_v1), a baseline */
    RTW_KERNEL_SIMPLE = 2      /* one lane per pixel (render_pixels_v0), a baseline */
};
enum {  /* rtw_tuning.lds: what the kernels may stage in LDS when it fits */
    RTW_LDS_NODES = 1u,        /* the 32-B node array (wavefront trace / fused step / tail) */
    RTW_LDS_CNODES = 2u,       /* the compact nodes of every octant copy (small static sphere SAH trees) */
    RTW_LDS_MATERIALS = 4u,    /* materials beside the compact nodes */
    RTW_LDS_SHADE = 8u,        /* materials | textures | image records of small scenes */
    RTW_LDS_GEOMETRY = 16u,    /* quads | members | instances of small object scenes */
    RTW_LDS_PERLIN = 32u,      /* Perlin tables (noise scenes) */
    RTW_LDS_MEGA_NODES = 64u,  /* the persistent megakernel's node stage */
    RTW_LDS_ALL = 127u
};
enum {  /* rtw_tuning.fuse */
    RTW_FUSE_STEP = 1u,        /* gen + trace + shade of an iteration in one kernel (trees staged in LDS) */
    RTW_FUSE_TAIL_LDS = 2u,    /* the tail kernel walks the LDS stage */
    RTW_FUSE_GLOBAL = 4u       /* the fused step also for trees read through L1/L2 */
};
#define RTW_OTREE_NO_CULL 0x100u  /* rtw_tuning.object_tree */
typedef struct rtw_tuning {
    uint32_t kernel;           /* rtw_kernel_kind (default WAVEFRONT) */
    uint32_t bvh_orders;       /* 0 = auto (SAH sphere scenes: 4 for small static untextured trees whose 4-copy
                                  compact stage fits half the LDS -- Book-1 --, else 8; other scenes 1), 1, 4 or 8
                                  (4: copies ordered by the x and z signs, the walk takes y's near/far per ray;
                                  half the compact-LDS stage; ABI 7) */
    uint32_t sah_max_leaf;     /* spheres per SAH leaf (default 1) */
    uint32_t compact_nodes;    /* 1 = 16-B fp16 node walk for static sphere SAH trees (default); 2 = 32-B nodes
                                  with fp32 boxes for packed FMAs, with bvh_orders 4 (else as 1; ABI 7) */
    uint32_t fast_box;         /* 1 = FMA slab test on the padded SAH boxes (default); 0 = aabb.zig arithmetic */
    uint32_t fast_reject;      /* 1 = exact sphere fast-reject filter (default) */
    uint32_t lds;              /* RTW_LDS_* (default RTW_LDS_ALL) */
    uint32_t fuse;             /* RTW_FUSE_* (default STEP | TAIL_LDS) */
    uint32_t wf_iters;         /* wavefront iterations before the tail kernel (1..100; default 0 = auto: 4, or 100 -- every bounce, no tail -- on image-textured scenes) */
    uint32_t mega_shade_min;   /* persistent kernel: lanes ready before a shading pass (default 48; 1..64) */
    uint32_t mega_waves;       /* persistent kernel: launch-bound variant (default 1; 1, 6 or 8) */
    uint32_t mega_tile_order;  /* persistent kernel: 1 = last tile row first (default) */
    uint32_t cpu_threads;      /* host context (RTW_DEVICE_CPU): render threads, 0 = every available core */
    uint32_t wide_walk;        /* 1 = two-wide stack walk for static sphere SAH trees read through L1/L2 (default) */
    uint64_t wf_paths;         /* wavefront batch capacity in paths; 0 = auto (2^29 within 35 % of free memory) */
    uint32_t tile_lists;       /* camera rays of static sphere scenes (fused step) test per-8x8-tile candidate lists:
                                  0 = off, 1 = default (lists of <= 32 spheres, 128 for trees of > 4096 nodes),
                                  2..128 = that cap (ABI 4; 128 since ABI 8) */
    uint32_t hoist;            /* SAH sphere scenes: spheres whose box dwarfs the rest of the scene (a ground
                                  sphere) are tested first by every walk, ahead of the tree (default 1; ABI 5) */
    uint32_t sort_iters;       /* fused step (trees staged in LDS): wavefront iterations 0 .. sort_iters-1 file
                                  their survivors into 64-slot blocks by direction, so the next iteration's
                                  waves walk coherent rays (default 3; 0 = plain appends; ABI 5) */
    uint32_t sort_bits;        /* direction-bucket key bits of those blocks: 0..4 (default 4 = 16 buckets: x, z signs,
                                  4 elevation levels; 0 = one block per wave, appends in order; ABI 5) */
    uint32_t sort_iters_split; /* the same for the split trace / shade kernels (trees through L1/L2: C4), whose
                                  HBM-bound shade pays more for the scattered block stores (default 1; ABI 5) */
    uint32_t object_tree;      /* SAH trees of object scenes (quads / instances / media), bits 0..7: inner nodes
                                  whose box has >= this % of the area of the node above are not emitted (their
                                  children take their place: box tests that almost always pass), 0 = the plain
                                  SAH tree, default 90; | RTW_OTREE_NO_CULL: instance and medium leaves do not
                                  test the instance's world box before its transforms and members (ABI 5,
                                  formerly padding) */
    uint32_t clds_shape;       /* compact-LDS kernels (fused step, tail) of a 4-copy tree: 0 = auto (= 4), 1 = one
                                  1024-thread block per CU, 4 = two blocks of 768 threads (6 waves per SIMD) when
                                  the stage fits half the LDS; the 8-copy stage always runs one block (ABI 7; ABI 8
                                  refuses the former 2 / 3, two blocks of 512 / 640 threads, which lost their A/Bs) */
    uint32_t deal;             /* how the wavefront's waves share work (ABI 8), RTW_DEAL_* bits; 0 = all static,
                                  default 59 = RUNS | TAIL | SMALL | ITERS | SINGLES16 */
} rtw_tuning;
enum {  /* rtw_tuning.deal (ABI 8: the per-stripe tail claims, bit 4, and the two-launch tail, bit 64, lost their
           A/Bs and were removed -- diag/deal_tail_modes.patch; both bits are now refused) */
    RTW_DEAL_RUNS = 1u,        /* iteration 0's runs of 16 samples of a tile (the last chunks singly) claimed from a
                                  counter per stripe group as its waves finish, instead of dealt round-robin */
    RTW_DEAL_TAIL = 2u,        /* the tail's input chunks claimed from one counter instead of each wave's own list */
    RTW_DEAL_SMALL = 8u,       /* the dynamic deal also on batches with fewer than 192 chunks of 64 paths per wave
                                  (which otherwise keep the static shares) */
    RTW_DEAL_ITERS = 16u,      /* the fused step's iterations >= 1 claim their stripe's chunks from a counter per
                                  stripe group */
    RTW_DEAL_SINGLES16 = 32u,  /* iteration 0's last 16 x (waves) chunks go singly (else the last 4 x) */
    RTW_DEAL_SMALL_SORT = 128u,/* direction bucketing (sort_iters / sort_iters_split) also on batches with fewer
                                  than 192 chunks per wave, which otherwise append in order: a test knob that runs
                                  the queues of the large benched batches on small images (same image) */
    RTW_DEAL_ALL = 187u
};

void rtw_tuning_defaults(rtw_tuning* out);
/* rtw_scene_create with explicit tuning (NULL = defaults). */
int rtw_scene_create_ex(const rtw_scene_desc* desc, int device, const rtw_tuning* tuning, rtw_ctx** out);
void rtw_scene_destroy(rtw_ctx* ctx);

/* Camera.render for the pixel range [pix_begin, pix_end) (linear index
 * i = y*W + x, the Task chunk of src/camera.zig:94-95) and the 0-based sample
 * range [spp_begin, spp_end) (number_of_samples = s+1, camera.zig:98).
 * accum: caller-owned HOST float4[W*H] (ColorAndSamples, camera.zig:21-39):
 * rgb += sample radiance in sample order, w = spp_end (camera.zig:55-56).
 * seed keys the counter-based RNG: identical (seed, pixel, sample) -> identical
 * draws regardless of ranges, batching, devices.  cancel (may be NULL) is
 * polled between sample batches (camera.zig:107).  Blocking. */
int rtw_render(rtw_ctx* ctx, const rtw_camera* cam, uint32_t pix_begin, uint32_t pix_end,
               uint32_t spp_begin, uint32_t spp_end, uint64_t seed, float* accum,
               const volatile int32_t* cancel, rtw_progress_fn progress, void* user);
/* ABI 5: the same with rtw_render_opts (spp_batch and the stop/progress fields; flags, counters and
 * timing must be 0/NULL).  A host context polls running/cancel per pixel as well (camera.zig:107).
 * A stopped call returns RTW_E_CANCELLED with the finished batches in accum. */
int rtw_render_ex(rtw_ctx* ctx, const rtw_camera* cam, uint32_t pix_begin, uint32_t pix_end,
                  uint32_t spp_begin, uint32_t spp_end, uint64_t seed, float* accum, const rtw_render_opts* opts);

/* Same, on a DEVICE buffer float4[W*H] already resident on ctx's device, on
 * `stream` (a hipStream_t, or NULL for the ctx's own stream).  With
 * RTW_RENDER_NO_SYNC the call only enqueues work. */
int rtw_render_device(rtw_ctx* ctx, const rtw_camera* cam, uint32_t pix_begin, uint32_t pix_end,
                      uint32_t spp_begin, uint32_t spp_end, uint64_t seed, float* d_accum,
                      void* stream, const rtw_render_opts* opts);

/* Row-interleaved shard of an image for multi-GPU:
 * renders rows r with (r / rows_per_block) % n_shards == shard into a compact
 * device buffer d_tile (float4[rows_in_shard * W], rows in increasing order). */
int rtw_render_rows_device(rtw_ctx* ctx, const rtw_camera* cam, uint32_t rows_per_block, uint32_t n_shards,
                           uint32_t shard, uint32_t spp_begin, uint32_t spp_end, uint64_t seed,
                           float* d_tile, void* stream, const rtw_render_opts* opts);
/* ABI 5: the same shard into a caller-owned HOST tile float4[rows_in_shard * W] (blocking), on a GPU
 * context or a host context (RTW_DEVICE_CPU: the shard rendered on host threads, e.g. one process per
 * rank without a GPU).  opts as rtw_render_ex (may be NULL). */
int rtw_render_rows(rtw_ctx* ctx, const rtw_camera* cam, uint32_t rows_per_block, uint32_t n_shards, uint32_t shard,
                    uint32_t spp_begin, uint32_t spp_end, uint64_t seed, float* tile, const rtw_render_opts* opts);
uint32_t rtw_shard_rows(uint32_t height, uint32_t rows_per_block, uint32_t n_shards, uint32_t shard);
/* Image row of row `tile_row` of a shard's compact tile (>= height: padding; 0xFFFFFFFF: bad spec).
 * The same function places rows in the render kernels and the multi-GPU gather. */
uint32_t rtw_shard_image_row(uint32_t rows_per_block, uint32_t n_shards, uint32_t shard, uint32_t tile_row);
/* ABI 7: rows_per_block | RTW_ROWS_BALANCED (every shard entry point, rtw_render_multi* included): rounds of
 * n_shards row blocks dealt in alternating order (round k: shard s takes the round's block s if k is even, block
 * n_shards - 1 - s if odd, so no shard always gets the lowest block of a round), then the rows left over (height
 * mod (rows_per_block * n_shards)) split evenly -- `sub` = ceil(rest / n_shards) consecutive rows per shard, in the
 * same alternating position, in one more block slot of its tile -- so the shards' row counts differ by at most sub
 * instead of by one block.  rtw_shard_image_row_h: the image row of a tile row under either layout (>= height:
 * padding; 0xFFFFFFFF: bad spec). */
#define RTW_ROWS_BALANCED 0x80000000u
uint32_t rtw_shard_image_row_h(uint32_t height, uint32_t rows_per_block, uint32_t n_shards, uint32_t shard,
                               uint32_t tile_row);

/* ---------------------------------------------------------------------------
 * Multi-GPU frame in one process (the north star's "8-GPU tile shard
 * + one RCCL gather" behind the FFI).  Replaces startRender's 8-thread split
 * (src/main.zig:314-326) of Camera.render (src/camera.zig:93-116) with N devices:
 * device k renders the row blocks b with b % N == k (rtw_render_rows_device) into
 * a compact tile; one grouped RCCL send/recv moves every tile to device 0, where
 * the rows are scattered into the frame.  Unless RTW_RENDER_FRESH, the frame's
 * current rows are first scattered to the devices the same way, so progressive
 * calls accumulate exactly as on one device: the result is bit-identical to
 * rtw_render_device for any N (counter-based RNG keyed by seed, pixel, sample).
 * ------------------------------------------------------------------------- */
typedef struct rtw_multi rtw_multi;
/* ctxs[k]: one context per device, each from rtw_scene_create(desc, device_k) with the
 * same desc; ctxs[0]'s device holds the frame.  Creates the RCCL communicators
 * (ncclCommInitAll) once.  The contexts must outlive the rtw_multi and must not be
 * rendered on by other callers during an rtw_render_multi* call. */
int rtw_multi_create(rtw_ctx* const* ctxs, uint32_t n, rtw_multi** out);
void rtw_multi_destroy(rtw_multi* m);
enum { RTW_RENDER_FRESH = 2u };  /* rtw_render_multi_device: start the range from zero, do not read d_accum */
/* d_accum: float4[W*H] on ctxs[0]'s device; stream: a hipStream_t of that device or NULL.
 * opts: spp_batch, flags (RTW_RENDER_NO_SYNC, RTW_RENDER_FRESH) and the ABI-5 stop/progress fields
 * are honoured (every device renders batch b, all of them finish, then progress and the flags are
 * polled; the tiles meet on device 0 once, after the last finished batch -- also on a stop, which
 * returns RTW_E_CANCELLED with the frame holding every finished batch); counters and timing must
 * be NULL. */
int rtw_render_multi_device(rtw_multi* m, const rtw_camera* cam, uint32_t rows_per_block, uint32_t spp_begin,
                            uint32_t spp_end, uint64_t seed, float* d_accum, void* stream,
                            const rtw_render_opts* opts);
/* Same on a caller-owned HOST float4[W*H] (ColorAndSamples), blocking; cancel is polled
 * between spp batches (rtw_render_multi_ex: the full rtw_render_opts, e.g. the Zig `running` flag
 * and a progress callback). */
int rtw_render_multi(rtw_multi* m, const rtw_camera* cam, uint32_t rows_per_block, uint32_t spp_begin,
                     uint32_t spp_end, uint64_t seed, float* accum, const volatile int32_t* cancel);
int rtw_render_multi_ex(rtw_multi* m, const rtw_camera* cam, uint32_t rows_per_block, uint32_t spp_begin,
                        uint32_t spp_end, uint64_t seed, float* accum, const rtw_render_opts* opts);
/* ABI 5: devices of the rtw_multi and ranks of its RCCL communicator (ncclCommCount of device 0's). */
int rtw_multi_info(rtw_multi* m, uint32_t* n_devices, int* rccl_ranks);

/* SharedStateImageWriter texel update: u8(256*clamp(sqrt(rgb/w),0,0.999)), alpha 255
 * (src/camera.zig:58-65, src/color.zig:43-62). Host, n pixels. */
int rtw_texture_from_accum(const float* accum, uint32_t n, uint8_t* rgba_out);
/* The same texel update on the device (d_accum float4[n] -> d_rgba u8x4[n], HBM), enqueued on
 * `stream` (NULL = the context's default device stream of device 0's current context). */
int rtw_texture_from_accum_device(const float* d_accum, uint32_t n, uint8_t* d_rgba, void* stream);

/* ---------------------------------------------------------------------------
 * Output formats (the reference's README TODO "Output selector"
 * and main.zig:47 "save to file").  Host-only, over the float4 accumulator.
 * ------------------------------------------------------------------------- */
enum rtw_ppm_style {
    RTW_PPM_WRITECOLOR = 0,    /* color.zig:64-69 writeColor: round(256 * toGamma(c)), "r g b\n" per pixel
                                  (the format of the reference's image2.ppm; values reach 256) */
    RTW_PPM_STDOUT = 1         /* stdout.zig:5-18 printPpmToStdout: floor(255.999 * toGamma(c)), "r g b\t"
                                  (the format of image.ppm) */
};
/* P3 PPM "P3\n<w> <h>\n255\n" + pixels row-major from the top row.  Writes at most cap
 * bytes; *len = bytes of the whole encoding (call with out = NULL to size the buffer).
 * Returns RTW_E_INVALID if out != NULL and cap < *len.  NaN components print "nan". */
int rtw_encode_ppm(const float* accum, uint32_t width, uint32_t height, uint32_t style, char* out, size_t cap,
                   size_t* len);
/* ---------------------------------------------------------------------------
 * Progressive / resumable renders.  rtw_render* accumulate
 * samples [spp_begin, spp_end) onto the buffer in sample order, so any split
 * of [0, spp) into consecutive calls -- including across a checkpoint -- is
 * bit-identical to one call.
 * ------------------------------------------------------------------------- */
/* countSamples (src/main.zig:470-477): f32 sum of accum[i][3] in index order -- the
 * control panel's progress (vs spp * n) and POWER (= samples / elapsed ms, :495-503). */
float rtw_count_samples(const float* accum, uint64_t n);
/* FNV-1a 64 of the scene's device image (nodes + geometry + materials + textures); a
 * checkpoint records it so a resume on a different scene or BVH is refused. */
int rtw_scene_hash(rtw_ctx* ctx, uint64_t* out);
/* Checkpoint file (little endian): "RTWCKPT1", u32 version 1, u32 spp_done, u64 seed,
 * u64 scene_hash, rtw_camera, u64 n_pixels, float4[n_pixels] accumulator, u32 CRC-32 of
 * everything before it.  read: cam/seed/hash/spp_done may be NULL; accum must hold
 * cap_pixels float4 (n_pixels must equal cap_pixels) -- RTW_E_INVALID on any mismatch or
 * corruption. */
int rtw_checkpoint_write(const char* path, const rtw_camera* cam, uint64_t seed, uint64_t scene_hash,
                         uint32_t spp_done, const float* accum);
int rtw_checkpoint_read(const char* path, rtw_camera* cam, uint64_t* seed, uint64_t* scene_hash,
                        uint32_t* spp_done, float* accum, uint64_t cap_pixels);

/* 8-bit RGBA PNG (zlib stored blocks, no filtering) of u8x4 texels, e.g. the
 * SharedStateImageWriter texture_buffer (rtw_texture_from_accum).  Same sizing contract. */
int rtw_encode_png(const uint8_t* rgba, uint32_t width, uint32_t height, uint8_t* out, size_t cap, size_t* len);

/* Host-only: build + flatten the BVH exactly as rtw_scene_create does, without
 * touching a device (nodes_out may be NULL to query the count). */
int rtw_scene_flatten(const rtw_scene_desc* desc, void* nodes_out, uint32_t cap, uint32_t* n_out,
                      uint32_t* depth_out);

/* Introspection for tests / reports. */
typedef struct rtw_scene_stats {
    uint32_t n_nodes, n_leaves, n_inner, depth;
    uint64_t device_bytes;
    uint32_t axis_draws;
    uint32_t n_hoisted;        /* spheres emitted ahead of the tree (rtw_tuning.hoist) */
    float extent;              /* ABI 6: E = max |coordinate| over every object box and inner node (SAH) */
    float box_pad;             /* ABI 6: E * 2^-19, the inner-box pad of the FMA slab test (0: exact walk) */
} rtw_scene_stats;
int rtw_scene_stats_get(rtw_ctx* ctx, rtw_scene_stats* out);
/* Copies the flattened node array (32 B per node) to host. */
int rtw_scene_nodes(rtw_ctx* ctx, void* out, uint32_t cap, uint32_t* n_out);

/* Debug / known-answer hooks, executed ON THE DEVICE by the same device
 * functions the render kernel uses. */
int rtw_debug_rng(rtw_ctx* ctx, uint64_t seed, uint32_t pixel, uint32_t sample, uint32_t n, float* out);
int rtw_debug_sample(rtw_ctx* ctx, const rtw_camera* cam, uint64_t seed, uint32_t pixel, uint32_t sample,
                     float out[3]);
/* ABI 6, host-only: the walk's sphere fast-reject (sphere_may_hit, the same fp32 operations as the
 * device) and Sphere.hit's exact accept (objects.zig:127-136, tmin = 0.001) for n sphere tests given
 * a = lengthSquared(d), half_b = dot(oc, d), c = lengthSquared(oc) - r*r and closest: the test suite
 * checks that the filter never rejects a test the exact arithmetic accepts. */
int rtw_debug_sphere_filter(uint32_t n, const float* a, const float* half_b, const float* c, const float* closest,
                            uint8_t* may_hit, uint8_t* accept);

#ifdef __cplusplus
}
#endif
#endif /* RTW_GPU_H */
