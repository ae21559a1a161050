// rtw_internal.h -- private declarations shared by the host runtime
// (rtw_host.hip), the BVH builder (rtw_bvh.hip) and the kernels (rtw_kernels.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <condition_variable>
#include <atomic>
#include <mutex>
#include <vector>

#include "rtw_layout.h"
#include "../../include/rtw_gpu.h"

struct rtw_scene_desc;

// Everything one launch of the path-tracing kernel reads (passed by value as
// kernel arguments; scalars live in SGPRs).
struct rtw_launch {
    // scene (device pointers)
    const float4* nodes;
    const uint4* cnodes;         // compact 16-B copy of `nodes` (static sphere SAH trees) or null; with cnode32
                                 // the 32-B fp32-box form (two uint4 per node, 4-copy trees)
    const uint4* w2nodes;        // two-wide records of ordering 0 (rtw_wide2_nodes) or null
    const uint32_t* w2leaf;      // their leaf slots' hit ids (ordering-0 leaf index)
    const float4* cvec;          // per-sphere center_vec (moving spheres)
    const rtw_dev_sphere* sph;   // every sphere (instance members)
    const rtw_dev_quad* quads;
    const rtw_dev_instance* insts;
    const uint32_t* members;
    const rtw_dev_medium* media;
    const rtw_dev_material* mats;
    const rtw_dev_texture* texs;
    const uint8_t* images;
    const rtw_dev_image* img_info;
    const float4* perlin;        // RTW_PERLIN_BYTES per table
    uint32_t n_nodes;
    uint32_t n_perlin;
    uint32_t w2_stack;           // entries of the two-wide walk's per-lane LDS stack (its max depth)
    uint32_t tile_lists;         // camera rays of the fused step of static sphere scenes test per-tile candidate
                                 // lists of at most this many spheres (0 = off; more candidates: the walk)

    // camera (Camera.init outputs, src/camera.zig:118-154)
    float center[3], pixel00[3], du[3], dv[3], disk_u[3], disk_v[3], background[3];
    float defocus_angle;
    uint32_t W, H, max_depth, bg_mode, pixel_offset;

    // work: rows [row0, row0 + n_rows) of the logical row space, pixels
    // restricted to linear range [pix_begin, pix_end); samples [s0, s1)
    uint32_t row0, n_rows;
    uint32_t pix_begin, pix_end;
    uint32_t s0, s1;
    // row mapping: logical row r -> image row
    //   shard mode (n_shards > 0): y = ((r / rpb) * n_shards + shard) * rpb + r % rpb, out idx = r*W + x
    //   plain mode: y = r, out idx = y*W + x
    uint32_t rpb, n_shards, shard;
    uint64_t key0;               // mix64(seed + 0*G): render-domain key
    float4* accum;
    unsigned long long* counters;  // RTW_STAT_COUNT or nullptr

    // persistent kernel (v1) work queue: tiles of RTW_TILE_W x RTW_TILE_H logical pixels
    uint32_t* work_counter;      // zeroed before every launch
    uint32_t n_tiles_x, n_tiles;
    uint32_t shade_min;          // lanes that must be ready before a shading pass (<= 64)
    uint32_t feat;               // RTW_F_* scene features (selects the kernel instantiation)
    uint32_t waves;              // launch-bound variant (min waves per SIMD): 1, 6 or 8
    uint32_t tile_order;         // 1 = last tile row first (default), 0 = first row first
    uint32_t use_lds;            // 1 = stage the BVH in LDS when it fits (default), 0 = read nodes from L1/L2
    uint32_t fast_reject;        // 1 = exact sphere fast-reject filter (default), 0 = always the IEEE path
    uint32_t fast_box;           // 1 = FMA slab test on padded boxes (SAH trees only), 0 = aabb.zig arithmetic
    uint32_t inst_cull;          // 1 = instance / medium leaves test the instance's padded world box first
                                 // (only with fast_box; rtw_tuning.object_tree without RTW_OTREE_NO_CULL)
    uint32_t n_orders;           // 1, or 4 / 8 sign-ordered copies of the node array (SAH sphere scenes)
    uint32_t cnode32;            // 1: cnodes are the 32-B fp32-box nodes (rtw_tuning.compact_nodes 2)
    uint32_t clds_shape;         // compact-LDS kernels of a 4-copy tree: 0 / 1 = one 1024-thread block per CU,
                                 // 4 = two blocks of 768 threads (rtw_tuning.clds_shape)
    uint32_t wf_lds;             // wavefront trace: stage the node array(s) in LDS when they fit
    uint32_t wf_clds;            // wavefront trace: stage the compact nodes (all orders) in LDS when they fit
    uint32_t wf_fuse;            // with the compact LDS stage: one gen+trace+shade kernel per iteration,
                                 // bit 1: the tail walks the LDS stage too
    uint32_t perlin_lds;         // fused step with the node array in LDS: Perlin tables staged in LDS too
    uint32_t mat_lds;            // compact-LDS fused step: bytes of the material array staged in LDS (0: off)
    uint32_t shade_lds;          // node-LDS kernels: bytes of materials | textures | image records (contiguous
                                 // in the scene blob) staged in LDS when small; 0 = read through L1/L2
    uint32_t geom_lds;           // node-LDS step/tail: bytes of quads | members | instances (contiguous in the
                                 // scene blob) staged in LDS too; 0 = read through L1/L2
};

#define RTW_TILE_W 16
#define RTW_TILE_H 16
#define RTW_TILE (RTW_TILE_W * RTW_TILE_H)

// scene feature bits: kernels are instantiated per feature set so Book-1
// (solid textures, static spheres, no lights) carries no texture/motion code
#define RTW_F_CHECKER 1u
#define RTW_F_IMAGE 2u
#define RTW_F_NOISE 4u
#define RTW_F_MOVING 8u
#define RTW_F_LIGHT 16u
#define RTW_F_GEOM 32u      // quads / instances (non-sphere BVH leaves)
#define RTW_F_MEDIUM 64u    // ConstantMedium leaves
#define RTW_F_SPHERES 31u   // every sphere-scene feature
#define RTW_F_ALL 127u

// max nodes staged in LDS by the persistent kernel (48 KiB)
#define RTW_MEGA_LDS_NODES_MAX 1536

struct rtw_kernel_info {
    int blocks_per_cu;
    int n_cu;
};
int rtw_persistent_grid(uint32_t feat, uint32_t n_nodes, int waves, bool use_lds);

void rtw_launch_render(const rtw_launch& L, void* stream, int variant, int grid);
void rtw_set_error(const char* msg);  // the thread's rtw_last_error() message (rtw_host.hip)
// ABI-5 stop flags of rtw_render_opts: RenderThread.running (a Zig bool, 0 = stop) or cancel (non-zero = stop)
inline bool rtw_stop_requested(const rtw_render_opts* o) {
    return o && ((o->running && *o->running == 0) || (o->cancel && *o->cancel != 0));
}
// does the caller poll between batches (stop flags or progress)?
inline bool rtw_polled(const rtw_render_opts* o) { return o && (o->running || o->cancel || o->progress); }

// host backend (rtw_cpu.hip): samples [L.s0, L.s1) of the logical pixels [begin, end) onto host float4 `out`.
// Plain launches (L.n_shards == 0): logical pixel = image pixel, out = the frame.  Shard launches: logical
// pixel r * W + x of the shard's tile (image row rtw_tile_row_image(L.rpb, L.n_shards, L.shard, r)), out =
// the tile.  `stop` (may be null) is polled per pixel, as Camera.render polls `running` (camera.zig:107).
int rtw_cpu_render(const rtw_launch& L, uint32_t begin, uint32_t end, float* out, uint32_t threads,
                   const rtw_render_opts* stop);
void rtw_launch_debug_rng(uint64_t seed, uint32_t pixel, uint32_t sample, uint32_t n, float* d_out, void* stream);
void rtw_launch_debug_sample(const rtw_launch& L, uint32_t pixel, uint32_t sample, float* d_out, void* stream);

// Per-kernel HIP-event timing of one render call (rtw_render_opts.timing).
struct rtw_timer {
    struct rec {
        int kind;
        hipEvent_t a, b;
    };
    std::vector<rec> recs;
    std::vector<hipEvent_t> pool;
    hipStream_t stream = nullptr;
    int cur = -1;
    hipEvent_t ev() {
        hipEvent_t e = nullptr;
        if (!pool.empty()) {
            e = pool.back();
            pool.pop_back();
        } else {
            (void)hipEventCreate(&e);
        }
        return e;
    }
    void begin(int kind) {
        recs.push_back({kind, ev(), nullptr});
        (void)hipEventRecord(recs.back().a, stream);
    }
    void end() {
        recs.back().b = ev();
        (void)hipEventRecord(recs.back().b, stream);
    }
};
// begin/end a timed launch when a timer is attached
#define RTW_TIME_BEGIN(T, kind) \
    if (T) (T)->begin(kind);
#define RTW_TIME_END(T) \
    if (T) (T)->end();

// Host copies of the device geometry arrays besides the nodes (rtw_layout.h records).
struct rtw_geometry {
    std::vector<float> cvec;                 // float4 per sphere: center_vec (moving spheres)
    std::vector<rtw_dev_sphere> spheres;     // every sphere
    std::vector<rtw_dev_quad> quads;
    std::vector<rtw_dev_instance> insts;
    std::vector<uint32_t> members;           // RTW_REF
    std::vector<rtw_dev_medium> media;
    uint32_t feat = 0;                       // RTW_F_GEOM | RTW_F_MEDIUM as present
};

// Validates the object graph, derives the geometry records and builds the BVH
// over world_objects.  box_pad/extent (out, may be null): SAH trees pad every
// inner box by extent * 2^-19 so the FMA slab test (box_next) stays conservative.
// SAH trees: `orders` (1 or 8) pre-order arrays, one per ray-direction octant when 8
// (concatenated; node indices and skip links are relative to each array).
// 16-B node of the compact walk (rtw_bvh.hip rtw_compact_nodes)
struct rtw_cnode {
    uint32_t v[4];
};
// false: the tree cannot be encoded (coordinates beyond fp16 range, non-finite radius).
// fp32 (4 copies only): 32-B nodes with fp32 boxes instead (2 rtw_cnode per node; rtw_compact_nodes)
bool rtw_compact_nodes(const std::vector<rtw_node>& nodes, uint32_t orders, std::vector<rtw_cnode>& out,
                       bool fp32 = false);

// two-wide 32-B records (2 x rtw_cnode per inner node) of ordering 0 for the stack walk of large static
// sphere SAH trees (rtw_bvh.hip rtw_wide2_nodes); false: not encodable (leaf runs, fp16 range)
bool rtw_wide2_nodes(const std::vector<rtw_node>& nodes, uint32_t n_per, std::vector<rtw_cnode>& out,
                     std::vector<uint32_t>& leaf_id, uint32_t* max_stack);

// hoist (SAH sphere scenes): emit spheres whose box dwarfs the rest ahead of the tree (*n_hoisted of them)
// flatten_pct (SAH trees): inner nodes with >= that % of the area of the node above are not emitted
// (0 = off; SahBuilder::emit_tree)
int rtw_build_bvh(const rtw_scene_desc& desc, std::vector<rtw_node>& nodes, rtw_geometry& geom,
                  uint32_t* depth, uint32_t* axis_draws, float* box_pad = nullptr, float* extent = nullptr,
                  uint32_t orders = 1, uint32_t sah_max_leaf = 1, uint32_t hoist = 0, uint32_t* n_hoisted = nullptr,
                  uint32_t flatten_pct = 0);

// One scene on one device (the opaque rtw_ctx of include/rtw_gpu.h).
struct rtw_ctx {
    int device = 0;                // RTW_DEVICE_CPU: a host context (rtw_cpu.hip)
    std::vector<uint8_t> host_blob;  // host context: the scene image the launch pointers address
    hipStream_t stream = nullptr;
    void* d_blob = nullptr;        // single allocation holding every scene array
    size_t blob_bytes = 0;
    rtw_launch base{};
    rtw_scene_stats stats{};
    std::vector<rtw_node> nodes_host;
    float* d_scratch = nullptr;    // host-API accum staging (rtw_render_ex: the callers' chunks of one frame)
    size_t scratch_bytes = 0;
    float* d_rows = nullptr;       // rtw_render_rows' tile staging (its own: render_ex chunks may be staged
    size_t rows_bytes = 0;         //   in d_scratch while it runs)
    float* d_dbg = nullptr;        // debug kernels output
    uint32_t* d_work = nullptr;    // persistent-kernel work counter (zeroed before each launch)
    uint32_t feat = 0;             // RTW_F_* scene features
    int grid = 0;                  // resident blocks of the persistent kernel
    int variant = 2;               // 2 = wavefront v2 (default), 1 = persistent v1, 0 = simple v0 (rtw_tuning.kernel)
    void* d_tl = nullptr;          // camera-ray tile candidate lists (rtw_wavefront.h), tl_cap tiles
    uint64_t tl_cap = 0;
    void* d_wf = nullptr;          // wavefront path state (rtw_wavefront.h), wf_cap paths
    uint64_t wf_cap = 0;
    uint64_t wf_max_paths = 1u << 26;  // paths per wavefront batch (x RTW_WF_PATH_BYTES); set at scene creation
    uint32_t wf_iters = 9;         // wavefront bounces before the tail kernel (rtw_tuning.wf_iters)
    uint32_t wf_sort_mask = 15;    // their bucket key bits (rtw_tuning.sort_bits)
    uint32_t wf_sort_iters_split = 1;  // the same for the split kernels (rtw_tuning.sort_iters_split)
    uint32_t wf_sort_iters = 3;    // iterations whose survivors are filed by direction (rtw_tuning.sort_iters)
    uint32_t cpu_threads = 0;      // host context: worker threads (rtw_tuning.cpu_threads; 0 = all)
    uint32_t wf_deal = 0;          // iteration 0's runs dealt dynamically (rtw_tuning.deal)
    int n_cu = 256;                // compute units of the device (wavefront grids)
    std::vector<hipEvent_t> ev_pool;  // recycled timing events
    uint64_t scene_hash = 0;       // FNV-1a 64 of the uploaded scene image
    float box_pad = 0;             // absolute pad baked into the inner boxes (SAH trees), 0 = none
    float extent = 0;              // max |coordinate| over the scene's boxes
    // Concurrent callers (the reference's 8 RenderThreads call Camera.render at once, main.zig:314-326):
    // one caller at a time enqueues work on a context -- the wavefront state and staging buffers are per
    // context -- and work on another stream than the previous enqueue's waits for that work on the
    // device.  The host-buffer API (rtw_render_ex) holds the lock only while it enqueues one spp batch,
    // so the 8 Tasks' batches interleave; host_calls counts its calls with a chunk staged in d_scratch.
    std::mutex mu;
    std::condition_variable host_cv;
    int host_calls = 0;
    std::atomic<uint32_t> cpu_calls{0};  // host context: calls rendering now (they share cpu_threads)
    hipEvent_t last_done = nullptr;
    hipStream_t last_stream = nullptr;
};
