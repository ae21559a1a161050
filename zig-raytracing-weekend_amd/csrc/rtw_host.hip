// rtw_host.hip -- C ABI implementation (include/rtw_gpu.h): scene upload,
// Camera.init, batched launches with cancel/progress, sharded row rendering.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "../../include/rtw_gpu.h"
#include "rtw_internal.h"
#include "rtw_layout.h"
#include "rtw_rng.h"
#include "rtw_wavefront.h"

namespace {

thread_local std::string g_err;

int fail(int code, const char* msg) {
    g_err = msg;
    return code;
}

int hip_fail(hipError_t e, const char* where) {
    g_err = std::string(where) + ": " + hipGetErrorString(e);
    return e == hipErrorOutOfMemory ? RTW_E_OOM : RTW_E_HIP;
}

#define HIP_TRY(expr)                                   \
    do {                                                \
        hipError_t _e = (expr);                         \
        if (_e != hipSuccess) return hip_fail(_e, #expr); \
    } while (0)

}  // namespace

void rtw_set_error(const char* msg) { g_err = msg ? msg : ""; }

// struct rtw_ctx: see rtw_internal.h

namespace {
uint32_t scene_features(const rtw_scene_desc* d) {
    uint32_t f = 0;
    for (uint32_t i = 0; i < d->n_spheres; i++)
        if (d->spheres[i].is_moving) f |= RTW_F_MOVING;
    for (uint32_t i = 0; i < d->n_materials; i++) {
        const rtw_material& m = d->materials[i];
        if (m.kind == RTW_MAT_DIFFUSE_LIGHT || m.kind == RTW_MAT_ISOTROPIC) f |= RTW_F_LIGHT;
        const bool textured = m.kind == RTW_MAT_LAMBERTIAN || m.kind == RTW_MAT_DIFFUSE_LIGHT || m.kind == RTW_MAT_ISOTROPIC;
        if (!textured) continue;
        const uint32_t k = d->textures[m.texture].kind;
        if (k == RTW_TEX_CHECKER) f |= RTW_F_CHECKER;
        if (k == RTW_TEX_IMAGE) f |= RTW_F_IMAGE;
        if (k == RTW_TEX_NOISE) f |= RTW_F_NOISE;
    }
    return f;
}
}  // namespace

extern "C" {

int rtw_version(void) { return RTW_ABI_VERSION; }

const char* rtw_last_error(void) { return g_err.c_str(); }

int rtw_device_count(int* out) {
    if (!out) return fail(RTW_E_INVALID, "null out");
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    if (e != hipSuccess) n = 0;
    *out = n;
    return RTW_OK;
}

// Camera.init (src/camera.zig:118-154).  Plain fp32 host arithmetic in the
// Zig expression order; tan is the host libm (the Zig std tan is a musl port).
int rtw_camera_init(const rtw_camera_params* p, rtw_camera* c) {
#pragma STDC FP_CONTRACT OFF
    if (!p || !c) return fail(RTW_E_INVALID, "null camera params");
    if (p->image_width == 0) return fail(RTW_E_INVALID, "image_width == 0");
    std::memset(c, 0, sizeof *c);
    uint32_t H = p->image_height;
    if (H == 0) H = (uint32_t)std::round((float)p->image_width / p->aspect_ratio);
    if (H < 1) H = 1;
    const uint32_t W = p->image_width;
    c->image_width = W;
    c->image_height = H;
    c->size = W * H;
    c->samples_per_pixel = p->samples_per_pixel;
    c->max_depth = p->max_depth;
    c->background_mode = p->background_mode;
    c->pixel_offset = p->pixel_offset;
    for (int k = 0; k < 3; k++) c->background[k] = p->background[k];
    const float pi = 3.1415926535897932385f;
    const float theta = p->vfov * pi / 180.0f;
    const float h = std::tan(theta / 2.0f);
    const float vh = 2 * h * p->focus_dist;
    const float vw = vh * ((float)W / (float)H);
    float w[3], u[3], v[3], tmp[3];
    for (int k = 0; k < 3; k++) tmp[k] = p->lookfrom[k] - p->lookat[k];
    auto unit = [](const float* a, float* o) {
        float l = std::sqrt(a[0] * a[0] + a[1] * a[1] + a[2] * a[2]);
        for (int k = 0; k < 3; k++) o[k] = a[k] / l;
    };
    auto cross = [](const float* a, const float* b, float* o) {
        o[0] = a[1] * b[2] - a[2] * b[1];
        o[1] = a[2] * b[0] - a[0] * b[2];
        o[2] = a[0] * b[1] - a[1] * b[0];
    };
    unit(tmp, w);
    cross(p->vup, w, tmp);
    unit(tmp, u);
    cross(w, u, v);
    float vu[3], vv[3];
    for (int k = 0; k < 3; k++) {
        vu[k] = vw * u[k];
        vv[k] = vh * -v[k];
        c->pixel_delta_u[k] = vu[k] / (float)W;
        c->pixel_delta_v[k] = vv[k] / (float)H;
        const float upper_left = ((p->lookfrom[k] - p->focus_dist * w[k]) - vu[k] / 2.0f) - vv[k] / 2.0f;
        c->pixel00_loc[k] = upper_left + 0.5f * (c->pixel_delta_u[k] + c->pixel_delta_v[k]);
        c->center[k] = p->lookfrom[k];
        c->u[k] = u[k];
        c->v[k] = v[k];
        c->w[k] = w[k];
    }
    const float defocus_radius = p->focus_dist * std::tan((p->defocus_angle / 2.0f) * pi / 180.0f);
    for (int k = 0; k < 3; k++) {
        c->defocus_disk_u[k] = u[k] * defocus_radius;
        c->defocus_disk_v[k] = v[k] * defocus_radius;
    }
    c->defocus_angle = p->defocus_angle;
    return RTW_OK;
}

void rtw_tuning_defaults(rtw_tuning* t) {
    if (!t) return;
    std::memset(t, 0, sizeof *t);
    t->kernel = RTW_KERNEL_WAVEFRONT;
    t->bvh_orders = 0;
    t->sah_max_leaf = 1;
    t->compact_nodes = 1;
    t->fast_box = 1;
    t->fast_reject = 1;
    t->lds = RTW_LDS_ALL;
    t->fuse = RTW_FUSE_STEP | RTW_FUSE_TAIL_LDS;
    t->wf_iters = 0;  // auto: 4, or every bounce (no tail) on image-textured scenes (profiles/r5_iters/)
    t->mega_shade_min = 48;  // tuned on C2: 8..64 -> 48 best
    t->mega_waves = 1;
    t->mega_tile_order = 1;
    t->cpu_threads = 0;
    t->wide_walk = 1;
    t->tile_lists = 1;
    t->hoist = 1;
    t->sort_iters = 3;
    t->sort_bits = RTW_WF_BUCKET_BITS;
    t->object_tree = 90;  // Cornell 1356 -> 1475, Cornell smoke +5.5 %
    t->sort_iters_split = 1;  // C4: 1 -> 2577, 3 -> 2518, 0 -> 2523 Msamples/s
    t->wf_paths = 0;
    // dynamic dealing of iteration 0 (runs, then 16 x waves singles), iterations >= 1 and the tail's input, on every
    // batch size: C2 +11 % over deal 3, C4 +7 %, C3 +9 %, a C2 shard of 8 +11 % (profiles/r5_deal/)
    t->deal = 59;
}

int rtw_scene_create(const rtw_scene_desc* d, int device, rtw_ctx** out) {
    return rtw_scene_create_ex(d, device, nullptr, out);
}

int rtw_scene_create_ex(const rtw_scene_desc* d, int device, const rtw_tuning* tuning, rtw_ctx** out) {
    if (!d || !out) return fail(RTW_E_INVALID, "null scene desc");
    rtw_tuning tu;
    rtw_tuning_defaults(&tu);
    if (tuning) tu = *tuning;
    if (tu.kernel > RTW_KERNEL_SIMPLE) return fail(RTW_E_INVALID, "tuning.kernel out of range");
    if (tu.bvh_orders != 0 && tu.bvh_orders != 1 && tu.bvh_orders != 4 && tu.bvh_orders != 8)
        return fail(RTW_E_INVALID, "tuning.bvh_orders must be 0, 1, 4 or 8");
    if (tu.clds_shape != 0 && tu.clds_shape != 1 && tu.clds_shape != 4)
        return fail(RTW_E_INVALID, "tuning.clds_shape must be 0, 1 or 4 (ABI 8)");
    if (tu.deal & ~(uint32_t)RTW_DEAL_ALL)
        return fail(RTW_E_INVALID, "tuning.deal: bits 1 | 2 | 8 | 16 | 32 | 128 (RTW_DEAL_*)");
    if (tu.wf_iters > RTW_WF_MAX_ITERS) return fail(RTW_E_INVALID, "tuning.wf_iters out of range");
    if ((tu.object_tree & 0xFFu) > 100 || (tu.object_tree & ~(0xFFu | RTW_OTREE_NO_CULL)))
        return fail(RTW_E_INVALID, "tuning.object_tree: 0..100 [| RTW_OTREE_NO_CULL]");
    if (tu.sort_bits > RTW_WF_BUCKET_BITS) return fail(RTW_E_INVALID, "tuning.sort_bits out of range");
    if (tu.mega_shade_min < 1 || tu.mega_shade_min > 64) return fail(RTW_E_INVALID, "tuning.mega_shade_min out of range");
    if (tu.mega_waves != 1 && tu.mega_waves != 6 && tu.mega_waves != 8) return fail(RTW_E_INVALID, "tuning.mega_waves must be 1, 6 or 8");
    if (tu.wf_paths && tu.wf_paths < 4096) return fail(RTW_E_INVALID, "tuning.wf_paths must be 0 or >= 4096");
    *out = nullptr;
    if ((d->n_spheres && !d->spheres) || (d->objects ? d->n_objects : d->n_spheres) == 0)
        return fail(RTW_E_INVALID, "scene has no objects");
    if (d->n_materials == 0 || !d->materials) return fail(RTW_E_INVALID, "scene has no materials");
    for (uint32_t i = 0; i < d->n_spheres; i++)
        if (d->spheres[i].material >= d->n_materials) return fail(RTW_E_INVALID, "sphere material index out of range");
    for (uint32_t i = 0; i < d->n_materials; i++) {
        const rtw_material& m = d->materials[i];
        if (m.kind > RTW_MAT_ISOTROPIC) return fail(RTW_E_INVALID, "unknown material kind");
        const bool textured = m.kind == RTW_MAT_LAMBERTIAN || m.kind == RTW_MAT_DIFFUSE_LIGHT || m.kind == RTW_MAT_ISOTROPIC;
        if (textured && m.texture >= d->n_textures) return fail(RTW_E_INVALID, "material texture index out of range");
    }
    for (uint32_t i = 0; i < d->n_textures; i++) {
        const rtw_texture& t = d->textures[i];
        if (t.kind > RTW_TEX_NOISE) return fail(RTW_E_INVALID, "unknown texture kind");
        if (t.kind == RTW_TEX_IMAGE && t.image >= d->n_images) return fail(RTW_E_INVALID, "texture image index out of range");
        if (t.kind == RTW_TEX_NOISE && t.perlin >= d->n_perlins) return fail(RTW_E_INVALID, "texture perlin index out of range");
    }
    for (uint32_t i = 0; i < d->n_images; i++) {
        const rtw_image& im = d->images[i];
        if (im.width && im.height && (!im.data || im.bytes_per_row < 4 * im.width))
            return fail(RTW_E_INVALID, "bad image");
    }
    const bool host = device == RTW_DEVICE_CPU;  // a host context: no GPU involved (rtw_cpu.hip)
    if (!host) {
        int ndev = 0;
        if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return fail(RTW_E_NODEVICE, "no HIP device visible");
        if (device < 0 || device >= ndev) return fail(RTW_E_INVALID, "device index out of range");
    }

    rtw_ctx* ctx = new rtw_ctx();
    ctx->device = device;
    rtw_geometry geom;
    uint32_t depth = 0, draws = 0;
    // SAH trees of sphere scenes: 8 octant-ordered copies of the node array (tuning.bvh_orders 4: copies by the
    // x and z signs; 1: one, ordered
    // along order_dir).  Scenes with quads/instances/media keep one order: their leaf tests are costly, and
    // lanes walking different orders stop executing them together (Cornell: -31 % with 8 orders).
    const bool objects = d->n_quads || d->n_instances || d->n_media;
    uint32_t orders = (d->bvh_mode == RTW_BVH_SAH && !objects) ? 8u : 1u;
    // Round 5: small static untextured sphere trees (Book-1, C2 / C3) take 4 copies (x, z signs): their compact
    // stage (+ materials) then fits half the LDS and the fused step and tail run two 768-thread blocks per CU, 6
    // waves per SIMD (C2 +4.6 %, profiles/r5_stage/).  (A tree of ~2 nodes per sphere; the check is redone on the
    // built tree by the launcher, which falls back to one block.)
    const uint32_t sfeat = scene_features(d);
    const size_t mat_b = (size_t)d->n_materials * sizeof(rtw_dev_material);
    if (orders == 8 && !tu.bvh_orders && tu.compact_nodes == 1 && tu.fast_box && !(sfeat & ~RTW_F_CHECKER) &&
        (2 * (size_t)d->n_spheres + 8) * 4 * 16 + mat_b <= RTW_WF_CLDS2_MAX)
        orders = 4;
    // (object scenes keep one ordering: their hit ids carry an instance member where sphere scenes carry the copy)
    if (tu.bvh_orders) orders = (d->bvh_mode == RTW_BVH_SAH && !objects && tu.bvh_orders > 1) ? tu.bvh_orders : 1u;
    uint32_t n_hoisted = 0;
    int rc = rtw_build_bvh(*d, ctx->nodes_host, geom, &depth, &draws, &ctx->box_pad, &ctx->extent, orders,
                           tu.sah_max_leaf, tu.hoist && !objects ? 1u : 0u, &n_hoisted, objects ? (tu.object_tree & 0xFFu) : 0u);
    if (rc != RTW_OK) {
        delete ctx;
        return fail(rc, "BVH build failed (bad object graph or bvh_mode)");
    }
    if ((geom.feat & RTW_F_GEOM) && ctx->nodes_host.size() >= (1u << RTW_HIT_NODE_BITS)) {
        delete ctx;
        return fail(RTW_E_INVALID, "scenes with instances are limited to 2^24 BVH nodes");
    }
    const std::vector<float>& cvec = geom.cvec;
    // compact 16-B walk for static sphere SAH trees (rtw_compact_nodes)
    std::vector<rtw_cnode> cnodes;
    bool cnode32 = false;
    {
        bool want = d->bvh_mode == RTW_BVH_SAH && !objects && ctx->box_pad > 0 && tu.compact_nodes && !host;
        for (uint32_t i = 0; want && i < d->n_spheres; i++) want = !d->spheres[i].is_moving;
        // compact_nodes 2: the 32-B fp32-box form where it applies (4 copies), else the 16-B fp16 form
        cnode32 = want && tu.compact_nodes == 2 && orders == 4 && rtw_compact_nodes(ctx->nodes_host, orders, cnodes, true);
        if (want && !cnode32 && !rtw_compact_nodes(ctx->nodes_host, orders, cnodes)) cnodes.clear();
    }
    // two-wide records for the stack walk of trees read through L1/L2 (rtw_wide2_nodes)
    std::vector<rtw_cnode> w2;
    std::vector<uint32_t> w2leaf;
    uint32_t w2_stack = 0;
    if (!cnodes.empty() && !cnode32 && tu.wide_walk && tu.sah_max_leaf <= 1 &&
        !rtw_wide2_nodes(ctx->nodes_host, (uint32_t)(ctx->nodes_host.size() / orders), w2, w2leaf, &w2_stack))
        w2.clear();
    if (w2_stack > RTW_W2_STACK_MAX) w2.clear();

    // Blob layout (each section 256-B aligned): nodes | cvec | spheres | quads | members | instances | media |
    // materials | textures | images-info | perlin | image bytes || compact nodes | two-wide records (not hashed)
    auto align = [](size_t x) { return (x + 255) & ~size_t(255); };
    const size_t n_nodes = ctx->nodes_host.size() / orders;  // per ordering
    size_t off = 0;
    const size_t o_nodes = off; off = align(off + ctx->nodes_host.size() * sizeof(rtw_node));
    const size_t o_cvec = off; off = align(off + cvec.size() * sizeof(float) + 16);
    const size_t o_sph = off; off = align(off + geom.spheres.size() * sizeof(rtw_dev_sphere) + 16);
    const size_t o_quad = off; off = align(off + geom.quads.size() * sizeof(rtw_dev_quad) + 16);
    const size_t o_memb = off; off = align(off + geom.members.size() * sizeof(uint32_t) + 16);
    const size_t o_inst = off; off = align(off + geom.insts.size() * sizeof(rtw_dev_instance) + 16);
    const size_t o_med = off; off = align(off + geom.media.size() * sizeof(rtw_dev_medium) + 16);
    const size_t o_mats = off; off = align(off + d->n_materials * sizeof(rtw_dev_material));
    const size_t o_texs = off; off = align(off + (d->n_textures + 1) * sizeof(rtw_dev_texture));
    const size_t o_imgi = off; off = align(off + (d->n_images + 1) * sizeof(rtw_dev_image));
    const size_t o_perl = off; off = align(off + (size_t)(d->n_perlins + 1) * RTW_PERLIN_BYTES);
    const size_t o_imgs = off;
    std::vector<rtw_dev_image> img_info(d->n_images + 1);
    size_t img_bytes = 0;
    for (uint32_t i = 0; i < d->n_images; i++) {
        img_info[i].offset = img_bytes;
        img_info[i].width = d->images[i].width;
        img_info[i].height = d->images[i].height;
        img_info[i].bytes_per_row = d->images[i].bytes_per_row;
        img_bytes += align((size_t)d->images[i].bytes_per_row * d->images[i].height);
    }
    off = align(off + img_bytes + 16);
    // the scene image: the walks' derived records below (compact nodes, two-wide records) depend on the
    // backend and the tuning, so a checkpoint's hash matches on every context of the same scene (the
    // node array, whose layout also follows the tuning, is left out of the hash as well)
    const size_t hashed = off;
    const size_t o_cnod = off; off = align(off + cnodes.size() * sizeof(rtw_cnode));
    const size_t o_w2 = off; off = align(off + w2.size() * sizeof(rtw_cnode));
    const size_t o_w2l = off; off = align(off + w2leaf.size() * sizeof(uint32_t));

    std::vector<uint8_t> blob(off, 0);
    std::memcpy(blob.data() + o_nodes, ctx->nodes_host.data(), ctx->nodes_host.size() * sizeof(rtw_node));
    auto put = [&](size_t o, const void* src, size_t nb) {
        if (nb) std::memcpy(blob.data() + o, src, nb);
    };
    put(o_cnod, cnodes.data(), cnodes.size() * sizeof(rtw_cnode));
    put(o_w2, w2.data(), w2.size() * sizeof(rtw_cnode));
    put(o_w2l, w2leaf.data(), w2leaf.size() * sizeof(uint32_t));
    put(o_cvec, cvec.data(), cvec.size() * sizeof(float));
    put(o_sph, geom.spheres.data(), geom.spheres.size() * sizeof(rtw_dev_sphere));
    put(o_quad, geom.quads.data(), geom.quads.size() * sizeof(rtw_dev_quad));
    put(o_memb, geom.members.data(), geom.members.size() * sizeof(uint32_t));
    put(o_inst, geom.insts.data(), geom.insts.size() * sizeof(rtw_dev_instance));
    put(o_med, geom.media.data(), geom.media.size() * sizeof(rtw_dev_medium));
    for (uint32_t i = 0; i < d->n_materials; i++) {
        rtw_dev_material m{};
        m.kind = d->materials[i].kind;
        m.texture = d->materials[i].texture;
        m.fuzz = d->materials[i].fuzz;
        m.ir = d->materials[i].ir;
        for (int k = 0; k < 3; k++) m.albedo[k] = d->materials[i].albedo[k];
        std::memcpy(blob.data() + o_mats + i * sizeof m, &m, sizeof m);
    }
    for (uint32_t i = 0; i < d->n_textures; i++) {
        rtw_dev_texture t{};
        const rtw_texture& s = d->textures[i];
        t.kind = s.kind; t.image = s.image; t.perlin = s.perlin; t.scale = s.scale;
        for (int k = 0; k < 3; k++) { t.even[k] = s.even[k]; t.odd[k] = s.odd[k]; }
        std::memcpy(blob.data() + o_texs + i * sizeof t, &t, sizeof t);
    }
    std::memcpy(blob.data() + o_imgi, img_info.data(), img_info.size() * sizeof(rtw_dev_image));
    for (uint32_t i = 0; i < d->n_perlins; i++) {
        uint8_t* base = blob.data() + o_perl + (size_t)i * RTW_PERLIN_BYTES;
        float* vec = reinterpret_cast<float*>(base);
        for (int k = 0; k < 256; k++) {
            vec[4 * k + 0] = d->perlins[i].ranvec[k][0];
            vec[4 * k + 1] = d->perlins[i].ranvec[k][1];
            vec[4 * k + 2] = d->perlins[i].ranvec[k][2];
            vec[4 * k + 3] = 0.0f;
        }
        uint32_t* perm = reinterpret_cast<uint32_t*>(base + 256 * 16);
        for (int k = 0; k < 256; k++) {
            perm[k] = d->perlins[i].perm_x[k];
            perm[256 + k] = d->perlins[i].perm_y[k];
            perm[512 + k] = d->perlins[i].perm_z[k];
        }
    }
    for (uint32_t i = 0; i < d->n_images; i++) {
        const size_t nb = (size_t)d->images[i].bytes_per_row * d->images[i].height;
        if (nb) std::memcpy(blob.data() + o_imgs + img_info[i].offset, d->images[i].data, nb);
    }

    if (!host) {
        hipError_t e = hipSetDevice(device);
        // blocking stream: orders with the legacy NULL stream (torch's default), so a caller passing
        // device buffers and stream == NULL sees its prior NULL-stream work (e.g. zero fills) complete first
        if (e == hipSuccess) e = hipStreamCreateWithFlags(&ctx->stream, hipStreamDefault);
        if (e == hipSuccess) e = hipMalloc(&ctx->d_blob, off);
        if (e == hipSuccess) e = hipMemcpy(ctx->d_blob, blob.data(), off, hipMemcpyHostToDevice);
        if (e == hipSuccess) e = hipMalloc(&ctx->d_dbg, 64 * sizeof(float));
        if (e == hipSuccess) e = hipMalloc(&ctx->d_work, 256);
        if (e != hipSuccess) {
            int code = hip_fail(e, "rtw_scene_create upload");
            rtw_scene_destroy(ctx);
            return code;
        }
    }
    ctx->blob_bytes = off;
    {   // FNV-1a 64 of the scene image (rtw_scene_hash): the tree kind (and the reference topology's seed),
        // then every section after the nodes -- the node array's layout depends on the tuning (orderings,
        // hoisting, object_tree), the image does not
        uint64_t h = 0xCBF29CE484222325ull;
        const uint64_t key[2] = {(uint64_t)d->bvh_mode, d->bvh_mode == RTW_BVH_REFERENCE ? (uint64_t)d->bvh_seed : 0ull};
        const unsigned char* kb = reinterpret_cast<const unsigned char*>(key);
        for (size_t i = 0; i < sizeof key; i++) h = (h ^ kb[i]) * 0x100000001B3ull;
        for (size_t i = o_cvec; i < hashed; i++) h = (h ^ blob[i]) * 0x100000001B3ull;
        ctx->scene_hash = h;
    }
    if (host) ctx->host_blob = blob;  // the launch pointers address the host copy
    uint8_t* dev = host ? ctx->host_blob.data() : static_cast<uint8_t*>(ctx->d_blob);
    rtw_launch& L = ctx->base;
    L.nodes = reinterpret_cast<const float4*>(dev + o_nodes);
    L.cnodes = cnodes.empty() ? nullptr : reinterpret_cast<const uint4*>(dev + o_cnod);
    L.w2nodes = w2.empty() ? nullptr : reinterpret_cast<const uint4*>(dev + o_w2);
    L.w2leaf = w2.empty() ? nullptr : reinterpret_cast<const uint32_t*>(dev + o_w2l);
    L.w2_stack = w2.empty() ? 0u : w2_stack;
    // default cap: 32 candidates for small trees (flat prepass: C2 16/32/64 -> 5765/5789/5769), 128 for large
    // ones (frustum-walked prepass: C4 32/64 -> 2440/2458; round 6, 64/96/128 -> 3147/3156/3166,
    // profiles/r6_late_rest/)
    L.tile_lists = tu.tile_lists == 1 ? (n_nodes <= 4096 ? 32u : 128u) : std::min<uint32_t>(tu.tile_lists, RTW_TL_MAX);
    L.cvec = reinterpret_cast<const float4*>(dev + o_cvec);
    L.sph = reinterpret_cast<const rtw_dev_sphere*>(dev + o_sph);
    L.quads = reinterpret_cast<const rtw_dev_quad*>(dev + o_quad);
    L.members = reinterpret_cast<const uint32_t*>(dev + o_memb);
    L.insts = reinterpret_cast<const rtw_dev_instance*>(dev + o_inst);
    L.media = reinterpret_cast<const rtw_dev_medium*>(dev + o_med);
    L.mats = reinterpret_cast<const rtw_dev_material*>(dev + o_mats);
    L.texs = reinterpret_cast<const rtw_dev_texture*>(dev + o_texs);
    L.img_info = reinterpret_cast<const rtw_dev_image*>(dev + o_imgi);
    L.perlin = reinterpret_cast<const float4*>(dev + o_perl);
    L.images = dev + o_imgs;
    L.n_nodes = (uint32_t)n_nodes;
    L.n_orders = orders;
    L.clds_shape = tu.clds_shape ? tu.clds_shape : 4u;  // auto: two 768-thread blocks where the stage fits
    ctx->wf_deal = tu.deal;
    L.cnode32 = cnode32 ? 1u : 0u;
    L.n_perlin = d->n_perlins;
    ctx->feat = scene_features(d) | geom.feat;
    L.feat = ctx->feat;
    L.work_counter = ctx->d_work;
    ctx->variant = tu.kernel == RTW_KERNEL_WAVEFRONT ? 2 : tu.kernel == RTW_KERNEL_PERSISTENT ? 1 : 0;
    {
        // wavefront batch capacity: up to 2^29 paths (BASELINE config 2 = 480M samples in one
        // batch: one drain of long paths per render instead of one per 64M), within ~35 % of
        // the device's FREE memory at scene creation (RTW_WF_PATH_BYTES per path); the
        // allocation halves the batch on failure (run_wavefront)
        size_t free_b = 0, total_b = 0;
        uint64_t cap = 1ull << 29;
        if (!host && hipMemGetInfo(&free_b, &total_b) == hipSuccess && free_b)
            cap = std::min<uint64_t>(cap, (uint64_t)(0.35 * (double)free_b) / RTW_WF_PATH_BYTES);
        ctx->wf_max_paths = tu.wf_paths ? tu.wf_paths : std::max<uint64_t>(cap, 1u << 20);
    }
    // Round 5, with the dynamic tail (deal bit 2): fewer iterations before the tail pay everywhere but on
    // image-textured scenes -- same-box A/B, 9 -> 4 iterations: C2 +3.7 %, C4 +3.3 %, Cornell +6.8 %, smoke
    // +1.2 %, simple_light +1.9 %.  Image-textured scenes run no tail at all (every bounce a wavefront
    // iteration: the launcher clamps to max_depth): C5 9 / 24 / 32 / 50 iterations 9425 / 9750 / 9816 / 9990
    // Msamples/s (profiles/r5_iters/).
    ctx->wf_iters = tu.wf_iters ? tu.wf_iters : (sfeat & RTW_F_IMAGE) ? (uint32_t)RTW_WF_MAX_ITERS : 4u;
    ctx->wf_sort_iters = tu.sort_iters;
    ctx->wf_sort_iters_split = tu.sort_iters_split;
    ctx->wf_sort_mask = (1u << tu.sort_bits) - 1u;
    {
        int n_cu = 0;
        if (host || hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess ||
            n_cu < 1)
            n_cu = 256;
        ctx->n_cu = n_cu;
    }
    L.shade_min = tu.mega_shade_min;
    L.waves = tu.mega_waves;
    L.tile_order = tu.mega_tile_order ? 1u : 0u;
    // (an unfiltered variant measured +-0 on C2 and -20 % on C4: its codegen slowed the L1/L2 walk)
    L.fast_reject = tu.fast_reject ? 1u : 0u;
    L.use_lds = orders == 1 && (tu.lds & RTW_LDS_MEGA_NODES) ? 1u : 0u;  // the octant copies do not fit the megakernel's stage
    // wavefront trace: node array staged in LDS when one ordering fits (object scenes,
    // reference trees; +2 % on Cornell); the 8 octant copies of SAH sphere trees do not
    L.wf_lds = (tu.lds & RTW_LDS_NODES) ? 1u : 0u;
    // small static sphere SAH trees: the compact nodes of all 8 orders in LDS (C2: +1 %)
    L.wf_clds = (tu.lds & RTW_LDS_CNODES) ? 1u : 0u;
    // compact LDS stage: gen, trace and shade of an iteration fused in one kernel
    // (the ray/hit hand-off through HBM disappears), tail on the LDS stage
    L.wf_fuse = tu.fuse;
    // Perlin tables (7 KiB each) staged in LDS by the fused step when at most 4 (noise scenes)
    L.perlin_lds = (ctx->feat & RTW_F_NOISE) && d->n_perlins <= 4 && (tu.lds & RTW_LDS_PERLIN) ? 1u : 0u;
    // materials of sphere scenes staged in LDS by the compact-LDS fused step when they fit beside the
    // nodes (wf_run_fused checks the total): hit_prep's material load stops waiting on L1/L2
    L.mat_lds = (tu.lds & RTW_LDS_MATERIALS) ? (uint32_t)((d->n_materials * sizeof(rtw_dev_material) + 15) & ~size_t(15)) : 0u;
    const size_t shade_bytes = (size_t)(o_perl - o_mats);
    L.shade_lds = shade_bytes <= 8192 && (tu.lds & RTW_LDS_SHADE) ? (uint32_t)shade_bytes : 0u;
    // quads, instance member lists and instances of small object scenes (Cornell: ~2 KiB) staged in LDS
    // with the node array: the member loop's loads stop waiting on L1
    const size_t geom_bytes = (size_t)(o_med - o_quad);
    L.geom_lds = (ctx->feat & RTW_F_GEOM) && geom_bytes <= 16384 && (tu.lds & RTW_LDS_GEOMETRY) ? (uint32_t)geom_bytes : 0u;
    // SAH trees: FMA slab test on the padded boxes (only enlarges the set of visited nodes;
    // reference trees keep the exact aabb.zig walk)
    L.fast_box = ctx->box_pad > 0 && tu.fast_box ? 1u : 0u;
    L.inst_cull = (tu.object_tree & RTW_OTREE_NO_CULL) ? 0u : 1u;  // consulted only with fast_box
    if (host) {  // the exact aabb.zig slab test and IEEE sphere test (the hardware estimates are device-only)
        L.fast_box = 0;
        L.fast_reject = 0;
    }
    ctx->cpu_threads = tu.cpu_threads;
    ctx->grid = host ? 0 : rtw_persistent_grid(ctx->feat, (uint32_t)n_nodes, (int)L.waves, L.use_lds != 0);

    ctx->stats.n_nodes = (uint32_t)n_nodes;
    ctx->stats.n_leaves = d->objects ? d->n_objects : d->n_spheres;
    ctx->stats.n_inner = (uint32_t)n_nodes - ctx->stats.n_leaves;
    ctx->stats.depth = depth;
    ctx->stats.device_bytes = off;
    ctx->stats.axis_draws = draws;
    ctx->stats.n_hoisted = n_hoisted;
    ctx->stats.extent = ctx->extent;
    ctx->stats.box_pad = ctx->box_pad;
    *out = ctx;
    return RTW_OK;
}

void rtw_scene_destroy(rtw_ctx* ctx) {
    if (!ctx) return;
    if (ctx->device == RTW_DEVICE_CPU) {
        delete ctx;
        return;
    }
    (void)hipSetDevice(ctx->device);
    if (ctx->last_done) (void)hipEventSynchronize(ctx->last_done);  // a render left on a caller's stream
    if (ctx->stream) (void)hipStreamSynchronize(ctx->stream);
    if (ctx->last_done) (void)hipEventDestroy(ctx->last_done);
    if (ctx->d_blob) (void)hipFree(ctx->d_blob);
    if (ctx->d_scratch) (void)hipFree(ctx->d_scratch);
    if (ctx->d_rows) (void)hipFree(ctx->d_rows);
    if (ctx->d_dbg) (void)hipFree(ctx->d_dbg);
    if (ctx->d_work) (void)hipFree(ctx->d_work);
    if (ctx->d_wf) (void)hipFree(ctx->d_wf);
    if (ctx->d_tl) (void)hipFree(ctx->d_tl);
    for (hipEvent_t e : ctx->ev_pool) (void)hipEventDestroy(e);
    if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
    delete ctx;
}

int rtw_scene_flatten(const rtw_scene_desc* d, void* out, uint32_t cap, uint32_t* n_out, uint32_t* depth_out) {
    if (!d || (d->n_spheres && !d->spheres) || (d->objects ? d->n_objects : d->n_spheres) == 0)
        return fail(RTW_E_INVALID, "scene has no objects");
    std::vector<rtw_node> nodes;
    rtw_geometry geom;
    uint32_t depth = 0, draws = 0;
    int rc = rtw_build_bvh(*d, nodes, geom, &depth, &draws);
    if (rc != RTW_OK) return fail(rc, "BVH build failed");
    const uint32_t n = (uint32_t)nodes.size();
    if (n_out) *n_out = n;
    if (depth_out) *depth_out = depth;
    if (out) std::memcpy(out, nodes.data(), sizeof(rtw_node) * (cap < n ? cap : n));
    return RTW_OK;
}

int rtw_scene_hash(rtw_ctx* ctx, uint64_t* out) {
    if (!ctx || !out) return fail(RTW_E_INVALID, "null ctx");
    *out = ctx->scene_hash;
    return RTW_OK;
}

int rtw_scene_stats_get(rtw_ctx* ctx, rtw_scene_stats* out) {
    if (!ctx || !out) return fail(RTW_E_INVALID, "null ctx");
    *out = ctx->stats;
    return RTW_OK;
}

int rtw_scene_nodes(rtw_ctx* ctx, void* out, uint32_t cap, uint32_t* n_out) {
    if (!ctx) return fail(RTW_E_INVALID, "null ctx");
    const uint32_t n = ctx->stats.n_nodes;  // the first ordering
    if (n_out) *n_out = n;
    if (out) std::memcpy(out, ctx->nodes_host.data(), sizeof(rtw_node) * (cap < n ? cap : n));
    return RTW_OK;
}

}  // extern "C"

namespace {

rtw_launch make_launch(const rtw_ctx* ctx, const rtw_camera* c, uint64_t seed) {
    rtw_launch L = ctx->base;
    for (int k = 0; k < 3; k++) {
        L.center[k] = c->center[k];
        L.pixel00[k] = c->pixel00_loc[k];
        L.du[k] = c->pixel_delta_u[k];
        L.dv[k] = c->pixel_delta_v[k];
        L.disk_u[k] = c->defocus_disk_u[k];
        L.disk_v[k] = c->defocus_disk_v[k];
        L.background[k] = c->background[k];
    }
    L.defocus_angle = c->defocus_angle;
    L.W = c->image_width;
    L.H = c->image_height;
    L.max_depth = c->max_depth;
    L.bg_mode = c->background_mode;
    L.pixel_offset = c->pixel_offset;
    L.key0 = rtw_mix64(seed);
    if (L.fast_box) {
        // the box pad covers ray origins with |o| <= 7 * extent (rtw_bvh.hip): primary
        // origins are the camera centre + the defocus disk; secondary ones lie in the scene
        float o = 0;
        for (int k = 0; k < 3; k++)
            o = std::max(o, std::fabs(c->center[k]) + std::fabs(c->defocus_disk_u[k]) +
                                std::fabs(c->defocus_disk_v[k]));
        if (!(o <= 7.0f * ctx->extent)) L.fast_box = 0;
    }
    return L;
}

uint32_t auto_batch(const rtw_ctx* ctx, uint64_t pixels, uint32_t spp) {
    // ~64M samples per launch (the wavefront: its batch capacity): long enough to
    // amortise the launches, short enough to poll cancel
    const uint64_t target = ctx->variant == 2 ? ctx->wf_max_paths : (64ull << 20);
    uint64_t b = pixels ? target / pixels : spp;
    if (b < 1) b = 1;
    if (b > spp) b = spp;
    return (uint32_t)b;
}

int validate_cam(const rtw_camera* cam) {
    if (!cam) return fail(RTW_E_INVALID, "null camera");
    if (cam->image_width == 0 || cam->image_height == 0) return fail(RTW_E_INVALID, "camera not initialised");
    if ((uint64_t)cam->image_width * cam->image_height > 0xFFFFFFFFull) return fail(RTW_E_INVALID, "image too large");
    return RTW_OK;
}

// Bytes of the wavefront state run_wavefront takes from one allocation: per slot set (two) the ray_o, ray_d,
// thr, acc streams (16 B) and rng (8 B); the hit records (8 B) by slot; the radiance (12 B) by path; the three
// stripe-counter sets; each take 256-B aligned.  RTW_WF_PATH_BYTES is the per-path part of the same sum.
size_t wf_state_bytes(uint64_t Q, uint64_t P) {
    auto al = [](uint64_t b) { return (size_t)((b + 255) & ~uint64_t(255)); };
    return 2 * (4 * al(Q * 16) + al(Q * 8)) + al(Q * 8) + al(P * sizeof(rtw_rgb)) +
           3 * al((uint64_t)RTW_WF_STRIPES * RTW_WF_LEN_STRIDE * 4) + al(RTW_WF_DEAL_COUNTERS * 4);
}
static_assert(RTW_WF_PATH_BYTES == 2 * (4 * 16 + 8) + 8 + sizeof(rtw_rgb), "RTW_WF_PATH_BYTES = wf_state_bytes per path");

// Wavefront (v2) render of samples [L.s0, L.s1): batches of n_s samples so that
// n_pix * n_s paths fit the path-state buffer (grown on demand, kept in the ctx).
int run_wavefront(rtw_ctx* ctx, rtw_launch L, hipStream_t stream, rtw_timer* T) {
    rtw_wf W{};
    W.n_tx = (L.W + 7) / 8;
    const uint64_t n_pix = (uint64_t)W.n_tx * ((L.n_rows + 7) / 8) * 64;
    const uint32_t spp = L.s1 - L.s0;
    uint64_t n_s = std::max<uint64_t>(1, ctx->wf_max_paths / n_pix);
    if (n_s > spp) n_s = spp;
    uint64_t need = n_pix * n_s;
    if (need > 0x7FFFFFFFull) return fail(RTW_E_INVALID, "wavefront batch too large");
    // stripe capacity: a stripe receives the survivors of nw/STRIPES waves that
    // each take <= ceil(chunks / nw) 64-path chunks (rtw_wavefront.h)
    const uint64_t max_waves = rtw_wavefront_max_waves(ctx->n_cu);
    // + direction-bucketed iterations: every wave of a stripe may leave one partly filled 64-slot block per
    //   bucket (wf_push_bucketed)
    const uint64_t bucket_blocks = (ctx->wf_sort_iters || ctx->wf_sort_iters_split) ? (max_waves / RTW_WF_STRIPES + 1) * RTW_WF_BUCKETS : 0;
    // + the dynamic deal of iteration 0 (rtw_tuning.deal bit 1): a stripe group claims whole runs of 16 chunks
    //   and then singles, so it may end up to one run and one single chunk above its even share (RUN + 1), whatever
    //   the grid's waves per stripe (a device or partition with few CUs)
    const uint64_t deal_slack = ctx->wf_deal ? (1u << 4) + 1u : 0u;
    auto stripe_cap = [&](uint64_t paths) {
        return ((paths + 63) / 64 / RTW_WF_STRIPES + 1 + max_waves / RTW_WF_STRIPES + bucket_blocks + deal_slack) * 64;
    };
    // slots per set: every path (iteration 0: slot = path id) or every stripe's capacity
    auto slots = [&](uint64_t paths) { return std::max<uint64_t>(paths, stripe_cap(paths) * RTW_WF_STRIPES); };
    if (ctx->wf_cap < need) {
        if (ctx->d_wf) {
            HIP_TRY(hipStreamSynchronize(stream));
            (void)hipFree(ctx->d_wf);
        }
        ctx->d_wf = nullptr;
        ctx->wf_cap = 0;
        for (;;) {  // device memory taken since scene creation (other contexts, torch): halve the batch
            const size_t bytes = wf_state_bytes(slots(need), need);
            const hipError_t e = hipMalloc(&ctx->d_wf, bytes);
            if (e == hipSuccess) break;
            if (e != hipErrorOutOfMemory || n_s == 1) return hip_fail(e, "wavefront path state");
            (void)hipGetLastError();  // clear the sticky OOM before the retry
            n_s = (n_s + 1) / 2;
            need = n_pix * n_s;
            ctx->wf_max_paths = need;  // later renders start from the size that fit
        }
        ctx->wf_cap = need;
    }
    if (n_s * n_pix > ctx->wf_cap) n_s = std::max<uint64_t>(1, ctx->wf_cap / n_pix);
    const uint64_t P = ctx->wf_cap, Q = slots(P);
    // (the takes below are the layout wf_state_bytes sizes)
    char* cur = static_cast<char*>(ctx->d_wf);
    auto take = [&](size_t nb) {
        char* p = cur;
        cur += (nb + 255) & ~size_t(255);
        return p;
    };
    for (int k = 0; k < 2; k++) {
        rtw_wf_set& S = W.set[k];
        S.ray_o = reinterpret_cast<float4*>(take(Q * 16));
        S.ray_d = reinterpret_cast<float4*>(take(Q * 16));
        S.thr = reinterpret_cast<float4*>(take(Q * 16));
        S.acc = reinterpret_cast<float4*>(take(Q * 16));
        S.rng = reinterpret_cast<uint64_t*>(take(Q * 8));
    }
    W.hit = reinterpret_cast<float2*>(take(Q * 8));
    W.ls = reinterpret_cast<rtw_rgb*>(take(P * sizeof(rtw_rgb)));
    for (int k = 0; k < 3; k++) W.len[k] = reinterpret_cast<uint32_t*>(take(RTW_WF_STRIPES * RTW_WF_LEN_STRIDE * 4));
    uint32_t* deal = reinterpret_cast<uint32_t*>(take(RTW_WF_DEAL_COUNTERS * 4));
    W.deal = ctx->wf_deal ? deal : nullptr;
    W.deal_mode = ctx->wf_deal;
    W.deal_it = nullptr;  // set per launch (deal bit 16)
    W.n_pix = (uint32_t)n_pix;
    W.iters = ctx->wf_iters;
    W.sort_iters = ctx->wf_sort_iters;
    W.sort_iters_split = ctx->wf_sort_iters_split;
    W.sort_mask = ctx->wf_sort_mask;
    W.run_log2 = 4;  // set per launch grid by wf_coherence (rtw_wavefront.hip)
    // camera-ray candidate lists (the compact-LDS fused step of static sphere scenes, rtw_tuning.tile_lists)
    if (L.tile_lists && L.cnodes && L.n_orders >= 4) {
        const uint64_t tiles = n_pix / 64;
        if (ctx->tl_cap < tiles) {
            if (ctx->d_tl) {
                HIP_TRY(hipStreamSynchronize(stream));
                (void)hipFree(ctx->d_tl);
            }
            ctx->d_tl = nullptr;
            ctx->tl_cap = 0;
            if (hipMalloc(&ctx->d_tl, tiles * RTW_TL_BYTES + 256) == hipSuccess) ctx->tl_cap = tiles;
            else (void)hipGetLastError();  // no lists: the walk
        }
        if (ctx->tl_cap >= tiles) {
            W.tl = static_cast<uint4*>(ctx->d_tl);
            W.tl_count = reinterpret_cast<uint32_t*>(static_cast<char*>(ctx->d_tl) + tiles * RTW_TL_MAX * 32);
        }
    }
    const uint32_t s_end = L.s1;
    for (uint32_t s = L.s0; s < s_end; s += (uint32_t)n_s) {
        L.s0 = s;
        L.s1 = (s_end - s < n_s) ? s_end : s + (uint32_t)n_s;
        W.n_s = L.s1 - L.s0;
        W.n_paths = (uint32_t)(n_pix * W.n_s);
        W.stripe_cap = (uint32_t)stripe_cap(W.n_paths);
        rtw_wavefront_batch(L, W, stream, ctx->n_cu, T);
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return hip_fail(e, "wavefront launch");
    }
    return RTW_OK;
}

// Enqueue [s0, s1) in batches of `batch` samples on `stream`.  When the caller polls (ctl's stop
// flags or progress, ABI 5) the stop flags are read before every batch and, after each one, the stream
// is synchronised and progress called: a stop keeps the finished batches (their .w = the last batch's end).
int run_batches(rtw_ctx* ctx, rtw_launch L, uint32_t s0, uint32_t s1, uint32_t batch, hipStream_t stream,
                const rtw_render_opts* ctl, uint64_t pixels, rtw_timer* T = nullptr) {
    const uint64_t total = pixels * (uint64_t)(s1 - s0);
    const bool polled = rtw_polled(ctl);
    for (uint32_t s = s0; s < s1; s += batch) {
        if (rtw_stop_requested(ctl)) return fail(RTW_E_CANCELLED, "cancelled");
        L.s0 = s;
        L.s1 = (s1 - s < batch) ? s1 : s + batch;
        if (ctx->variant == 2) {
            if (int rc = run_wavefront(ctx, L, stream, T)) return rc;
        } else {
            if (ctx->variant == 1) HIP_TRY(hipMemsetAsync(ctx->d_work, 0, 256, stream));
            RTW_TIME_BEGIN(T, RTW_K_MEGA)
            rtw_launch_render(L, stream, ctx->variant, ctx->grid);
            RTW_TIME_END(T)
            hipError_t e = hipGetLastError();
            if (e != hipSuccess) return hip_fail(e, "render launch");
        }
        if (polled) {
            HIP_TRY(hipStreamSynchronize(stream));
            if (ctl->progress && ctl->progress(pixels * (uint64_t)(L.s1 - s0), total, ctl->user))
                return fail(RTW_E_CANCELLED, "cancelled by progress callback");
        }
    }
    return RTW_OK;
}

// Host context: samples [s0, s1) in batches on host threads (rtw_cpu.hip), stop flags polled per pixel,
// progress after each batch.  begin/end/out as rtw_cpu_render.
int run_host(rtw_ctx* ctx, rtw_launch L, uint32_t begin, uint32_t end, uint32_t s0, uint32_t s1,
             uint32_t batch, float* out, const rtw_render_opts* ctl, uint64_t pixels) {
    // concurrent callers (the 8 Tasks on one host context) share the context's threads instead of each
    // starting a pool of its own: a call takes cpu_threads / (calls in flight), at least 1
    struct Count {
        std::atomic<uint32_t>& c;
        uint32_t n;
        explicit Count(std::atomic<uint32_t>& a) : c(a), n(a.fetch_add(1) + 1) {}
        ~Count() { c.fetch_sub(1); }
    } in_flight(ctx->cpu_calls);
    const uint32_t pool = ctx->cpu_threads ? ctx->cpu_threads : std::max(1u, std::thread::hardware_concurrency());
    const uint32_t threads = std::max(1u, pool / in_flight.n);
    // stop flags: with an explicit spp_batch they are polled between batches only, so a stopped render
    // holds whole batches (every pixel's .w is the last finished batch's end, and a resume from it adds
    // no sample twice); without one, per pixel as Camera.render polls `running` (camera.zig:107) --
    // then each pixel's .w says how far that pixel got
    const bool per_pixel = batch == 0;
    if (!batch) batch = s1 - s0;
    const uint64_t total = pixels * (uint64_t)(s1 - s0);
    for (uint32_t s = s0; s < s1; s += batch) {
        if (!per_pixel && rtw_stop_requested(ctl)) return fail(RTW_E_CANCELLED, "cancelled");
        L.s0 = s;
        L.s1 = (s1 - s < batch) ? s1 : s + batch;
        if (rtw_cpu_render(L, begin, end, out, threads, per_pixel ? ctl : nullptr) == RTW_E_CANCELLED)
            return fail(RTW_E_CANCELLED, "cancelled");
        if (ctl && ctl->progress && ctl->progress(pixels * (uint64_t)(L.s1 - s0), total, ctl->user))
            return fail(RTW_E_CANCELLED, "cancelled by progress callback");
    }
    return RTW_OK;
}

// the ABI-5 options of the host-buffer entry points: stop/progress and spp_batch only
int check_host_opts(const rtw_render_opts* o) {
    if (o && (o->flags || o->counters || o->timing))
        return fail(RTW_E_INVALID, "host-buffer render: flags, counters and timing must be 0/NULL");
    return RTW_OK;
}

// Synchronise and sum the timer's events per kernel kind into `out`.
int harvest_timing(rtw_ctx* ctx, rtw_timer& T, rtw_kernel_timing* out) {
    HIP_TRY(hipStreamSynchronize(T.stream));
    std::memset(out, 0, sizeof *out);
    for (const rtw_timer::rec& r : T.recs) {
        float ms = 0;
        HIP_TRY(hipEventElapsedTime(&ms, r.a, r.b));
        if (r.kind >= 0 && r.kind < RTW_K_COUNT) {
            out->ms[r.kind] += ms;
            out->launches[r.kind]++;
        }
        ctx->ev_pool.push_back(r.a);
        ctx->ev_pool.push_back(r.b);
    }
    T.recs.clear();
    return RTW_OK;
}

void set_tiles(rtw_launch& L) {
    L.n_tiles_x = (L.W + RTW_TILE_W - 1) / RTW_TILE_W;
    L.n_tiles = L.n_tiles_x * ((L.n_rows + RTW_TILE_H - 1) / RTW_TILE_H);
}

// the context's device staging buffer of the host-buffer entry points, >= bytes
int ensure_scratch(rtw_ctx* ctx, size_t bytes) {
    if (ctx->scratch_bytes >= bytes) return RTW_OK;
    if (ctx->d_scratch) {
        HIP_TRY(hipStreamSynchronize(ctx->stream));
        (void)hipFree(ctx->d_scratch);
    }
    ctx->d_scratch = nullptr;
    ctx->scratch_bytes = 0;
    HIP_TRY(hipMalloc(&ctx->d_scratch, bytes));
    ctx->scratch_bytes = bytes;
    return RTW_OK;
}

// Order this call's stream after the previous call's work on this context (another stream).
int stream_enter(rtw_ctx* ctx, hipStream_t s) {
    if (ctx->last_stream && ctx->last_stream != s) HIP_TRY(hipStreamWaitEvent(s, ctx->last_done, 0));
    return RTW_OK;
}
int stream_leave(rtw_ctx* ctx, hipStream_t s) {
    if (!ctx->last_done) HIP_TRY(hipEventCreateWithFlags(&ctx->last_done, hipEventDisableTiming));
    HIP_TRY(hipEventRecord(ctx->last_done, s));
    ctx->last_stream = s;
    return RTW_OK;
}

// A GPU context's shard render into the device tile on stream s (the caller holds ctx->mu and has set
// the device and entered the stream): row blocks b with b % n_shards == shard, tile rows in order.
int render_rows_locked(rtw_ctx* ctx, const rtw_camera* cam, uint32_t rpb, uint32_t n_shards, uint32_t shard,
                       uint32_t spp_begin, uint32_t spp_end, uint64_t seed, float* d_tile, hipStream_t s,
                       const rtw_render_opts* opts, uint32_t rows) {
    rtw_launch L = make_launch(ctx, cam, seed);
    L.accum = reinterpret_cast<float4*>(d_tile);
    L.row0 = 0;
    // logical rows 0 .. (the shard's whole blocks); rows past H (or past a balanced shard's share) are masked
    L.n_rows = rtw_shard_tile_rows(cam->image_height, rpb, n_shards, shard);
    L.rpb = rpb;
    L.n_shards = n_shards;
    L.shard = shard;
    L.pix_begin = 0;
    L.pix_end = cam->size;
    L.counters = opts ? reinterpret_cast<unsigned long long*>(opts->counters) : nullptr;
    set_tiles(L);
    uint32_t batch = opts && opts->spp_batch ? opts->spp_batch : auto_batch(ctx, (uint64_t)rows * cam->image_width, spp_end - spp_begin);
    rtw_timer T;
    T.stream = s;
    T.pool.swap(ctx->ev_pool);
    rtw_timer* tp = (opts && opts->timing) ? &T : nullptr;
    int rc = run_batches(ctx, L, spp_begin, spp_end, batch, s, opts, (uint64_t)rows * cam->image_width, tp);
    ctx->ev_pool.swap(T.pool);
    if (int rl = stream_leave(ctx, s)) return rl;
    if (tp && rc == RTW_OK) rc = harvest_timing(ctx, T, opts->timing);
    if (rc) return rc;
    if (!(opts && (opts->flags & RTW_RENDER_NO_SYNC))) HIP_TRY(hipStreamSynchronize(s));
    return RTW_OK;
}

}  // namespace

extern "C" {

int rtw_render(rtw_ctx* ctx, const rtw_camera* cam, uint32_t pix_begin, uint32_t pix_end, uint32_t spp_begin,
               uint32_t spp_end, uint64_t seed, float* accum, const volatile int32_t* cancel,
               rtw_progress_fn progress, void* user) {
    rtw_render_opts o{};
    o.cancel = cancel;
    o.progress = progress;
    o.user = user;
    return rtw_render_ex(ctx, cam, pix_begin, pix_end, spp_begin, spp_end, seed, accum, &o);
}

int rtw_render_ex(rtw_ctx* ctx, const rtw_camera* cam, uint32_t pix_begin, uint32_t pix_end, uint32_t spp_begin,
                  uint32_t spp_end, uint64_t seed, float* accum, const rtw_render_opts* opts) {
    if (!ctx || !accum) return fail(RTW_E_INVALID, "null ctx/accum");
    if (int rc = validate_cam(cam)) return rc;
    if (int rc = check_host_opts(opts)) return rc;
    if (pix_end > cam->size || pix_begin > pix_end) return fail(RTW_E_INVALID, "pixel range out of image");
    if (spp_begin > spp_end) return fail(RTW_E_INVALID, "bad sample range");
    if (pix_begin == pix_end || spp_begin == spp_end) return RTW_OK;
    const uint32_t ubatch = opts ? opts->spp_batch : 0u;
    if (ctx->device == RTW_DEVICE_CPU) {  // host context: Camera.render on host threads (rtw_cpu.hip)
        rtw_launch L;
        {
            std::lock_guard<std::mutex> lock(ctx->mu);
            L = make_launch(ctx, cam, seed);
        }
        // the scene image is read-only: concurrent callers (the 8 Tasks) render their ranges at once
        L.n_shards = 0;
        return run_host(ctx, L, pix_begin, pix_end, spp_begin, spp_end, ubatch, accum, opts, pix_end - pix_begin);
    }
    // GPU context.  The context lock is held only while a call enqueues work, never while it waits for
    // the device, so concurrent callers -- the reference's 8 Tasks on disjoint chunks (main.zig:314-326)
    // -- interleave their spp batches on the context's stream and advance samples-outer together, as
    // the 8 workers of camera.zig:98-111 do.  Each call stages only its own chunk of the shared
    // full-frame device buffer, so the chunks never overlap.
    const size_t bytes = (size_t)cam->size * 16;
    const size_t o = (size_t)pix_begin * 16, nb = (size_t)(pix_end - pix_begin) * 16;
    const uint64_t pixels = pix_end - pix_begin;
    hipEvent_t done = nullptr;
    uint32_t batch = 0;
    {
        std::unique_lock<std::mutex> lock(ctx->mu);
        HIP_TRY(hipSetDevice(ctx->device));
        // the staging buffer grows only while no other host-buffer call has a chunk staged in it
        ctx->host_cv.wait(lock, [&] { return ctx->scratch_bytes >= bytes || ctx->host_calls == 0; });
        if (int rc = stream_enter(ctx, ctx->stream)) return rc;
        if (int rc = ensure_scratch(ctx, bytes)) return rc;
        HIP_TRY(hipMemcpyAsync((char*)ctx->d_scratch + o, (char*)accum + o, nb, hipMemcpyHostToDevice, ctx->stream));
        if (int rc = stream_leave(ctx, ctx->stream)) return rc;
        HIP_TRY(hipEventCreateWithFlags(&done, hipEventDisableTiming));  // (last: no early return leaks it)
        ctx->host_calls++;
        batch = ubatch ? ubatch : auto_batch(ctx, pixels, spp_end - spp_begin);
    }
    const bool polled = rtw_polled(opts);
    const uint64_t total = pixels * (uint64_t)(spp_end - spp_begin);
    int rc = RTW_OK;
    for (uint32_t s = spp_begin; s < spp_end && rc == RTW_OK; s += batch) {
        if (rtw_stop_requested(opts)) {
            rc = fail(RTW_E_CANCELLED, "cancelled");
            break;
        }
        const uint32_t s_end = (spp_end - s < batch) ? spp_end : s + batch;
        {
            std::lock_guard<std::mutex> lock(ctx->mu);
            if (hipSetDevice(ctx->device) != hipSuccess || stream_enter(ctx, ctx->stream)) {
                rc = fail(RTW_E_HIP, "rtw_render_ex: device");
                break;
            }
            rtw_launch L = make_launch(ctx, cam, seed);
            L.accum = reinterpret_cast<float4*>(ctx->d_scratch);
            L.pix_begin = pix_begin;
            L.pix_end = pix_end;
            L.row0 = pix_begin / cam->image_width;
            L.n_rows = (pix_end - 1) / cam->image_width - L.row0 + 1;
            L.n_shards = 0;
            L.counters = nullptr;
            set_tiles(L);
            rc = run_batches(ctx, L, s, s_end, s_end - s, ctx->stream, nullptr, pixels);
            if (rc == RTW_OK) rc = stream_leave(ctx, ctx->stream);
            if (rc == RTW_OK && hipEventRecord(done, ctx->stream) != hipSuccess) rc = fail(RTW_E_HIP, "event");
        }
        if (rc == RTW_OK && polled) {  // wait for this batch without the lock, then report it
            if (hipEventSynchronize(done) != hipSuccess) rc = fail(RTW_E_HIP, "rtw_render_ex: batch");
            else if (opts->progress && opts->progress(pixels * (uint64_t)(s_end - spp_begin), total, opts->user))
                rc = fail(RTW_E_CANCELLED, "cancelled by progress callback");
        }
    }
    // copy back whatever was rendered (also on cancel: completed batches are valid)
    hipError_t e;
    {
        std::lock_guard<std::mutex> lock(ctx->mu);
        e = hipSetDevice(ctx->device);
        if (e == hipSuccess && ctx->last_stream && ctx->last_stream != ctx->stream)
            e = hipStreamWaitEvent(ctx->stream, ctx->last_done, 0);
        if (e == hipSuccess)
            e = hipMemcpyAsync((char*)accum + o, (char*)ctx->d_scratch + o, nb, hipMemcpyDeviceToHost, ctx->stream);
        if (e == hipSuccess) e = hipEventRecord(done, ctx->stream);
        if (e == hipSuccess) (void)stream_leave(ctx, ctx->stream);
    }
    if (e == hipSuccess) e = hipEventSynchronize(done);
    (void)hipEventDestroy(done);
    {
        std::lock_guard<std::mutex> lock(ctx->mu);
        ctx->host_calls--;
    }
    ctx->host_cv.notify_all();
    if (e != hipSuccess) return hip_fail(e, "rtw_render copy back");
    return rc;
}

int rtw_render_device(rtw_ctx* ctx, const rtw_camera* cam, uint32_t pix_begin, uint32_t pix_end, uint32_t spp_begin,
                      uint32_t spp_end, uint64_t seed, float* d_accum, void* stream, const rtw_render_opts* opts) {
    if (!ctx || !d_accum) return fail(RTW_E_INVALID, "null ctx/accum");
    if (ctx->device == RTW_DEVICE_CPU) return fail(RTW_E_INVALID, "host context: use rtw_render");
    if (int rc = validate_cam(cam)) return rc;
    if (pix_end > cam->size || pix_begin > pix_end) return fail(RTW_E_INVALID, "pixel range out of image");
    if (spp_begin > spp_end) return fail(RTW_E_INVALID, "bad sample range");
    if (pix_begin == pix_end || spp_begin == spp_end) return RTW_OK;
    std::lock_guard<std::mutex> lock(ctx->mu);
    HIP_TRY(hipSetDevice(ctx->device));
    hipStream_t s = stream ? (hipStream_t)stream : ctx->stream;
    if (int rc = stream_enter(ctx, s)) return rc;
    rtw_launch L = make_launch(ctx, cam, seed);
    L.accum = reinterpret_cast<float4*>(d_accum);
    L.pix_begin = pix_begin;
    L.pix_end = pix_end;
    L.row0 = pix_begin / cam->image_width;
    L.n_rows = (pix_end - 1) / cam->image_width - L.row0 + 1;
    L.n_shards = 0;
    L.counters = opts ? reinterpret_cast<unsigned long long*>(opts->counters) : nullptr;
    set_tiles(L);
    uint32_t batch = opts && opts->spp_batch ? opts->spp_batch : auto_batch(ctx, pix_end - pix_begin, spp_end - spp_begin);
    rtw_timer T;
    T.stream = s;
    T.pool.swap(ctx->ev_pool);
    rtw_timer* tp = (opts && opts->timing) ? &T : nullptr;
    int rc = run_batches(ctx, L, spp_begin, spp_end, batch, s, opts, pix_end - pix_begin, tp);
    ctx->ev_pool.swap(T.pool);
    if (int rl = stream_leave(ctx, s)) return rl;
    if (tp && rc == RTW_OK) rc = harvest_timing(ctx, T, opts->timing);
    if (rc) return rc;
    if (!(opts && (opts->flags & RTW_RENDER_NO_SYNC))) HIP_TRY(hipStreamSynchronize(s));
    return RTW_OK;
}

uint32_t rtw_shard_rows(uint32_t H, uint32_t rpb, uint32_t n_shards, uint32_t shard) {
    if (!(rpb & ~RTW_ROWS_FLAGS) || !n_shards || shard >= n_shards) return 0;
    uint32_t rows = 0;
    const uint32_t t = rtw_shard_tile_rows(H, rpb, n_shards, shard);
    for (uint32_t r = 0; r < t; r++) rows += rtw_shard_row(H, rpb, n_shards, shard, r) < H ? 1u : 0u;
    return rows;
}

uint32_t rtw_shard_image_row(uint32_t rpb, uint32_t n_shards, uint32_t shard, uint32_t tile_row) {
    if (!rpb || (rpb & RTW_ROWS_FLAGS) || !n_shards || shard >= n_shards) return 0xFFFFFFFFu;
    return rtw_tile_row_image(rpb, n_shards, shard, tile_row);
}

uint32_t rtw_shard_image_row_h(uint32_t H, uint32_t rpb, uint32_t n_shards, uint32_t shard, uint32_t tile_row) {
    if (!(rpb & ~RTW_ROWS_FLAGS) || !n_shards || shard >= n_shards) return 0xFFFFFFFFu;
    return rtw_shard_row(H, rpb, n_shards, shard, tile_row);
}

int rtw_render_rows_device(rtw_ctx* ctx, const rtw_camera* cam, uint32_t rpb, uint32_t n_shards, uint32_t shard,
                           uint32_t spp_begin, uint32_t spp_end, uint64_t seed, float* d_tile, void* stream,
                           const rtw_render_opts* opts) {
    if (!ctx || !d_tile) return fail(RTW_E_INVALID, "null ctx/tile");
    if (ctx->device == RTW_DEVICE_CPU) return fail(RTW_E_INVALID, "host context: use rtw_render_rows");
    if (int rc = validate_cam(cam)) return rc;
    if (!(rpb & ~RTW_ROWS_FLAGS) || !n_shards || shard >= n_shards) return fail(RTW_E_INVALID, "bad shard spec");
    if (spp_begin > spp_end) return fail(RTW_E_INVALID, "bad sample range");
    const uint32_t rows = rtw_shard_rows(cam->image_height, rpb, n_shards, shard);
    if (rows == 0 || spp_begin == spp_end) return RTW_OK;
    std::lock_guard<std::mutex> lock(ctx->mu);
    HIP_TRY(hipSetDevice(ctx->device));
    hipStream_t s = stream ? (hipStream_t)stream : ctx->stream;
    if (int rc = stream_enter(ctx, s)) return rc;
    return render_rows_locked(ctx, cam, rpb, n_shards, shard, spp_begin, spp_end, seed, d_tile, s, opts, rows);
}

int rtw_render_rows(rtw_ctx* ctx, const rtw_camera* cam, uint32_t rpb, uint32_t n_shards, uint32_t shard,
                    uint32_t spp_begin, uint32_t spp_end, uint64_t seed, float* tile, const rtw_render_opts* opts) {
    if (!ctx || !tile) return fail(RTW_E_INVALID, "null ctx/tile");
    if (int rc = validate_cam(cam)) return rc;
    if (int rc = check_host_opts(opts)) return rc;
    if (!(rpb & ~RTW_ROWS_FLAGS) || !n_shards || shard >= n_shards) return fail(RTW_E_INVALID, "bad shard spec");
    if (spp_begin > spp_end) return fail(RTW_E_INVALID, "bad sample range");
    const uint32_t rows = rtw_shard_rows(cam->image_height, rpb, n_shards, shard);
    if (rows == 0 || spp_begin == spp_end) return RTW_OK;
    std::lock_guard<std::mutex> lock(ctx->mu);
    const uint32_t W = cam->image_width;
    if (ctx->device == RTW_DEVICE_CPU) {  // the shard on host threads (rtw_cpu.hip), tile rows in order
        rtw_launch L = make_launch(ctx, cam, seed);
        L.rpb = rpb;
        L.n_shards = n_shards;
        L.shard = shard;
        return run_host(ctx, L, 0, rows * W, spp_begin, spp_end, opts ? opts->spp_batch : 0u, tile, opts,
                        (uint64_t)rows * W);
    }
    HIP_TRY(hipSetDevice(ctx->device));
    if (int rc = stream_enter(ctx, ctx->stream)) return rc;
    // the tile is staged in its own buffer, never in d_scratch: rtw_render_ex calls on this context release
    // the lock between batches with their chunks staged there
    const size_t nb = (size_t)rows * W * 16;
    if (ctx->rows_bytes < nb) {
        if (ctx->d_rows) {
            HIP_TRY(hipStreamSynchronize(ctx->stream));
            (void)hipFree(ctx->d_rows);
        }
        ctx->d_rows = nullptr;
        ctx->rows_bytes = 0;
        HIP_TRY(hipMalloc(&ctx->d_rows, nb));
        ctx->rows_bytes = nb;
    }
    HIP_TRY(hipMemcpyAsync(ctx->d_rows, tile, nb, hipMemcpyHostToDevice, ctx->stream));
    rtw_render_opts ctl{};
    if (opts) ctl = *opts;
    int rc = render_rows_locked(ctx, cam, rpb, n_shards, shard, spp_begin, spp_end, seed, ctx->d_rows, ctx->stream,
                                &ctl, rows);
    hipError_t e = hipMemcpyAsync(tile, ctx->d_rows, nb, hipMemcpyDeviceToHost, ctx->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
    if (e != hipSuccess) return hip_fail(e, "rtw_render_rows copy back");
    ctx->last_stream = nullptr;  // synchronised
    return rc;
}

int rtw_texture_from_accum(const float* accum, uint32_t n, uint8_t* out) {
#pragma STDC FP_CONTRACT OFF
    if (!accum || !out) return fail(RTW_E_INVALID, "null buffer");
    for (uint32_t i = 0; i < n; i++) {
        const float* px = accum + 4 * (size_t)i;
        const float scale = 1.0f / px[3];
        for (int k = 0; k < 3; k++) {
            float x = std::sqrt(px[k] * scale);
            if (x < 0.0f) x = 0.0f;
            if (x > 0.999f) x = 0.999f;
            out[4 * (size_t)i + k] = (x == x) ? (uint8_t)(256 * x) : 0;  // NaN (UB in the reference): 0
        }
        out[4 * (size_t)i + 3] = 255;
    }
    return RTW_OK;
}

int rtw_debug_rng(rtw_ctx* ctx, uint64_t seed, uint32_t pixel, uint32_t sample, uint32_t n, float* out) {
    if (!ctx || !out || n > 64) return fail(RTW_E_INVALID, "bad debug_rng args (n <= 64)");
    if (ctx->device == RTW_DEVICE_CPU) return fail(RTW_E_INVALID, "host context");
    std::lock_guard<std::mutex> lock(ctx->mu);
    HIP_TRY(hipSetDevice(ctx->device));
    if (int rc = stream_enter(ctx, ctx->stream)) return rc;
    ctx->last_stream = nullptr;  // synchronised below
    rtw_launch_debug_rng(seed, pixel, sample, n, ctx->d_dbg, ctx->stream);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipMemcpyAsync(out, ctx->d_dbg, n * sizeof(float), hipMemcpyDeviceToHost, ctx->stream));
    HIP_TRY(hipStreamSynchronize(ctx->stream));
    return RTW_OK;
}

int rtw_debug_sample(rtw_ctx* ctx, const rtw_camera* cam, uint64_t seed, uint32_t pixel, uint32_t sample,
                     float out[3]) {
    if (!ctx || !out) return fail(RTW_E_INVALID, "null args");
    if (ctx->device == RTW_DEVICE_CPU) return fail(RTW_E_INVALID, "host context");
    if (int rc = validate_cam(cam)) return rc;
    if (pixel >= cam->size) return fail(RTW_E_INVALID, "pixel out of range");
    std::lock_guard<std::mutex> lock(ctx->mu);
    HIP_TRY(hipSetDevice(ctx->device));
    if (int rc = stream_enter(ctx, ctx->stream)) return rc;
    ctx->last_stream = nullptr;  // synchronised below
    rtw_launch L = make_launch(ctx, cam, seed);
    rtw_launch_debug_sample(L, pixel, sample, ctx->d_dbg, ctx->stream);
    HIP_TRY(hipGetLastError());
    float tmp[32];
    HIP_TRY(hipMemcpyAsync(tmp, ctx->d_dbg, sizeof tmp, hipMemcpyDeviceToHost, ctx->stream));
    HIP_TRY(hipStreamSynchronize(ctx->stream));
    out[0] = tmp[0];
    out[1] = tmp[1];
    out[2] = tmp[2];
    return RTW_OK;
}

}  // extern "C"
