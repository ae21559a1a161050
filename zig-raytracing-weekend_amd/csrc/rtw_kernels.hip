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
#include "rtw_device.h"

namespace {

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
//  * the BVH (<= RTW_MEGA_LDS_NODES_MAX nodes) is staged once per block in LDS.
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
    const float4* nb = nodes;  // this lane's node array (octant copy, order_base)
    uint32_t oct = 0;
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
        // per lane, the defocus-disk rejection loop, then time.
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
            if (defocus && starting) seq_reject<2>(rng, dsk);
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
                    rt = ray_trav(ray, L.fast_box != 0);
                    oct = order_of(L, ray);
                    nb = order_base(nodes, L, oct);
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
                        ti = trav_step<FEAT>(nb, L, ray, rt, ti, closest, hit, cnt, rng.s);
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
        // randomUnitVector rejection loop of the lanes that need it, then the material.
        {
            const bool shading = st == ST_SHADE;
            HitPrep hp;
            bool need_uv = false;
            if (shading && hit >= 0) {
                hp = hit_prep<FEAT>(nodes, L, ray, hit_with_order(hit, oct), closest);
                need_uv = needs_unit_vector<FEAT>(hp.m.kind);
            }
            float ruv3[3] = {0.0f, 0.0f, 0.0f};
            if (need_uv) seq_reject<3>(rng, ruv3);
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
                        rt = ray_trav(ray, L.fast_box != 0);
                        oct = order_of(L, ray);
                    nb = order_base(nodes, L, oct);
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
    for (uint32_t k = 0; k < n; k++) out[k] = rtw_path_float(r);
}

// Diagnostic: for every bounce of one sample, brute-force all leaves with the
// exact test and with the fast-reject filter; record the first leaf the filter
// would wrongly reject (out[8..]).
__device__ void debug_filter_check(const rtw_launch& L, const Ray& r, float* out) {
    const RayTrav rt = ray_trav(r, L.fast_box != 0);
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
        const int hit = traverse<RTW_F_ALL>(L.nodes, L, r, t, cnt, rng.s);
        // brute-force exact closest over all leaves
        {
            const RayTrav rt = ray_trav(r, L.fast_box != 0);
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

uint32_t pick_feat(uint32_t f) {
    if ((f & ~RTW_F_CHECKER) == 0) return f ? RTW_F_CHECKER : 0u;
    return RTW_F_ALL;
}


// (launch-bound variants forcing 6 or 8 waves/SIMD spilled and were slower: removed)
template <uint32_t FEAT, bool LDS>
void launch_waves(const rtw_launch& L, hipStream_t st, int grid, int) {
    launch_v1<FEAT, LDS, 1>(L, st, grid);
}
template <uint32_t FEAT, bool LDS>
int occ_waves(size_t lds, int) {
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
    const bool lds = L.n_nodes <= RTW_MEGA_LDS_NODES_MAX && L.use_lds;
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
    const bool lds = n_nodes <= RTW_MEGA_LDS_NODES_MAX && use_lds;
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
