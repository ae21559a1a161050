// rtw_wavefront.hip -- v2: wavefront path tracing (the default kernel path).
//
// The megakernels (v0/v1, rtw_kernels.hip) keep a whole path in registers, so
// the BVH walk -- 60 % of their time -- runs at the occupancy the shading code
// allows (~100 VGPRs, 4 waves/SIMD).  Measured on MI355X (diag/trav_bench.hip)
// the same walk in a ~40-VGPR kernel runs 4-6x more node steps per second.
// v2 therefore splits a batch of paths into kernels over HBM-resident SoA state:
//
//   gen    (pixel, sample) -> camera ray           Camera.getRay  camera.zig:169-180
//   trace  ray -> closest hit (t, leaf)            BVHNode.hit    bvh.zig:122-136
//   shade  hit -> emission/background, scatter     rayColor       camera.zig:182-208
//          (survivors appended to the next queue)
//   tail   the few paths still alive after RTW_WF_ITERS bounces, to completion
//   reduce per pixel: accum += sample radiances in sample order (camera.zig:55-56)
//
// A batch holds n_pix logical pixels x n_s samples; path p = s_local * n_pix + q,
// q in 8x8 pixel tiles so a wave's primary rays are one tile.  Every path runs
// the same operations in the same order as in v0/v1 (same RNG stream, same
// iterative radiance), and the reduce adds the samples of a pixel in sample
// order onto the accumulator, so v2 is bit-identical to v0/v1.
#include "rtw_device.h"
#include "rtw_wavefront.h"

namespace {

// logical pixel q of the batch -> image pixel / output slot (false = padding)
__device__ __forceinline__ bool wf_pixel(const rtw_launch& L, const rtw_wf& W, uint32_t q, uint32_t& pixel,
                                         uint32_t& out_idx, uint32_t& x, uint32_t& y) {
    const uint32_t tile = q >> 6, k = q & 63u;
    x = (tile % W.n_tx) * 8u + (k & 7u);
    const uint32_t r = L.row0 + (tile / W.n_tx) * 8u + (k >> 3);
    if (x >= L.W || r >= L.row0 + L.n_rows) return false;
    if (!map_row(L, r, y)) return false;
    pixel = y * L.W + x;
    if (!L.n_shards && (pixel < L.pix_begin || pixel >= L.pix_end)) return false;
    out_idx = r * L.W + x;
    return true;
}

// Entry k of segment g at iteration it -> path id (false: padding or no path).
// Iteration 0 deals 64-path chunks round-robin (chunk c -> segment c % SEGS).
__device__ __forceinline__ bool wf_entry(const rtw_wf& W, uint32_t it, uint32_t g, uint32_t k, uint32_t& p) {
    if (it == 0) {
        p = (((k >> 6) * RTW_WF_SEGS + g) << 6) | (k & 63u);
        return p < W.n_paths;
    }
    p = W.queue[it & 1u][(size_t)g * W.seg_cap + k];
    return true;
}

__device__ __forceinline__ uint32_t wf_seg_len(const rtw_wf& W, uint32_t it, uint32_t g) {
    return it == 0 ? W.seg_cap : W.seg_len[it & 1u][g];
}

__device__ __forceinline__ uint32_t wf_wave() { return blockIdx.x * 4u + (threadIdx.x >> 6); }
__device__ __forceinline__ uint32_t wf_nwaves() { return gridDim.x * 4u; }

__device__ __forceinline__ Ray wf_load_ray(const rtw_wf& W, uint32_t p, uint32_t& depth) {
    const float4 o = W.ray_o[p], d = W.ray_d[p];
    Ray r;
    r.o = mk(o.x, o.y, o.z);
    r.time = o.w;
    r.d = mk(d.x, d.y, d.z);
    depth = fbits(d.w);
    return r;
}

__device__ __forceinline__ void wf_store_ray(const rtw_wf& W, uint32_t p, const Ray& r, uint32_t depth) {
    W.ray_o[p] = make_float4(r.o.x, r.o.y, r.o.z, r.time);
    W.ray_d[p] = make_float4(r.d.x, r.d.y, r.d.z, __uint_as_float(depth));
}

template <uint32_t FEAT>
__global__ __launch_bounds__(256) void wf_gen(rtw_launch L, rtw_wf W) {
    const uint32_t p = blockIdx.x * 256u + threadIdx.x;
    if (p >= W.n_paths) return;
    const uint32_t s_local = p / W.n_pix, q = p - s_local * W.n_pix;
    uint32_t pixel, out_idx, x, y;
    W.ls[p] = make_float4(0, 0, 0, 0);
    if (wf_pixel(L, W, q, pixel, out_idx, x, y) && L.max_depth > 0) {
        const uint32_t s = L.s0 + s_local;
        rtw_rng rng;
        rng.s = rtw_mix64(L.key0 ^ (((uint64_t)pixel << 32) | (uint64_t)s));
        const Ray r = get_ray(L, x + L.pixel_offset, y + L.pixel_offset, rng);  // camera.zig:100-101
        wf_store_ray(W, p, r, L.max_depth);
        W.thr[p] = make_float4(1, 1, 1, 0);
        W.rng[p] = rng.s;
    } else {
        W.ray_d[p] = make_float4(0, 0, 0, 0);  // depth 0: no path (padding / outside the range)
    }
}

// trace: closest hit per queued ray (no shading state in registers)
template <uint32_t FEAT>
__global__ __launch_bounds__(256) void wf_trace(rtw_launch L, rtw_wf W, uint32_t it) {
    Counters cnt;
    for (uint32_t g = wf_wave(); g < RTW_WF_SEGS; g += wf_nwaves()) {
        const uint32_t n = wf_seg_len(W, it, g);
        for (uint32_t k = __lane_id(); k - __lane_id() < n; k += 64) {
            uint32_t p;
            if (k < n && wf_entry(W, it, g, k, p)) {
                uint32_t depth;
                const Ray r = wf_load_ray(W, p, depth);
                if (depth) {
                    float t;
                    const int h = traverse<FEAT>(L.nodes, L, r, t, cnt);
                    W.hit[p] = make_float2(t, __int_as_float(h));
                    cnt.rays++;
                }
            }
        }
    }
    flush_counters(L, cnt, 0);
}

// shade: emission / background and Material.scatter; survivors -> the same
// segment of the next queue, compacted with a ballot prefix (no atomics)
template <uint32_t FEAT>
__global__ __launch_bounds__(256) void wf_shade(rtw_launch L, rtw_wf W, uint32_t it) {
    uint32_t* next = W.queue[(it + 1u) & 1u];
    const uint32_t lane = __lane_id();
    const uint64_t lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
    for (uint32_t g = wf_wave(); g < RTW_WF_SEGS; g += wf_nwaves()) {
        const uint32_t n = wf_seg_len(W, it, g);
        uint32_t* out = next + (size_t)g * W.seg_cap;
        uint32_t n_out = 0;
        for (uint32_t k = lane; k - lane < n; k += 64) {
            bool push = false;
            uint32_t p = 0;
            if (k < n && wf_entry(W, it, g, k, p)) {
                uint32_t depth;
                const Ray r = wf_load_ray(W, p, depth);
                if (depth) {
                    const float2 h = W.hit[p];
                    const int hit = __float_as_int(h.y);
                    const float4 t4 = W.thr[p], l4 = W.ls[p];
                    f3 thr = mk(t4.x, t4.y, t4.z), acc = mk(l4.x, l4.y, l4.z);
                    if (hit < 0) {
                        acc = acc + thr * background(L, r);
                    } else {
                        rtw_rng rng;
                        rng.s = W.rng[p];
                        f3 att;
                        Ray sc;
                        if (shade<FEAT>(L.nodes, L, r, hit, h.x, rng, thr, acc, att, sc) && depth > 1) {
                            wf_store_ray(W, p, sc, depth - 1);
                            thr = thr * att;
                            W.thr[p] = make_float4(thr.x, thr.y, thr.z, 0);
                            W.rng[p] = rng.s;
                            push = true;
                        }
                    }
                    W.ls[p] = make_float4(acc.x, acc.y, acc.z, 0);
                }
            }
            const uint64_t m = __ballot(push);
            if (push) out[n_out + (uint32_t)__popcll(m & lt)] = p;
            n_out += (uint32_t)__popcll(m);
        }
        if (lane == 0) W.seg_len[(it + 1u) & 1u][g] = n_out;
    }
}

// tail: the paths still queued after the last wavefront iteration, each to completion
template <uint32_t FEAT>
__global__ __launch_bounds__(256) void wf_tail(rtw_launch L, rtw_wf W, uint32_t it) {
    Counters cnt;
    for (uint32_t g = wf_wave(); g < RTW_WF_SEGS; g += wf_nwaves()) {
        const uint32_t n = wf_seg_len(W, it, g);
        for (uint32_t k = __lane_id(); k - __lane_id() < n; k += 64) {
            uint32_t p;
            if (k < n && wf_entry(W, it, g, k, p)) {
                uint32_t depth;
                Ray r = wf_load_ray(W, p, depth);
                const float4 t4 = W.thr[p], l4 = W.ls[p];
                f3 thr = mk(t4.x, t4.y, t4.z), acc = mk(l4.x, l4.y, l4.z);
                rtw_rng rng;
                rng.s = W.rng[p];
                for (; depth > 0; depth--) {  // the rest of rayColor's iterations
                    cnt.rays++;
                    float t;
                    const int hit = traverse<FEAT>(L.nodes, L, r, t, cnt);
                    if (hit < 0) {
                        acc = acc + thr * background(L, r);
                        break;
                    }
                    f3 att;
                    Ray sc;
                    if (!shade<FEAT>(L.nodes, L, r, hit, t, rng, thr, acc, att, sc)) break;
                    thr = thr * att;
                    r = sc;
                }
                W.ls[p] = make_float4(acc.x, acc.y, acc.z, 0);
            }
        }
    }
    flush_counters(L, cnt, 0);
}

// reduce: accum[pixel] += radiance of samples s0.. in sample order; .w = sample count
__global__ __launch_bounds__(256) void wf_reduce(rtw_launch L, rtw_wf W) {
    const uint32_t q = blockIdx.x * 256u + threadIdx.x;
    Counters cnt;
    uint32_t samples = 0;
    if (q < W.n_pix) {
        uint32_t pixel, out_idx, x, y;
        if (wf_pixel(L, W, q, pixel, out_idx, x, y)) {
            float4 a = L.accum[out_idx];
            for (uint32_t s = 0; s < W.n_s; s++) {
                const float4 c = W.ls[(size_t)s * W.n_pix + q];
                if (is_nan3(mk(c.x, c.y, c.z))) cnt.nans++;
                a.x += c.x;
                a.y += c.y;
                a.z += c.z;
            }
            a.w = (float)(L.s0 + W.n_s);  // writeColor: buffer[i][3] = number_of_samples (camera.zig:56)
            L.accum[out_idx] = a;
            samples = W.n_s;
        }
    }
    flush_counters(L, cnt, samples);
}

template <typename K>
uint32_t wf_resident(K kernel, int n_cu) {
    int b = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, kernel, 256, 0) != hipSuccess || b < 1) b = 1;
    return (uint32_t)(b * n_cu);
}

template <uint32_t FEAT>
void wf_run(const rtw_launch& L, const rtw_wf& W, hipStream_t st, int n_cu) {
    // grids = resident blocks (each wave then walks SEGS / waves segments)
    static const uint32_t g_trace = wf_resident(wf_trace<FEAT>, n_cu);
    static const uint32_t g_shade = wf_resident(wf_shade<FEAT>, n_cu);
    static const uint32_t g_tail = wf_resident(wf_tail<FEAT>, n_cu);
    hipLaunchKernelGGL(wf_gen<FEAT>, dim3((W.n_paths + 255u) / 256u), dim3(256), 0, st, L, W);
    const uint32_t iters = L.max_depth < W.iters ? L.max_depth : W.iters;
    for (uint32_t it = 0; it < iters; it++) {
        hipLaunchKernelGGL(wf_trace<FEAT>, dim3(g_trace), dim3(256), 0, st, L, W, it);
        hipLaunchKernelGGL(wf_shade<FEAT>, dim3(g_shade), dim3(256), 0, st, L, W, it);
    }
    if (iters < L.max_depth) hipLaunchKernelGGL(wf_tail<FEAT>, dim3(g_tail), dim3(256), 0, st, L, W, iters);
    hipLaunchKernelGGL(wf_reduce, dim3((W.n_pix + 255u) / 256u), dim3(256), 0, st, L, W);
}

uint32_t wf_pick_feat(uint32_t f) {
    if ((f & ~RTW_F_CHECKER) == 0) return f ? RTW_F_CHECKER : 0u;
    return RTW_F_ALL;
}

}  // namespace

void rtw_wavefront_batch(const rtw_launch& L, const rtw_wf& W, void* stream, int n_cu) {
    hipStream_t st = (hipStream_t)stream;
    switch (wf_pick_feat(L.feat)) {
    case 0u: wf_run<0u>(L, W, st, n_cu); break;
    case RTW_F_CHECKER: wf_run<RTW_F_CHECKER>(L, W, st, n_cu); break;
    default: wf_run<RTW_F_ALL>(L, W, st, n_cu); break;
    }
}
