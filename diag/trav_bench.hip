// DIAGNOSTIC ONLY (not the product): the walk ceiling of the compact LDS walk.
//
// A kernel that does nothing but the product's compact-node walk (traverse_compact<.., LDS>, rtw_device.h)
// over the scene's own LDS stage -- same node forms, same 1024-thread block per CU, no path state, no
// shading, no queues -- on C2's rays: camera rays of 8x8 tiles (Camera.getRay with jitter and defocus, as
// the product draws them) and, with `bounce`, one diffuse bounce from each hit (n + a random unit vector).
// Its node-steps per second (inner boxes + sphere tests) is the rate the walk code reaches when nothing else
// shares the CU: bench.py prices the product's device node visits per second against it (roofline.walk).
//
// Built into build/rtw_trav.so with the product objects (csrc/Makefile `trav`), so it walks the same
// stage the product stages; driven by diag/run_walk_ceiling.py.
#include "../zig-raytracing-weekend_amd/csrc/rtw_device.h"

namespace {

template <int CN>
__global__ __launch_bounds__(1024) void walk_ceiling(rtw_launch L, uint32_t rays_per_lane, uint32_t bounce,
                                                     unsigned long long* out) {
    extern __shared__ uint4 lds[];
    {   // the product's stage (rtw_wavefront.hip stage_clds): skip offsets rebased to LDS addresses
        const uint32_t q = L.cnode32 ? 2u : 1u, n4 = L.n_nodes * L.n_orders * q, lb = lds_addr(lds);
        for (uint32_t k = threadIdx.x; k < n4; k += blockDim.x) {
            uint4 c = L.cnodes[k];
            if (L.cnode32) {
                if ((k & 1u) && !(c.z & RTW_LEAF_BIT)) c.z += lb;
            } else if (!(c.w & RTW_LEAF_BIT)) {
                c.w += lb;
            }
            lds[k] = c;
        }
        __syncthreads();
    }
    Counters cnt;
    const uint32_t lane = threadIdx.x & 63u, wave = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    const uint32_t nw = gridDim.x * (blockDim.x >> 6), ntx = (L.W + 7u) / 8u, nt = ntx * ((L.H + 7u) / 8u);
    float acc = 0.0f;
    uint32_t walks = 0;
    for (uint32_t k = 0; k < rays_per_lane; k++) {
        const uint32_t tile = (wave + k * nw) % nt;
        const uint32_t x = min((tile % ntx) * 8u + (lane & 7u), L.W - 1u), y = min((tile / ntx) * 8u + (lane >> 3), L.H - 1u);
        rtw_rng rng;
        rng.s = rtw_mix64(L.key0 ^ (((uint64_t)(y * L.W + x) << 32) | k));
        Ray r = get_ray(L, x + 1u, y + 1u, rng);
        float t;
        constexpr bool Y4 = CN != 0, F32 = CN == 2;
        int h = traverse_compact<true, true, Y4, F32>(L, lds, r, t, cnt);
        walks++;
        if (bounce && h >= 0) {
            const float4* nb = order_base(L.nodes, L, (uint32_t)h >> RTW_HIT_NODE_BITS);
            const uint32_t i = (uint32_t)h & ((1u << RTW_HIT_NODE_BITS) - 1u);
            const float4 A = nb[2u * i], B = nb[2u * i + 1u];
            const f3 p = r.o + splat(t) * r.d;
            const f3 n = divs(p - mk(A.x, A.y, A.z), B.x);
            const uint64_t hs = rtw_mix64(rng.s);
            const f3 u = mk((float)(hs & 0xFFFFFu) * (2.0f / 1048576.0f) - 1.0f,
                            (float)((hs >> 20) & 0xFFFFFu) * (2.0f / 1048576.0f) - 1.0f,
                            (float)((hs >> 40) & 0xFFFFFu) * (2.0f / 1048576.0f) - 1.0f);
            Ray r2;
            r2.o = p;
            r2.d = n + divs(u, __builtin_sqrtf(length_squared(u)) + 1e-6f);
            r2.time = 0.0f;
            h = traverse_compact<true, true, Y4, F32>(L, lds, r2, t, cnt);
            walks++;
        }
        acc += h >= 0 ? t : 0.0f;
    }
    if (acc == 12345.0f) out[7] = 1;  // keep the walks live
    atomicAdd(&out[0], (unsigned long long)cnt.nodes);
    atomicAdd(&out[1], (unsigned long long)cnt.leaves);
    atomicAdd(&out[2], (unsigned long long)walks);
}

}  // namespace

// out (device, 8 x u64, zeroed by the caller): [0] inner-node steps, [1] sphere tests, [2] walks; *ms: kernel time
extern "C" int rtw_diag_walk_ceiling(rtw_ctx* ctx, const rtw_camera* cam, uint32_t rays_per_lane, uint32_t bounce,
                                     unsigned long long* d_out, float* ms, uint32_t* grid_out) {
    rtw_launch L = ctx->base;
    if (!L.cnodes || !cam) return RTW_E_INVALID;
    for (int k = 0; k < 3; k++) {
        L.center[k] = cam->center[k];
        L.pixel00[k] = cam->pixel00_loc[k];
        L.du[k] = cam->pixel_delta_u[k];
        L.dv[k] = cam->pixel_delta_v[k];
        L.disk_u[k] = cam->defocus_disk_u[k];
        L.disk_v[k] = cam->defocus_disk_v[k];
    }
    L.defocus_angle = cam->defocus_angle;
    L.W = cam->image_width;
    L.H = cam->image_height;
    L.key0 = rtw_mix64(0);
    const size_t lds = (size_t)L.n_nodes * L.n_orders * (L.cnode32 ? 32u : 16u);
    const int cn = L.cnode32 ? 2 : L.n_orders == 4 ? 1 : 0;
    auto kern = cn == 2 ? walk_ceiling<2> : cn == 1 ? walk_ceiling<1> : walk_ceiling<0>;
    int b = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, kern, 1024, lds) != hipSuccess || b < 1) b = 1;
    const uint32_t grid = (uint32_t)(b * ctx->n_cu);
    if (grid_out) *grid_out = grid;
    hipEvent_t e0, e1;
    (void)hipSetDevice(ctx->device);
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    (void)hipEventRecord(e0, ctx->stream);
    hipLaunchKernelGGL(kern, dim3(grid), dim3(1024), lds, ctx->stream, L, rays_per_lane, bounce, d_out);
    (void)hipEventRecord(e1, ctx->stream);
    (void)hipEventSynchronize(e1);
    (void)hipEventElapsedTime(ms, e0, e1);
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    return (int)hipGetLastError();
}
