// DIAGNOSTIC ONLY (not the product): traversal-only microbenchmark.
// Compiles the product kernel TU and adds a kernel that walks primary rays
// (pixel centres, no jitter/RNG/shading) with the same trav_step, so the cost
// of a node step can be measured without the megakernel around it.
#include "../zig-raytracing-weekend_amd/csrc/rtw_kernels.hip"

namespace {
template <int MODE>
__global__ __launch_bounds__(256) void trav_only(rtw_launch L, uint32_t rays_per_lane, uint32_t coherent, uint32_t secondary, unsigned long long* out) {
    extern __shared__ float4 lds_nodes[];
    const uint32_t n4 = 2 * L.n_nodes;
    for (uint32_t k = threadIdx.x; k < n4; k += blockDim.x) lds_nodes[k] = L.nodes[k];
    __syncthreads();
    const float4* nodes = MODE == 1 ? L.nodes : lds_nodes;
    Counters cnt;
    const uint32_t gid = blockIdx.x * blockDim.x + threadIdx.x;
    float acc = 0;
    for (uint32_t k = 0; k < rays_per_lane; k++) {
        const uint32_t pix = coherent ? (gid + k * gridDim.x * blockDim.x) % (L.W * L.H)
                                       : (gid * 7919u + k * 104729u) % (L.W * L.H);
        const uint32_t x = pix % L.W, y = pix / L.W;
        Ray r;
        const f3 du = ld3(L.du), dv = ld3(L.dv);
        const f3 pc = (ld3(L.pixel00) + du * splat((float)x)) + dv * splat((float)y);
        r.o = ld3(L.center);
        r.d = pc - r.o;
        r.time = 0;
        float t;
        int h = traverse<0u>(nodes, L, r, t, cnt);
        acc += h >= 0 ? t : 0.0f;
        if (secondary && h >= 0) {
            // a diffuse bounce: n + (hash-based unit-ish vector), origin on the sphere
            const float4 A = nodes[2 * h], B = nodes[2 * h + 1];
            const f3 p = r.o + splat(t) * r.d;
            const f3 n = divs(p - mk(A.x, A.y, A.z), B.x);
            uint64_t hs = rtw_mix64(((uint64_t)gid << 32) | k);
            const float ux = (float)(hs & 0xFFFFF) * (2.0f / 1048576.0f) - 1.0f;
            const float uy = (float)((hs >> 20) & 0xFFFFF) * (2.0f / 1048576.0f) - 1.0f;
            const float uz = (float)((hs >> 40) & 0xFFFFF) * (2.0f / 1048576.0f) - 1.0f;
            const f3 u = mk(ux, uy, uz);
            Ray r2;
            r2.o = p;
            r2.d = n + divs(u, __builtin_sqrtf(length_squared(u)) + 1e-6f);
            r2.time = 0;
            h = traverse<0u>(nodes, L, r2, t, cnt);
            acc += h >= 0 ? t : 0.0f;
        }
    }
    if (acc == 12345.0f) out[7] = 1;  // keep live
    atomicAdd(&out[0], (unsigned long long)cnt.nodes);
    atomicAdd(&out[1], (unsigned long long)cnt.leaves);
}
}  // namespace

extern "C" int rtw_diag_trav(rtw_ctx* ctx, const rtw_camera* cam, int mode, uint32_t blocks, uint32_t rays_per_lane,
                             unsigned long long* d_out, float* ms) {
    rtw_launch L = ctx->base;
    for (int k = 0; k < 3; k++) {
        L.center[k] = cam->center[k]; L.pixel00[k] = cam->pixel00_loc[k];
        L.du[k] = cam->pixel_delta_u[k]; L.dv[k] = cam->pixel_delta_v[k];
    }
    L.W = cam->image_width; L.H = cam->image_height;
    hipEvent_t a, b;
    (void)hipEventCreate(&a); (void)hipEventCreate(&b);
    (void)hipEventRecord(a, ctx->stream);
    const size_t lds = (size_t)L.n_nodes * 32;
    const uint32_t coh = (mode >> 1) & 1, sec = (mode >> 2) & 1;
    if (mode & 1) hipLaunchKernelGGL(trav_only<1>, dim3(blocks), dim3(256), lds, ctx->stream, L, rays_per_lane, coh, sec, d_out);
    else hipLaunchKernelGGL(trav_only<0>, dim3(blocks), dim3(256), lds, ctx->stream, L, rays_per_lane, coh, sec, d_out);
    (void)hipEventRecord(b, ctx->stream);
    (void)hipEventSynchronize(b);
    (void)hipEventElapsedTime(ms, a, b);
    return (int)hipGetLastError();
}
