// rtw_cpu.hip -- the host backend of the C ABI (rtw_scene_create(desc, RTW_DEVICE_CPU, ...)):
// Camera.render (src/camera.zig:93-116) on host threads, for machines without a GPU and for the
// reference's own CPU configuration (BASELINE config 1: 400x225, 10 spp, the 8-thread path of
// src/main.zig:314-326).
//
// Not a fallback: a context is a host context only when the caller asks for one, and a GPU
// context never runs here.  Each sample is sample_radiance() of rtw_device.h -- the very
// function the GPU's v0 kernel runs per lane, compiled for the host -- so a host render is
// bit-identical to the GPU's (same fp32 operations: correctly rounded division and sqrt, the
// restated pow / acos / atan2 / sin / log, the counter-based RNG; a host context walks the
// exact aabb.zig slab test and the IEEE sphere test, which the GPU's fast paths reproduce
// bit for bit).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <thread>
#include <vector>

#include "rtw_device.h"

int rtw_cpu_render(const rtw_launch& L, uint32_t begin, uint32_t end, float* out, uint32_t threads,
                   const rtw_render_opts* stop) {
    const uint32_t n = end - begin;
    if (threads == 0) threads = std::max(1u, std::thread::hardware_concurrency());
    threads = std::min<uint32_t>(threads, std::max(1u, n));
    std::atomic<bool> stopped{false};
    // contiguous chunks, as startRender's Tasks (main.zig:318-324); samples in order per pixel
    auto work = [&](uint32_t t) {
        const uint32_t a = begin + (uint32_t)((uint64_t)n * t / threads);
        const uint32_t b = begin + (uint32_t)((uint64_t)n * (t + 1) / threads);
        Counters cnt;
        for (uint32_t i = a; i < b; i++) {
            if (rtw_stop_requested(stop)) {  // polled per pixel, as Camera.render polls `running` (camera.zig:107)
                stopped = true;
                return;
            }
            const uint32_t x = i % L.W;
            uint32_t y = i / L.W;
            if (L.n_shards && !map_row(L, y, y)) continue;  // a shard's logical row -> image row (rows past H: none)
            if (y >= L.H) continue;
            const uint32_t pixel = y * L.W + x;
            float* px = out + 4 * (size_t)i;
            float r = px[0], g = px[1], bl = px[2];
            for (uint32_t s = L.s0; s < L.s1; s++) {
                const f3 c = sample_radiance<RTW_F_ALL>(L.nodes, L, pixel, x + L.pixel_offset, y + L.pixel_offset, s,
                                                        cnt);
                r += c.x;
                g += c.y;
                bl += c.z;
            }
            px[0] = r;
            px[1] = g;
            px[2] = bl;
            px[3] = (float)L.s1;  // writeColor: number_of_samples (camera.zig:56)
        }
    };
    std::vector<std::thread> pool;
    pool.reserve(threads);
    for (uint32_t t = 1; t < threads; t++) pool.emplace_back(work, t);
    work(0);
    for (std::thread& th : pool) th.join();
    return stopped ? RTW_E_CANCELLED : RTW_OK;
}

// ABI 6 test hook (include/rtw_gpu.h): the walk's sphere fast-reject against Sphere.hit's exact accept, on
// the host -- sphere_may_hit is the device's code (rtw_device.h), the same fp32 operations
extern "C" int rtw_debug_sphere_filter(uint32_t n, const float* a, const float* half_b, const float* c, const float* closest,
                            uint8_t* may_hit, uint8_t* accept) {
    if (n && (!a || !half_b || !c || !closest || !may_hit || !accept)) return RTW_E_INVALID;
    for (uint32_t i = 0; i < n; i++) {
        // the ray constants as ray_trav derives them from a (fast_reject on)
        const float aa = a[i], hb = half_b[i];
        const bool in_range = aa >= 0x1p-40f && aa <= 0x1p40f;
        const float tk = aa * 0.001f, ktk = tk * 9.5367432e-07f, gk = in_range ? 0.99999905f : 0.0f;
        const float disc = hb * hb - aa * c[i];
        may_hit[i] = sphere_may_hit(hb, disc, aa, closest[i], tk, ktk, gk) ? 1 : 0;
        // Sphere.hit (objects.zig:127-136): nearest root in the open interval (0.001, closest)
        bool ok = false;
        if (disc >= 0) {
            const float sq = std::sqrt(disc);
            float root = (-hb - sq) / aa;
            ok = 0.001f < root && root < closest[i];
            if (!ok) {
                root = (-hb + sq) / aa;
                ok = 0.001f < root && root < closest[i];
            }
        }
        accept[i] = ok ? 1 : 0;
    }
    return RTW_OK;
}
