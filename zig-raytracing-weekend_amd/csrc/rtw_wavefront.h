// rtw_wavefront.h -- HBM state of the wavefront kernels (rtw_wavefront.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "rtw_internal.h"

#define RTW_WF_MAX_ITERS 100
#define RTW_WF_STRIPES 256    // output queues (one atomic counter each)
#define RTW_WF_LEN_STRIDE 16  // counters 64 B apart

// One batch: n_pix logical pixels (8x8 tiles over the launch rows) x n_s samples.
// Path p = s_local * n_pix + q.  SoA, 16-B records, all sized n_paths (<= capacity).
//
// Work lists: iteration 0 deals the 64-path chunks round-robin over the waves
// of the grid (each chunk one 8x8 tile: coherent primary rays; every wave
// samples the whole image: balanced).  shade appends the survivors of wave w
// to stripe w % STRIPES of the other queue (one wave-aggregated atomic per 64
// paths, 256 counters: no hot spot); later iterations give stripe s to the
// waves w with w % STRIPES == s, which stride over its 64-entry chunks.  The
// grids are multiples of STRIPES waves.
struct rtw_wf {
    float4* ray_o;      // o.xyz, time
    float4* ray_d;      // d.xyz, bits(remaining depth); depth 0 = no path
    float4* thr;        // throughput.xyz
    float4* ls;         // radiance so far .xyz (final after the batch)
    uint64_t* rng;      // RNG state
    float2* hit;        // t, bits(hit leaf or -1)
    uint32_t* queue[2]; // ping-pong queues, stripe s at [s * stripe_cap, ...)
    uint32_t* len[2];   // stripe lengths, [s * RTW_WF_LEN_STRIDE]
    uint32_t n_pix, n_s, n_paths, n_tx;
    uint32_t stripe_cap;
    uint32_t iters;     // wavefront iterations before the tail kernel
};

// bytes of device state per path (queues extra)
#define RTW_WF_PATH_BYTES (4 * 16 + 8 + 8)

void rtw_wavefront_batch(const rtw_launch& L, const rtw_wf& W, void* stream, int n_cu, rtw_timer* T);
// waves of the largest wavefront grid (bounds the stripe capacity)
uint32_t rtw_wavefront_max_waves(int n_cu);
