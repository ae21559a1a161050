// rtw_wavefront.h -- HBM state of the wavefront kernels (rtw_wavefront.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "rtw_internal.h"

#define RTW_WF_MAX_ITERS 100
#define RTW_WF_SEGS 32768  // queue segments (wave-sized work lists, walked round-robin by the resident waves)

// One batch: n_pix logical pixels (8x8 tiles over the launch rows) x n_s samples.
// Path p = s_local * n_pix + q.  SoA, 16-B records, all sized n_paths (<= capacity).
//
// Work lists without atomics: the paths are dealt to RTW_WF_SEGS segments in
// 64-path chunks, chunk c -> segment c % RTW_WF_SEGS (so every segment samples
// the whole image: balanced), each chunk one 8x8 tile (coherent primary rays).
// Iteration 0 walks that deal implicitly; shade compacts a segment's survivors
// into the same segment of the other queue (ballot prefix, no atomics) and
// stores its length in seg_len[it+1 & 1][segment].
struct rtw_wf {
    float4* ray_o;      // o.xyz, time
    float4* ray_d;      // d.xyz, bits(remaining depth)
    float4* thr;        // throughput.xyz
    float4* ls;         // radiance so far .xyz (final after the batch)
    uint64_t* rng;      // RNG state
    float2* hit;        // t, bits(hit leaf or -1)
    uint32_t* queue[2]; // ping-pong path queues, segment g at [g * seg_cap, ...)
    uint32_t* seg_len[2];
    uint32_t n_pix, n_s, n_paths, n_tx;
    uint32_t seg_cap;   // entries per segment = ceil(chunks / RTW_WF_SEGS) * 64
    uint32_t iters;     // wavefront iterations before the tail kernel
};

// bytes of device state per path (+ queues: 2 x 4 B per segment entry)
#define RTW_WF_PATH_BYTES (4 * 16 + 8 + 8)

void rtw_wavefront_batch(const rtw_launch& L, const rtw_wf& W, void* stream, int n_cu);
