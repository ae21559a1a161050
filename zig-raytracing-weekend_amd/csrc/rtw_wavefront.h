// rtw_wavefront.h -- HBM state of the wavefront kernels (rtw_wavefront.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "rtw_internal.h"

#define RTW_WF_MAX_ITERS 100
#define RTW_WF_STRIPES 256    // output queues (one atomic counter each)
#define RTW_WF_LEN_STRIDE 16  // counters 64 B apart
// coherent queues (wf_push_bucketed): a wave keeps one open 64-slot block per direction bucket
#define RTW_WF_BUCKET_BITS 4
#define RTW_WF_BUCKETS (1u << RTW_WF_BUCKET_BITS)
#define RTW_TL_MAX 128         // camera-ray candidate list capacity per 8x8 tile (rtw_tuning.tile_lists caps it)
#define RTW_TL_WALK 0xFFFFFFFFu
#define RTW_TL_BYTES (RTW_TL_MAX * 32 + 4)  // per tile
#define RTW_WF_CLDS2_MAX (80u * 1024u)  // their stage (+ materials) per block: half the CU's LDS
#define RTW_W2_STACK_MAX 32   // deepest per-lane LDS stack of the two-wide walk (256 threads x 32 x 4 B = 32 KiB)

// One batch: n_pix logical pixels (8x8 tiles over the launch rows) x n_s samples.
// Path p = ((q / 64) * n_s + s_local) * 64 + q % 64 (tile-major, wf_path).
//
// Path state lives in *slot space* and moves with the compaction: iteration it
// reads set[it & 1] and shade writes each surviving path's state to its new slot
// in set[(it + 1) & 1], so every state access of trace / shade is a coalesced
// 16-B-per-lane stream (a path-indexed layout made later iterations gather
// scattered 16-B pieces of 64-B lines).  Only the final radiance is stored by
// path id (ls[p], once per path).
//
// Slots: iteration 0 deals the 64-path chunks in runs of 16 samples of one tile
// round-robin over the waves of the grid (slot = p; each chunk one 8x8 tile:
// coherent primary rays; every wave samples the whole image: balanced).  shade
// appends the survivors of wave w to stripe w % STRIPES of the other set (one
// wave-aggregated atomic per push, 256 counters: no hot spot), in the first
// sort_iters iterations into 64-slot blocks per direction bucket; later
// iterations give stripe s to the waves w with w % STRIPES == s, which stride
// over its 64-slot chunks.  The grids are multiples of STRIPES waves.
struct rtw_wf_set {
    float4* ray_o;      // o.xyz, time
    float4* ray_d;      // d.xyz, bits(remaining depth); depth 0 = no path
    float4* thr;        // throughput.xyz, bits(path id) (implicit 1 and slot on the first bounce; packed state:
                        // thr.z, path id, RNG state -- rtw_wavefront.hip wf_packed)
    float4* acc;        // radiance so far (scenes with emitters only)
    uint64_t* rng;      // RNG state
};

// a finished sample's radiance (12 B: the reduce reads 5.8 GB instead of 7.7 GB for C2's 480 M samples)
struct rtw_rgb {
    float x, y, z;
};

struct rtw_wf {
    rtw_wf_set set[2];
    float2* hit;        // t, bits(hit leaf or -1), by slot of the iteration's input set
    rtw_rgb* ls;        // final radiance by path id
    uint32_t* len[3];   // stripe lengths of iteration it's input: len[it % 3][s * RTW_WF_LEN_STRIDE]
                        // (three sets: a fused step kernel zeroes the counters of
                        // iteration it+2 while it appends to those of it+1)
    uint4* tl;          // camera-ray candidate lists: tile t's entry k at tl[2 * (t * RTW_TL_MAX + k)] (2 x 16 B)
    uint32_t* tl_count; // candidates of tile t, or RTW_TL_WALK (too many: walk the tree); null = off
    uint32_t n_pix, n_s, n_paths, n_tx;
    uint32_t stripe_cap;
    uint32_t iters;     // wavefront iterations before the tail kernel
    uint32_t sort_iters;  // iterations it < sort_iters push their survivors into direction-bucketed blocks
    uint32_t sort_iters_split;  // the same for the split trace / shade kernels (wf_run copies it to sort_iters)
    uint32_t sort_mask;   // the bucket key bits they use ((1 << rtw_tuning.sort_bits) - 1)
    uint32_t run_log2;    // iteration 0's tile runs: 2^run_log2 samples of one tile per run (wf_coherence)
    uint32_t packed;      // this render's queues hold the packed path state (wf_packed; set by wf_run*)
    uint32_t* deal;       // dynamic dealing (rtw_tuning.deal): this launch's counters (zeroed per batch), or null
    uint32_t deal_mode;   // rtw_tuning.deal bits (RTW_DEAL_*): 1 iteration 0, 2 the tail, 8 dynamic even on small
                          // batches, 16 iterations >= 1 (per stripe group), 32 long singles, 128 bucketing on small
                          // batches
    uint32_t* deal_it;    // this launch's per-stripe counters for iteration it >= 1 (deal bit 16), or null
};
#define RTW_WF_DEAL_LAUNCH (2 * RTW_WF_STRIPES)  // counters of one launch dealing iteration 0 (runs, singles per group)
#define RTW_WF_DEAL_COUNTERS0 (2 * RTW_WF_DEAL_LAUNCH + RTW_WF_STRIPES)  // split trace's, shade's, the tail's
// per batch: those, then RTW_WF_STRIPES per iteration it >= 1 (deal bit 16): the fused step's or the split trace's at
// RTW_WF_DEAL_COUNTERS0 + it * 256, the split shade's at RTW_WF_DEAL_SHADE + it * 256
#define RTW_WF_DEAL_SHADE (RTW_WF_DEAL_COUNTERS0 + (RTW_WF_MAX_ITERS + 1) * RTW_WF_STRIPES)
#define RTW_WF_DEAL_COUNTERS (RTW_WF_DEAL_SHADE + (RTW_WF_MAX_ITERS + 1) * RTW_WF_STRIPES)

// bytes of device state per path (two slot sets + hit + ls; the batch's counters aside)
#define RTW_WF_PATH_BYTES (2 * (4 * 16 + 8) + 8 + 12)

void rtw_wavefront_batch(const rtw_launch& L, const rtw_wf& W, void* stream, int n_cu, rtw_timer* T);
// waves of the largest wavefront grid (bounds the stripe capacity)
uint32_t rtw_wavefront_max_waves(int n_cu);
