// rtw_wavefront.hip -- v2: wavefront path tracing (the default kernel path).
//
// The megakernels (v0/v1, rtw_kernels.hip) keep a whole path in registers, so
// the BVH walk -- 60 % of their time -- runs at the occupancy the shading code
// allows (~100 VGPRs, 4 waves/SIMD).  Measured on MI355X (diag/trav_bench.hip)
// the same walk in a ~40-VGPR kernel runs 4-6x more node steps per second.
// v2 therefore splits a batch of paths into kernels over HBM-resident SoA state:
//
//   camera (pixel, sample) -> camera ray           Camera.getRay  camera.zig:169-180
//          (in registers, by iteration 0's kernels: wf_camera)
//   trace  ray -> closest hit (t, leaf)            BVHNode.hit    bvh.zig:122-136
//   shade  hit -> emission/background, scatter     rayColor       camera.zig:182-208
//          (survivors appended to the next queue)
//   tail   the few paths still alive after RTW_WF_ITERS bounces, to completion
//   reduce per pixel: accum += sample radiances in sample order (camera.zig:55-56)
//
// A batch holds n_pix logical pixels x n_s samples, q in 8x8 pixel tiles so a wave's
// primary rays are one tile; path ids are tile-major (wf_path).  Every path runs
// the same operations in the same order as in v0/v1 (same RNG stream, same
// iterative radiance), and the reduce adds the samples of a pixel in sample
// order onto the accumulator, so v2 is bit-identical to v0/v1.
#include "rtw_device.h"
#include "rtw_wavefront.h"

#include <algorithm>
#include <cstdlib>
#include <map>
#include <mutex>

// Waves-per-SIMD targets of the 256-thread kernels (1 = no target: the registers the code needs;
// MI355X_MICROARCH.md: <= 96 VGPRs -> 5 waves, <= 80 -> 6, <= 72 -> 7), same-box A/Bs of round 6
// (profiles/r6_waves/).  Once round 6 had cut the live state (profiles/r6_late_rest/), more waves paid despite
// a few spills: the split trace (C4: 83 VGPRs, 5 waves) at 6 waves -8.5 % trace time, at 7 a further -3.5 %; the
// split shade at 6 (C4 +3.5 % with the trace at 6; 5 alone: +-0); the two-wide tail (93 VGPRs) at 6: -3.4 % tail
// time; the LDS tail of the object scenes (Cornell: 113 VGPRs, 4 waves) at 5: +7 %, at 6 a further +2 % on
// Cornell but -8 % on Cornell smoke (media: 126 VGPRs), which keeps 5; the fused wf_step at 5 instead of 4:
// Cornell -3 %, smoke -8 %, C5 -9 % (its spills grow)
#ifndef RTW_WPE_TRACE
#define RTW_WPE_TRACE 7
#endif
#ifndef RTW_WPE_SHADE
#define RTW_WPE_SHADE 6
#endif
#ifndef RTW_WPE_TAIL_W5
#define RTW_WPE_TAIL_W5 6
#endif
// The media scenes' LDS tail parks the path state it does not need during the walk in LDS (wf_tail_body PARK):
// Cornell smoke's tail 112 -> 80 B of scratch, -6.5 % tail time (+3 %); Cornell's (no media) loses 0.7 % with it
// (same box, profiles/r6_waves/j/)
#ifndef RTW_TAIL_PARK
#define RTW_TAIL_PARK 1
#endif
// the cooperative rejection loop in the textured fused step too: once round 6 freed its registers (the IT0
// split, the hit record after the loop) C5 +0.6 % (two rounds, profiles/r6_waves/l/; round 4: -2.3 % at the cap)
#ifndef RTW_COOP_TEXTURED
#define RTW_COOP_TEXTURED 1
#endif

#ifndef RTW_WPE_TAIL_LDS  // object classes with media / textures / motion; the plain one RTW_WPE_TAIL_LDS_OBJ
#define RTW_WPE_TAIL_LDS 5
#endif
#ifndef RTW_WPE_TAIL_LDS_OBJ
#define RTW_WPE_TAIL_LDS_OBJ 6
#endif
// the split trace / shade targets apply to the untextured static sphere classes they were measured on (C4);
// the other classes' split kernels (large object or textured trees: 100-200 VGPRs) keep no target
template <uint32_t FEAT>
constexpr int wf_split_wpe(int w) { return (FEAT & ~RTW_F_CHECKER) == 0 ? w : 1; }
template <uint32_t FEAT>
constexpr int wf_tail_lds_wpe() {
    // the object class without media, textures or motion (Cornell) at 6; the media class (Cornell smoke, 126 VGPRs)
    // at 5; every other class keeps no target -- simple_light's all-features tail at 5 or 6 waves spilled 184 B and
    // lost 27 % of its tail time (profiles/r6_waves/o/, q/)
    constexpr uint32_t tex = RTW_F_IMAGE | RTW_F_NOISE | RTW_F_MOVING;
    if constexpr (!(FEAT & RTW_F_GEOM) || (FEAT & tex)) return 1;
    return (FEAT & RTW_F_MEDIUM) ? RTW_WPE_TAIL_LDS : RTW_WPE_TAIL_LDS_OBJ;
}
#ifndef RTW_WPE_STEP
#define RTW_WPE_STEP 4
#endif

namespace {

#if defined(RTW_DIAG_WALK)
// diagnostic build: per-slot record of the compact walks of one wavefront iteration (tools/diag_sort.py):
// rec[2 slot] = (steps | sphere tests << 16, bits(d.xyz)), rec[2 slot + 1] = (bits(o.xyz), path id + 1)
__device__ uint4* rtw_diag_rec;
__device__ uint32_t rtw_diag_rec_cap;
__device__ uint32_t rtw_diag_rec_it;
#endif

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

__device__ __forceinline__ uint32_t wf_wave() { return blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); }
__device__ __forceinline__ uint32_t wf_nwaves() { return gridDim.x * (blockDim.x >> 6); }

// Iteration 0 deals its chunks (64 paths = one 8x8 tile of one sample) in runs of RUN = 2^W.run_log2 (<= 16,
// wf_coherence) consecutive samples of one tile: in tile-major order c = tile * n_s + s_local, run R = c / RUN goes to
// wave R % nw, so a wave takes RUN chunks of the same tile in a row (the blocks its survivors fill,
// wf_push_bucketed, then hold rays that left one tile) while the runs, dealt round-robin, keep the waves'
// shares of sky and ground even.  A wave's k-th chunk: c = ((k / RUN) * nw + w) * RUN + k % RUN, which grows
// with k (false: past the last chunk).  slot0: the chunk's first path id.
__device__ __forceinline__ bool wf_chunk0(const rtw_wf& W, uint32_t w, uint32_t nw, uint32_t k, uint32_t& slot0) {
    const uint32_t lg = W.run_log2;
    const uint32_t c = ((((k >> lg) * nw + w)) << lg) + (k & ((1u << lg) - 1u));
    if (c >= (W.n_paths >> 6)) return false;
    slot0 = c << 6;
    return true;
}

// Path ids are tile-major: path p is sample s_local of pixel q (in tile order) with
// p = ((q / 64) * n_s + s_local) * 64 + q % 64, so chunk c = p / 64 is sample c % n_s of tile c / n_s and
// the paths of one tile-run (wf_chunk0) are RUN consecutive chunks: the radiance stores of a block's rays
// (W.ls[pid], pids of one run) stay within 12 KB, and the reduce reads 64 consecutive pixels per sample.
__device__ __forceinline__ void wf_path(const rtw_wf& W, uint32_t p, uint32_t& s_local, uint32_t& q) {
    const uint32_t c = p >> 6, t = c / W.n_s;
    s_local = c - t * W.n_s;
    q = (t << 6) | (p & 63u);
}

// Dynamic dealing of iteration 0 (W.deal, rtw_tuning.deal).  The waves of stripe group g (the waves w with
// w % RTW_WF_STRIPES == g, whose survivors all go to stripe g) share the runs r = g + 256 k (RUN chunks of one
// tile, tile-major): a wave claims the group's next k from W.deal[g] -- one atomic per run, issued a run ahead
// so its latency is hidden -- until the group's runs run out.  Within the group the waves that draw cheap tiles
// (sky) take more runs, so its 16-odd waves drain together however few runs each gets, and the runs keep their
// full 16 samples on small batches (a shard of a multi-GPU render), where the static deal must shorten them to
// keep every wave's share even.  Each group still takes exactly every 256th run, so a stripe receives the
// survivors of the same share of the batch as under the static deal and its capacity holds (rtw_host.hip
// stripe_cap; a global deal let one stripe's waves take more than their share and overflow it).  The last
// 4 x (waves) chunks -- 16 x with deal bit 32, as long as a run, so that a wave that took the last run does not
// leave the others idle -- go one at a time, the group's every 256th (W.deal[256 + g]).  Deal bit 16: iteration
// it >= 1's waves of group g claim the chunks of stripe g from one counter (W.deal_it[g]) instead of a fixed
// stride; their survivors still go to stripe g, so the capacities hold as before.
__device__ __forceinline__ uint32_t wf_claim(uint32_t* c) {  // lane 0 holds the claimed run
    uint32_t v = 0;
    if (__lane_id() == 0) v = atomicAdd(c, 1u);
    return v;
}

// The slots of iteration `it` handed to this wave, 64 at a time:
//   for (WfIter e(W, it); e.more(); e.next()) { uint32_t slot; if (e.get(W, slot)) ... }
// (wave-uniform loop; get() is per lane)
struct WfIter {
    uint32_t it, j, step, n, base, off, w, nw, slot0;
    uint32_t run, kk, next_run;  // dynamic iteration 0: the run (or single chunk), the chunk in it, the next claim
    uint32_t runs;               //   (lane 0); runs dealt whole, then single chunks
    bool single;
    bool live0;  // iteration 0: chunk j exists
    __device__ WfIter(const rtw_wf& W, uint32_t it_) : it(it_) {
        w = wf_wave();
        nw = wf_nwaves();
        if (it == 0) {
            j = 0;
            step = 1;
            if (W.deal && (W.deal_mode & 1u)) {
                const uint32_t nc = W.n_paths >> 6, tail = (W.deal_mode & 32u) ? nw << W.run_log2 : 4u * nw;
                runs = nc > tail ? (nc - tail) >> W.run_log2 : 0u;
                single = false;
                run = __builtin_amdgcn_readfirstlane(wf_claim(W.deal + w % RTW_WF_STRIPES));
                next_run = wf_claim(W.deal + w % RTW_WF_STRIPES);
                kk = 0;
                if (grp(run) >= runs) to_single(W);
                live0 = dyn_chunk(W);
            } else {
                live0 = wf_chunk0(W, w, nw, 0, slot0);
            }
        } else {
            const uint32_t s = w % RTW_WF_STRIPES;
            j = w / RTW_WF_STRIPES;
            step = nw / RTW_WF_STRIPES;
            base = W.len[it % 3u][s * RTW_WF_LEN_STRIDE];  // slots used in the stripe
            n = (base + 63u) >> 6;
            off = s * W.stripe_cap;
            if (W.deal_it) {  // deal bit 16: the group's waves claim stripe s's chunks, one claim issued ahead
                j = __builtin_amdgcn_readfirstlane(wf_claim(W.deal_it + s));
                next_run = wf_claim(W.deal_it + s);
            }
        }
        W_ = &W;
    }
    const rtw_wf* W_;
    // the group's k-th run / single chunk (k claimed from the group's counter)
    __device__ uint32_t grp(uint32_t k) const { return k * RTW_WF_STRIPES + w % RTW_WF_STRIPES; }
    __device__ void to_single(const rtw_wf& W) {
        single = true;
        run = __builtin_amdgcn_readfirstlane(wf_claim(W.deal + RTW_WF_STRIPES + w % RTW_WF_STRIPES));
        next_run = wf_claim(W.deal + RTW_WF_STRIPES + w % RTW_WF_STRIPES);
    }
    __device__ bool dyn_chunk(const rtw_wf& W) {
        const uint32_t c = single ? (runs << W.run_log2) + grp(run) : (grp(run) << W.run_log2) + kk;
        slot0 = c << 6;
        return c < (W.n_paths >> 6);
    }
    __device__ bool more() const { return it == 0 ? live0 : j < n; }
    __device__ void next() {
        if (it != 0 && W_->deal_it) {
            j = __builtin_amdgcn_readfirstlane(next_run);
            next_run = wf_claim(W_->deal_it + w % RTW_WF_STRIPES);
            return;
        }
        j += step;
        if (it == 0) {
            if (W_->deal && (W_->deal_mode & 1u)) {
                if (single) {
                    run = __builtin_amdgcn_readfirstlane(next_run);
                    next_run = wf_claim(W_->deal + RTW_WF_STRIPES + w % RTW_WF_STRIPES);
                } else if (++kk == (1u << W_->run_log2)) {
                    run = __builtin_amdgcn_readfirstlane(next_run);
                    next_run = wf_claim(W_->deal + w % RTW_WF_STRIPES);
                    kk = 0;
                    if (grp(run) >= runs) to_single(*W_);
                }
                live0 = dyn_chunk(*W_);
            } else {
                live0 = wf_chunk0(*W_, w, nw, j, slot0);
            }
        }
    }
    __device__ bool get(const rtw_wf& W, uint32_t& slot) const {
        if (it == 0) {
            slot = slot0 | __lane_id();
            return true;
        }
        const uint32_t k = (j << 6) | __lane_id();
        slot = off + k;
        return k < base;
    }
};

// m-th slot of this wave's list at iteration it (the WfIter order); false past the
// end or for padding.  `end` is set when m is past the list.
__device__ __forceinline__ bool wf_nth(const rtw_wf& W, uint32_t it, uint32_t m, uint32_t& slot, bool& end) {
    const uint32_t w = wf_wave(), nw = wf_nwaves();
    if (it == 0) {
        uint32_t slot0 = 0;
        end = !wf_chunk0(W, w, nw, m >> 6, slot0);
        slot = slot0 | (m & 63u);
        return !end;
    }
    const uint32_t s = w % RTW_WF_STRIPES, R = nw / RTW_WF_STRIPES;
    const uint32_t k = ((((m >> 6) * R) + w / RTW_WF_STRIPES) << 6) | (m & 63u);
    const uint32_t n = W.len[it % 3u][s * RTW_WF_LEN_STRIDE];
    end = (k & ~63u) >= n;
    slot = s * W.stripe_cap + k;
    return k < n;
}

// wave-aggregated slot allocation in this wave's output stripe of set[(it+1)&1]
// (its counter: len[(it+1) % 3])
__device__ __forceinline__ uint32_t wf_push(const rtw_wf& W, uint32_t it, bool push) {
    const uint64_t m = __ballot(push);
    if (!m) return 0;
    const uint32_t s = wf_wave() % RTW_WF_STRIPES, lane = __lane_id();
    uint32_t* len = &W.len[(it + 1u) % 3u][s * RTW_WF_LEN_STRIDE];
    uint32_t base = 0;
    if (lane == 0) base = atomicAdd(len, (uint32_t)__popcll(m));
    base = __shfl(base, 0);
    const uint64_t lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
    return s * W.stripe_cap + base + (uint32_t)__popcll(m & lt);
}

// Coherent queues (iterations it < W.sort_iters).  A wave files its survivors into 64-slot blocks of its
// output stripe, one open block per direction bucket (RTW_WF_BUCKETS: the signs of the scattered
// direction's x and z and four levels of its elevation), so a block -- one chunk of the next iteration --
// holds rays of similar direction that left the few tiles the wave worked on: the walks of a wave then
// take similar paths through the tree (tools/diag_sort.py: C2 iteration 1 walk lane utilisation 0.60 as
// appended, 0.78 tile + direction).  The open blocks live in the lanes: lane b holds
// bucket b's block (first slot `bb`, slots used `bf`; 64 = none).  Per push: lanes with equal keys by
// one ballot per key bit; each bucket's lanes take consecutive slots of its block, and buckets whose
// block overflows take fresh blocks, all of them with one atomic on the stripe counter.  A partly filled
// block's unused slots are marked dead (depth 0) when the wave's iteration ends (wf_close_blocks).
// vec3.randomInUnitSphere (vec3.zig:40-45) for every lane of the wave with `need`, cooperatively: the
// same accepted candidate and the same final RNG state as seq_reject<3> per lane.  The draws are
// counter-based (rtw_path_float: the k-th draw after state s hashes s + k*G), so candidate c of a lane
// -- draws 3c+1 .. 3c+3 -- can be evaluated on any lane from the owner's state.  Trip 0: every lane
// evaluates its own candidate 0 (~52 % accept).  Then, while lanes are pending, each of the R pending
// lanes gets a group of g = 64 / R (a power of two) lanes that evaluate its next g candidates at once
// and it takes the first accepted one: ~3 trips for the wave instead of the ~7 the slowest of 64
// independent loops takes, and the idle lanes do the work.  Called by the whole wave (converged).
__device__ __forceinline__ void wf_cand3(uint64_t s, float& x, float& y, float& z) {
    rtw_rng r;
    r.s = s;
    x = rtw_path_range(r, -1, 1);
    y = rtw_path_range(r, -1, 1);
    z = rtw_path_range(r, -1, 1);
}
__device__ __forceinline__ void wf_reject3(bool need, rtw_rng& rng, float (&out)[3]) {
    const uint32_t lane = __lane_id();
    const uint64_t s0 = rng.s;
    float x = 0.0f, y = 0.0f, z = 0.0f;
    bool ok = false;
    if (need) {
        wf_cand3(s0, x, y, z);
        ok = x * x + y * y + z * z < 1;  // lengthSquared < 1 (vec3.zig:43)
    }
    if (ok) {
        out[0] = x;
        out[1] = y;
        out[2] = z;
        rng.s = s0 + 3ull * RTW_GOLDEN;
    }
    uint64_t pend = __ballot(need && !ok);
    uint32_t kb = 1;  // candidates every pending lane has rejected so far
    const uint64_t lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
    while (pend) {
        const uint32_t R = (uint32_t)__popcll(pend);
        const uint32_t lg = R > 32 ? 0u : R > 16 ? 1u : R > 8 ? 2u : R > 4 ? 3u : R > 2 ? 4u : R > 1 ? 5u : 6u;
        const bool mine = (pend >> lane) & 1ull;
        const uint32_t rank = (uint32_t)__popcll(pend & lt);
        // the owner's state to the first lane of its group (forward permute), then to the whole group
        const int dst = (int)((mine ? (rank << lg) : 63u) * 4u);
        int lo = __builtin_amdgcn_ds_permute(dst, (int)(uint32_t)s0);
        int hi = __builtin_amdgcn_ds_permute(dst, (int)(uint32_t)(s0 >> 32));
        const int lead = (int)((lane & ~((1u << lg) - 1u)) * 4u);
        lo = __builtin_amdgcn_ds_bpermute(lead, lo);
        hi = __builtin_amdgcn_ds_bpermute(lead, hi);
        const bool act = (lane >> lg) < R;
        const uint32_t c = kb + (lane & ((1u << lg) - 1u));
        float cx = 0.0f, cy = 0.0f, cz = 0.0f;
        bool acc = false;
        if (act) {
            const uint64_t so = ((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo;
            wf_cand3(so + (uint64_t)(3u * c) * RTW_GOLDEN, cx, cy, cz);
            acc = cx * cx + cy * cy + cz * cz < 1;
        }
        const uint64_t A = __ballot(act && acc);
        int src = (int)(lane * 4u);
        uint32_t idx = 0;
        bool got = false;
        if (mine) {
            const uint64_t gm = lg == 6u ? ~0ull : ((1ull << (1u << lg)) - 1ull);
            const uint64_t grp = (A >> (rank << lg)) & gm;
            if (grp) {
                const uint32_t o = (uint32_t)__builtin_ctzll(grp);
                src = (int)(((rank << lg) + o) * 4u);
                idx = kb + o;
                got = true;
            }
        }
        const float gx = __int_as_float(__builtin_amdgcn_ds_bpermute(src, __float_as_int(cx)));
        const float gy = __int_as_float(__builtin_amdgcn_ds_bpermute(src, __float_as_int(cy)));
        const float gz = __int_as_float(__builtin_amdgcn_ds_bpermute(src, __float_as_int(cz)));
        if (got) {
            out[0] = gx;
            out[1] = gy;
            out[2] = gz;
            rng.s = s0 + (uint64_t)(3u * (idx + 1u)) * RTW_GOLDEN;
        }
        pend = __ballot(mine && !got);
        kb += 1u << lg;
    }
}

__device__ __forceinline__ uint32_t wf_bucket(f3 d) {
    const float ilen = __builtin_amdgcn_rsqf(d.x * d.x + d.y * d.y + d.z * d.z);  // approximate: a sort key only
    const float uy = d.y * ilen;
    const uint32_t qy = (uy > -0.5f ? 1u : 0u) + (uy > 0.0f ? 1u : 0u) + (uy > 0.5f ? 1u : 0u);
    return (d.x < 0.0f ? 1u : 0u) | (d.z < 0.0f ? 2u : 0u) | (qy << 2);
}

__device__ __forceinline__ uint32_t wf_push_bucketed(const rtw_wf& W, uint32_t it, bool push, uint32_t key,
                                                     uint32_t& bb, uint32_t& bf) {
    const uint64_t act = __ballot(push);
    if (!act) return 0;
    const uint32_t lane = __lane_id();
    key = push ? key : 0u;
    uint64_t eq = act, eqh = act;  // eq: lanes with my key; eqh: lanes whose key is my lane (holder view)
#pragma unroll
    for (uint32_t k = 0; k < RTW_WF_BUCKET_BITS; k++) {
        const uint64_t m = __ballot(push && ((key >> k) & 1u));
        eq &= ((key >> k) & 1u) ? m : ~m;
        eqh &= ((lane >> k) & 1u) ? m : ~m;
    }
    if (lane >= RTW_WF_BUCKETS) eqh = 0;
    const uint64_t lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
    const uint32_t rank = (uint32_t)__popcll(eq & lt), cnt = (uint32_t)__popcll(eq);
    const uint32_t leader = (uint32_t)__builtin_ctzll(eq | (1ull << 63));  // push lanes: eq != 0
    const uint32_t base = __shfl(bb, (int)key), fill = __shfl(bf, (int)key);  // my bucket's open block
    const uint32_t room = 64u - fill;
    // buckets whose block cannot take all their lanes get a fresh block (one atomic for the wave)
    const uint64_t need = __ballot(push && rank == 0 && cnt > room);
    uint32_t b0 = 0;
    if (need) {
        const uint32_t s = wf_wave() % RTW_WF_STRIPES;
        uint32_t* len = &W.len[(it + 1u) % 3u][s * RTW_WF_LEN_STRIDE];
        if (lane == 0) b0 = atomicAdd(len, 64u * (uint32_t)__popcll(need));
        b0 = s * W.stripe_cap + __shfl(b0, 0);
    }
    const uint64_t llt = leader >= 63 ? (need & ~(1ull << 63)) : (need & ((1ull << leader) - 1ull));
    const uint32_t fresh = b0 + 64u * (uint32_t)__popcll(llt);  // my bucket's fresh block, if it took one
    // holder lanes: the new state of their bucket
    const uint32_t hc = (uint32_t)__popcll(eqh);
    if (hc) {
        const uint32_t hl = (uint32_t)__builtin_ctzll(eqh);
        const uint64_t hlt = hl == 0 ? 0ull : (need & (~0ull >> (64 - hl)));
        const uint32_t hroom = 64u - bf;
        if (hc <= hroom) {
            bf += hc;
        } else {
            bb = b0 + 64u * (uint32_t)__popcll(hlt);
            bf = hc - hroom;
        }
    }
    return rank < room ? base + fill + rank : fresh + (rank - room);
}

// packed path state (see wf_load_ray_it)
template <uint32_t FEAT>
constexpr bool wf_packed() { return (FEAT & (RTW_F_MOVING | RTW_F_LIGHT | RTW_F_GEOM | RTW_F_MEDIUM)) == 0; }
// the 60-B layout of scenes without ray time or medium keys (object scenes): the RNG state rides in the ray
// records' spare words (time, remaining depth), so no rng stream; liveness and depth as in the packed state
template <uint32_t FEAT>
constexpr bool wf_rng_in_ray() { return (FEAT & (RTW_F_MOVING | RTW_F_MEDIUM)) == 0; }
// max_depth - it as a per-lane value: left uniform, the compiler's handling of the split trace (C4) made its
// walk 12-15 % slower with the same walk instructions (profiles/r4_c4_trace_probe/)
__device__ __forceinline__ uint32_t wf_iter_depth(const rtw_launch& L, uint32_t it) {
    uint32_t md = L.max_depth - it;
    asm volatile("" : "+v"(md));
    return md;
}

// the unused slots of the wave's partly filled blocks: dead (depth 0; packed state: d = 0), so the next
// iteration skips them
template <uint32_t FEAT>
__device__ __forceinline__ void wf_close_blocks(const rtw_wf& W, uint32_t it, uint32_t bb, uint32_t bf, bool pk) {
    const rtw_wf_set& O = W.set[(it + 1u) & 1u];
    uint64_t open = __ballot(__lane_id() < RTW_WF_BUCKETS && bf > 0u && bf < 64u);
    while (open) {
        const uint32_t h = (uint32_t)__builtin_ctzll(open);
        open &= open - 1ull;
        const uint32_t base = __shfl(bb, (int)h), fill = __shfl(bf, (int)h);
        if (__lane_id() >= fill) {
            O.ray_d[base + __lane_id()] = make_float4(0, 0, 0, 0);
            if (wf_packed<FEAT>() && pk) O.ray_o[base + __lane_id()] = make_float4(0, 0, 0, 0);
        }
    }
}

__device__ __forceinline__ Ray wf_load_ray(const rtw_wf_set& S, uint32_t slot, uint32_t& depth) {
    const float4 o = S.ray_o[slot], d = S.ray_d[slot];
    Ray r;
    r.o = mk(o.x, o.y, o.z);
    r.time = o.w;
    r.d = mk(d.x, d.y, d.z);
    depth = fbits(d.w);
    return r;
}

__device__ __forceinline__ void wf_store_ray(const rtw_wf_set& S, uint32_t slot, const Ray& r, uint32_t depth) {
    S.ray_o[slot] = make_float4(r.o.x, r.o.y, r.o.z, r.time);
    S.ray_d[slot] = make_float4(r.d.x, r.d.y, r.d.z, __uint_as_float(depth));
}

// the path's RNG state keys ConstantMedium draws (only read in scenes with media)
template <uint32_t FEAT>
__device__ __forceinline__ uint64_t wf_mkey(const rtw_wf_set& S, uint32_t slot) {
    if constexpr ((FEAT & RTW_F_MEDIUM) != 0) return S.rng[slot];
    return 0;
}

// Packed path state (round 4) of static sphere scenes without emitters (BASELINE configs 2-5): no ray time
// is ever read (no moving sphere), no radiance is carried (no emitter), and the remaining depth of every
// path in iteration it's input set is max_depth - it, so a path is three 16-B streams instead of five
// (60 B): ray_o = (o.xyz, d.x), ray_d = (d.y, d.z, thr.x, thr.y), thr = (thr.z, pid, rng lo, rng hi).  A dead
// slot (a closed block's tail) has d = 0: no queued ray has a zero direction (Lambertian replaces a
// near-zero one by the normal, material.zig:47-50; Metal absorbs dot(d, n) <= 0, :68; Dielectric's is a
// unit-length reflection or refraction, :80-98).  The same values in the same registers: bit-identical.
// The 60-B form (every other scene class): ray_o = (o, time), ray_d = (d, remaining depth), thr = (thr.xyz,
// pid), rng, and acc (radiance so far) in scenes with emitters; without ray time or media (wf_rng_in_ray)
// the RNG state's halves replace time and depth and the rng stream is unused.
// the ray of slot `slot` of iteration it's input set; depth 0 = no path.  txy: packed only, thr.xy
template <uint32_t FEAT>
__device__ __forceinline__ Ray wf_load_ray_it(const rtw_launch& L, const rtw_wf_set& S, uint32_t slot, uint32_t it,
                                              uint32_t& depth, float2& txy,
                                              bool pk) {
    if (wf_packed<FEAT>() && pk) {
        const float4 o = S.ray_o[slot], d = S.ray_d[slot];
        Ray r;
        r.o = mk(o.x, o.y, o.z);
        r.d = mk(o.w, d.x, d.y);
        r.time = 0.0f;
        depth = ((fbits(o.w) | fbits(d.x) | fbits(d.y)) << 1) ? wf_iter_depth(L, it) : 0u;  // +-0 components: d = 0
        txy = make_float2(d.z, d.w);
        return r;
    } else if constexpr (wf_rng_in_ray<FEAT>()) {
        const float4 o = S.ray_o[slot], d = S.ray_d[slot];
        Ray r;
        r.o = mk(o.x, o.y, o.z);
        r.d = mk(d.x, d.y, d.z);
        r.time = 0.0f;
        depth = ((fbits(d.x) | fbits(d.y) | fbits(d.z)) << 1) ? wf_iter_depth(L, it) : 0u;
        txy = make_float2(o.w, d.w);  // the RNG state's halves
        return r;
    } else {
        txy = make_float2(0.0f, 0.0f);
        return wf_load_ray(S, slot, depth);
    }
}

// throughput / radiance / RNG state / path id of a live path of iteration it >= 1 (the first bounce's are
// implicit: thr 1, radiance 0, and the camera code makes the RNG state and pid = slot)
template <uint32_t FEAT>
__device__ __forceinline__ void wf_load_rest(const rtw_launch& L, const rtw_wf_set& S, uint32_t slot, uint32_t depth,
                                             float2 txy, f3& thr, f3& acc, uint64_t& rng, uint32_t& pid, bool pk) {
    if (wf_packed<FEAT>() && pk) {
        const float4 c = S.thr[slot];
        thr = mk(txy.x, txy.y, c.x);
        acc = mk(0, 0, 0);
        pid = fbits(c.y);
        rng = (uint64_t)fbits(c.z) | ((uint64_t)fbits(c.w) << 32);
    } else {
        const float4 t4 = S.thr[slot];
        thr = mk(t4.x, t4.y, t4.z);
        pid = fbits(t4.w);
        if constexpr (wf_rng_in_ray<FEAT>()) rng = (uint64_t)fbits(txy.x) | ((uint64_t)fbits(txy.y) << 32);
        else rng = S.rng[slot];
        acc = mk(0, 0, 0);
        if constexpr ((FEAT & RTW_F_LIGHT) != 0) {
            const float4 l4 = S.acc[slot];
            acc = mk(l4.x, l4.y, l4.z);
        }
        (void)L;
        (void)depth;
    }
}

// a surviving path into slot `out` of the output set (depth: its remaining depth after this bounce)
template <uint32_t FEAT>
__device__ __forceinline__ void wf_store_path(const rtw_wf_set& O, uint32_t out, const Ray& r, uint32_t depth, f3 thr,
                                              uint64_t rng, uint32_t pid, f3 acc, bool pk) {
    if (wf_packed<FEAT>() && pk) {
        O.ray_o[out] = make_float4(r.o.x, r.o.y, r.o.z, r.d.x);
        O.ray_d[out] = make_float4(r.d.y, r.d.z, thr.x, thr.y);
        O.thr[out] = make_float4(thr.z, __uint_as_float(pid), __uint_as_float((uint32_t)rng),
                                 __uint_as_float((uint32_t)(rng >> 32)));
        (void)depth;
        (void)acc;
    } else {
        if constexpr (wf_rng_in_ray<FEAT>()) {
            O.ray_o[out] = make_float4(r.o.x, r.o.y, r.o.z, __uint_as_float((uint32_t)rng));
            O.ray_d[out] = make_float4(r.d.x, r.d.y, r.d.z, __uint_as_float((uint32_t)(rng >> 32)));
            (void)depth;
        } else {
            wf_store_ray(O, out, r, depth);
            O.rng[out] = rng;
        }
        O.thr[out] = make_float4(thr.x, thr.y, thr.z, __uint_as_float(pid));
        if constexpr ((FEAT & RTW_F_LIGHT) != 0) O.acc[out] = make_float4(acc.x, acc.y, acc.z, 0);
    }
}

// Iteration 0: path `slot`'s camera ray and RNG state (camera.zig:169-180 with the +1 pixel offset,
// camera.zig:100-101), generated in registers by the kernel that needs them -- the fused step, and both
// the split trace and the split shade (each recomputes it: no ray or RNG state goes through HBM before
// the first bounce).  Called by the whole wave (sphere scenes: get_ray_wave's one disk rejection loop).
// false: padding, or depth 0 (rayColor = 0).
template <uint32_t FEAT>
__device__ __forceinline__ bool wf_camera(const rtw_launch& L, const rtw_wf& W, bool got, uint32_t slot, Ray& r,
                                          rtw_rng& rng) {
    uint32_t s_local = 0, q = 0, pixel = 0, out_idx, x = 0, y = 0;
    bool live = false;
    if (got) {
        wf_path(W, slot, s_local, q);
        live = wf_pixel(L, W, q, pixel, out_idx, x, y) && L.max_depth > 0;
    }
    rng.s = live ? rtw_mix64(L.key0 ^ (((uint64_t)pixel << 32) | (uint64_t)(L.s0 + s_local))) : 0ull;
    r.o = r.d = mk(0, 0, 0);
    r.time = 0;
    if constexpr ((FEAT & (RTW_F_GEOM | RTW_F_MEDIUM)) == 0) {
        r = get_ray_wave(L, live, x + L.pixel_offset, y + L.pixel_offset, rng);
    } else {
        if (live) r = get_ray(L, x + L.pixel_offset, y + L.pixel_offset, rng);
    }
    return live;
}

// a split kernel's input ray: the camera ray in iteration 0's instantiation (CAM, wf_camera: kept
// out of the later iterations' kernels, whose walk would pay for its registers), else the input set's;
// depth 0 = no path.  rng: the camera ray's RNG state (CAM).
template <uint32_t FEAT, bool CAM>
__device__ __forceinline__ Ray wf_input_ray(const rtw_launch& L, const rtw_wf& W, const rtw_wf_set& S,
                                            uint32_t slot, uint32_t it, uint32_t& depth, rtw_rng& rng, float2& txy,
                                            bool pk) {
    if constexpr (CAM) {
        Ray r;
        depth = wf_camera<FEAT>(L, W, true, slot, r, rng) ? L.max_depth : 0u;
        txy = make_float2(0.0f, 0.0f);
        return r;
    }
    rng.s = 0;
    return wf_load_ray_it<FEAT>(L, S, slot, it, depth, txy, pk);
}

// L.geom_lds: copy the scene's quads | members | instances (one contiguous range of the scene
// blob, 16-B aligned) to `lds` and point a copy of L at it (the caller synchronises)
__device__ __forceinline__ rtw_launch stage_geom(const rtw_launch& L, float4* lds) {
    const float4* src = reinterpret_cast<const float4*>(L.quads);
    for (uint32_t k = threadIdx.x; k < L.geom_lds / 16u; k += blockDim.x) lds[k] = src[k];
    rtw_launch G = L;
    const char* base = reinterpret_cast<const char*>(L.quads);
    char* lb = reinterpret_cast<char*>(lds);
    G.quads = reinterpret_cast<const rtw_dev_quad*>(lb);
    G.members = reinterpret_cast<const uint32_t*>(lb + (reinterpret_cast<const char*>(L.members) - base));
    G.insts = reinterpret_cast<const rtw_dev_instance*>(lb + (reinterpret_cast<const char*>(L.insts) - base));
    return G;
}

// The compact node forms a walk can read (traverse_compact):
//   CN_F16_8  16-B nodes, fp16 boxes, 8 octant copies (the default)
//   CN_F16_4  16-B nodes, fp16 boxes, 4 copies by the x and z signs (y slabs by med3)
//   CN_F32_4  32-B nodes, fp32 boxes for packed FMAs, 4 copies (rtw_tuning.compact_nodes 2)
enum { CN_F16_8 = 0, CN_F16_4 = 1, CN_F32_4 = 2 };
// uint4s per node of the launch's compact form
__device__ __forceinline__ uint32_t cn_quads(const rtw_launch& L) { return L.cnode32 ? 2u : 1u; }
template <bool COUNT, bool LDS, int CN>
__device__ __forceinline__ int walk_compact(const rtw_launch& L, const uint4* base, const Ray& r, float& t, Counters& cnt) {
    return traverse_compact<COUNT, LDS, CN != CN_F16_8, CN == CN_F32_4>(L, base, r, t, cnt);
}

// every copy of the compact nodes into this block's LDS, inner nodes' skip offsets rebased to
// absolute LDS addresses (traverse_compact<.., true> steps through them as they are)
__device__ __forceinline__ void stage_clds(const rtw_launch& L, uint4* lds) {
    const uint32_t n4 = L.n_nodes * L.n_orders * cn_quads(L), lb = lds_addr(lds);
    if (L.cnode32) {  // the skip / leaf word is the second uint4's z
        for (uint32_t k = threadIdx.x; k < n4; k += blockDim.x) {
            uint4 c = L.cnodes[k];
            if ((k & 1u) && !(c.z & RTW_LEAF_BIT)) c.z += lb;
            lds[k] = c;
        }
    } else {
        for (uint32_t k = threadIdx.x; k < n4; k += blockDim.x) {
            uint4 c = L.cnodes[k];
            if (!(c.w & RTW_LEAF_BIT)) c.w += lb;
            lds[k] = c;
        }
    }
    __syncthreads();
}

// The two-wide stack walk (rtw_bvh.hip rtw_wide2_nodes: large static sphere SAH trees
// read through L1/L2).  Each step loads one 32-B record: a leaf child's sphere is
// tested at once (Sphere.hit on (0.001, closest), objects.zig:116-136, no box:
// bvh.zig:123-125), an inner child's box with the FMA slab test of the compact walk
// (fp16 bounds, supersets of the padded boxes); of two entered inner children the
// nearer is walked first and the other pushed.  Any visiting order of a superset
// of the boxes the reference walk enters finds the same closest hit (bvh.zig:122-136
// keeps the nearest root; Interval.surrounds is strict).  The hit id is the leaf's
// index in ordering 0 (octant bits 0).  Per-lane stack in the kernel's dynamic LDS,
// entry k at [k * 256 + threadIdx.x] (256-thread blocks, L.w2_stack entries each:
// the tree's inner depth, so it never overflows).
__device__ __forceinline__ void w2_box(uint4 c, const RayTrav& rt, uint32_t sx, uint32_t sy, uint32_t sz,
                                       float closest, float& lo, float& hi) {
    // per axis the (near | far << 16) pair of this ray: swapped where the direction is negative
    const uint32_t x = __builtin_amdgcn_perm(c.x, c.x, sx), y = __builtin_amdgcn_perm(c.y, c.y, sy),
                   z = __builtin_amdgcn_perm(c.z, c.z, sz);
    const float tnx = __builtin_fmaf(h_lo(x), rt.inv.x, rt.oinv.x), tfx = __builtin_fmaf(h_hi(x), rt.inv.x, rt.oinv.x);
    const float tny = __builtin_fmaf(h_lo(y), rt.inv.y, rt.oinv.y), tfy = __builtin_fmaf(h_hi(y), rt.inv.y, rt.oinv.y);
    const float tnz = __builtin_fmaf(h_lo(z), rt.inv.z, rt.oinv.z), tfz = __builtin_fmaf(h_hi(z), rt.inv.z, rt.oinv.z);
    lo = __builtin_fmaxf(__builtin_fmaxf(kTmin, tnx), __builtin_fmaxf(tny, tnz));
    hi = __builtin_fminf(__builtin_fminf(closest, tfx), __builtin_fminf(tfy, tfz));
}

template <bool COUNT>
__device__ __forceinline__ int traverse_wide2(const rtw_launch& L, const Ray& r, float& t_out, Counters& cnt) {
    extern __shared__ uint32_t wf_w2_stack[];
    uint32_t* __restrict__ stk = wf_w2_stack + threadIdx.x;
    const RayTrav rt = ray_trav(r, true);
    constexpr uint32_t KEEP = 0x03020100u, SWAP = 0x01000302u;  // v_perm_b32 byte selectors
    const uint32_t sx = rt.inv.x < 0.0f ? SWAP : KEEP, sy = rt.inv.y < 0.0f ? SWAP : KEEP,
                   sz = rt.inv.z < 0.0f ? SWAP : KEEP;
    const uint4* __restrict__ wn = L.w2nodes;
    float closest = kInf;
    int hit = -1;  // the record slot 2 * node + k of the closest sphere
    uint32_t node = 0, sp = 0;
    for (;;) {
        const uint4 a = wn[2u * node], b = wn[2u * node + 1u];
        const bool f0 = (a.w & RTW_LEAF_BIT) != 0, f1 = (b.w & RTW_LEAF_BIT) != 0;
        if (f0) {
            if constexpr (COUNT) cnt.leaves++;
            sphere_leaf(L, r, rt, mk(ubits(a.x), ubits(a.y), ubits(a.z)), ubits(a.w & ~RTW_LEAF_BIT), 2u * node,
                        closest, hit);
        }
        if (f1) {
            if constexpr (COUNT) cnt.leaves++;
            sphere_leaf(L, r, rt, mk(ubits(b.x), ubits(b.y), ubits(b.z)), ubits(b.w & ~RTW_LEAF_BIT),
                        2u * node + 1u, closest, hit);
        }
        if constexpr (COUNT) cnt.nodes += (f0 ? 0u : 1u) + (f1 ? 0u : 1u);
        float lo0, hi0, lo1, hi1;
        w2_box(a, rt, sx, sy, sz, closest, lo0, hi0);
        w2_box(b, rt, sx, sy, sz, closest, lo1, hi1);
        // next node without nested control flow (an if / else-if chain with the exit in one arm
        // compiles to nested loops: lanes that pop wait for the lanes that descend).  (Stack
        // entries carrying their entry distance, so that stale ones are dropped unloaded, measured
        // slower: C4 trace +4 %.)
        const bool i0 = !f0 && !(hi0 <= lo0), i1 = !f1 && !(hi1 <= lo1);
        const bool second = lo1 < lo0;
        uint32_t nxt = (i0 && !(i1 && second)) ? a.w : b.w;
        if (i0 && i1) stk[sp * 256u] = second ? a.w : b.w;
        sp += (i0 && i1) ? 1u : 0u;
        const bool pop = !(i0 || i1), done = pop && sp == 0;
        if (pop && !done) {
            sp--;
            nxt = stk[sp * 256u];
        }
        if (done) break;
        node = nxt;
    }
    t_out = closest;
    return hit < 0 ? hit : (int)L.w2leaf[hit];
}


// the walk of a static sphere scene through L1/L2: two-wide when the records exist and the FMA slab
// test is allowed (its fp16 boxes are supersets only of boxes padded for |o| <= 7 * extent: make_launch
// clears fast_box for a farther camera, and tuning.fast_box = 0 asks for the exact aabb.zig walk)
template <uint32_t FEAT>
__device__ __forceinline__ int wf_traverse_global(const rtw_launch& L, const Ray& r, float& t, Counters& cnt,
                                                  uint64_t mkey) {
    if constexpr ((FEAT & (RTW_F_GEOM | RTW_F_MEDIUM | RTW_F_MOVING)) == 0) {
        if (L.w2nodes && L.fast_box)
            return L.counters ? traverse_wide2<true>(L, r, t, cnt) : traverse_wide2<false>(L, r, t, cnt);
    }
    return traverse<FEAT>(L.nodes, L, r, t, cnt, mkey);
}

// ---------------------------------------------------------------------------
// Camera-ray candidate lists (iteration 0 of the compact-LDS fused step).
// A wave's camera rays are one 8x8 tile of one sample (wf_pixel), and every ray of
// the tile starts on the defocus disk and passes through the tile's pixel rectangle
// widened by the +-0.5 jitter (Camera.getRay, camera.zig:169-180).  wf_tile_lists
// keeps, per tile, every sphere such a ray can reach (a conservative superset,
// margins far above fp32 rounding) sorted by a lower bound of its ray parameter;
// the step then runs the exact Sphere.hit (objects.zig:116-136, the walk's
// sphere_leaf) on the list in order -- the same code on every lane of the wave, no
// divergent walk -- and stops once every lane's closest hit is nearer than the next
// candidate's bound.  The closest of a superset of the spheres the walk would test
// is the same hit (bvh.zig:122-136 keeps the nearest root), so the image is the
// same; the hit id is the ordering-0 leaf index, as the two-wide walk's.  A tile
// with more than L.tile_lists candidates walks the tree.
//
// Geometry: with f the unit normal of the pixel plane (du x dv) and h its distance
// from the camera centre (the focus distance), every ray's depth grows by h per unit
// of t, so all rays reach depth z = (C - centre).f at t = z / h, where they lie in
// the tile's rectangle scaled by t plus a disk of radius |1 - t| * r_disk.  A ray
// passes within rho of C only if that cross-section comes within rho * sec(phi) of
// C (phi: the largest angle of a ray to f); a hit has depth >= z - rho, i.e.
// t >= (z - rho) / h.  Spheres wholly behind the camera plane (z < -rho) are never kept (a ray's
// depth is t * h > 0); those straddling it are kept when near the axis (tile_reach).
// The tile's ray set (see above): pixel rectangle at depth h in the (uh, vh) frame around the
// camera centre, defocus radius rd, sec of the widest ray angle
struct TileFrustum {
    f3 ctr, fz, uh, vh;
    float h, ru0, ru1, rv0, rv1, rd, sec;
    bool ok;  // false: no usable frame (the tile walks the tree)
};

__device__ __forceinline__ TileFrustum tile_frustum(const rtw_launch& L, float x0, float x1, float y0, float y1) {
    TileFrustum F;
    const f3 du = ld3(L.du), dv = ld3(L.dv);
    F.ctr = ld3(L.center);
    const f3 fw = cross(du, dv);
    const float fl = __builtin_sqrtf(length_squared(fw)), ul = __builtin_sqrtf(length_squared(du)),
                vl = __builtin_sqrtf(length_squared(dv));
    F.fz = divs(fw, fl);
    F.uh = divs(du, ul);
    F.vh = divs(dv, vl);
    const f3 p0 = ld3(L.pixel00) - F.ctr;
    F.h = dot(p0, F.fz);
    const float pu = dot(p0, F.uh), pv = dot(p0, F.vh);
    // the pixel plane must face the rays and du, dv be orthogonal (Camera.init)
    F.ok = F.h > 0.0f && fl > 0.0f && __builtin_fabsf(dot(du, dv)) <= 1e-4f * ul * vl;
    const float off = (float)L.pixel_offset;
    F.ru0 = pu + (x0 + off - 0.5f) * ul;
    F.ru1 = pu + (x1 + off + 0.5f) * ul;
    F.rv0 = pv + (y0 + off - 0.5f) * vl;
    F.rv1 = pv + (y1 + off + 0.5f) * vl;
    F.rd = L.defocus_angle > 0 ? fmaxf(__builtin_sqrtf(length_squared(ld3(L.disk_u))),
                                       __builtin_sqrtf(length_squared(ld3(L.disk_v)))) : 0.0f;
    const float mu = fmaxf(__builtin_fabsf(F.ru0), __builtin_fabsf(F.ru1)),
                mv = fmaxf(__builtin_fabsf(F.rv0), __builtin_fabsf(F.rv1));
    const float tphi = (__builtin_sqrtf(mu * mu + mv * mv) + F.rd) / F.h;
    F.sec = __builtin_sqrtf(1.0f + tphi * tphi) * 1.001f;
    return F;
}

// Can a ray of the tile pass within rho of c?  (conservative; tlow: a lower bound of the ray
// parameter of any such hit, 0 when the sphere reaches the camera plane)
__device__ __forceinline__ bool tile_reach(const TileFrustum& F, f3 c, float rho, float& tlow) {
    const f3 cc = c - F.ctr;
    const float z = dot(cc, F.fz), cu = dot(cc, F.uh), cv = dot(cc, F.vh);
    const float slack = 1e-3f * (__builtin_fabsf(z) + __builtin_fabsf(cu) + __builtin_fabsf(cv) + rho) + 1e-5f;
    tlow = 0.0f;
    if (z < -(rho + slack)) return false;  // wholly behind the camera plane: rays only go forward (t > 0)
    if (!(z > rho + slack)) {
        // straddles the camera plane: a hit has depth in (0, z + rho], so t <= t1 and the hit point is
        // within |1 - t| rd + t |T| <= max(1, t1) rd + t1 |T|max of the axis (T: the pixel-plane target)
        const float t1 = fmaxf(0.0f, (z + rho + slack) / F.h);
        const float tmax = __builtin_sqrtf(fmaxf(F.ru0 * F.ru0, F.ru1 * F.ru1) + fmaxf(F.rv0 * F.rv0, F.rv1 * F.rv1));
        const float lat = __builtin_sqrtf(cu * cu + cv * cv);
        return !(lat > rho + fmaxf(1.0f, t1) * F.rd + t1 * tmax + slack);  // NaN: tested
    }
    const float t = z / F.h;
    const float dx = fmaxf(0.0f, fmaxf(t * F.ru0 - cu, cu - t * F.ru1));
    const float dy = fmaxf(0.0f, fmaxf(t * F.rv0 - cv, cv - t * F.rv1));
    const float gap = __builtin_sqrtf(dx * dx + dy * dy) - __builtin_fabsf(1.0f - t) * F.rd;
    tlow = fmaxf(0.0f, (z - rho - slack) / F.h * 0.9999f);
    return !(gap > rho * F.sec + slack);
}

// the tile's pixel bounds over its lanes' pixels (wave-wide min / max); false: no pixel rendered
__device__ __forceinline__ bool tile_bounds(const rtw_launch& L, const rtw_wf& W, uint32_t q, float& x0, float& x1,
                                            float& y0, float& y1) {
    uint32_t pixel, out_idx, x = 0, y = 0;
    const bool ok = wf_pixel(L, W, q, pixel, out_idx, x, y);
    x0 = ok ? (float)x : 1e30f; x1 = ok ? (float)x : -1e30f;
    y0 = ok ? (float)y : 1e30f; y1 = ok ? (float)y : -1e30f;
    for (int o = 32; o > 0; o >>= 1) {
        x0 = fminf(x0, __shfl_xor(x0, o));
        x1 = fmaxf(x1, __shfl_xor(x1, o));
        y0 = fminf(y0, __shfl_xor(y0, o));
        y1 = fmaxf(y1, __shfl_xor(y1, o));
    }
    return x0 <= x1;
}

// write tile's list from (tlow, ordering-0 leaf index) pairs in LDS, ranked by (tlow, index)
__device__ __forceinline__ void tile_emit(const rtw_launch& L, const rtw_wf& W, uint32_t tile, const float* s_t,
                                          const uint32_t* s_id, uint32_t count, uint32_t k) {
    if (k >= count) return;
    const float me = s_t[k];
    uint32_t rank = 0;
    for (uint32_t j = 0; j < count; j++) rank += (s_t[j] < me || (s_t[j] == me && j < k)) ? 1u : 0u;
    const uint32_t id = s_id[k];
    const float4 A = L.nodes[2u * id], B = L.nodes[2u * id + 1u];  // ordering 0 leaf: center, radius
    const float rr = B.x * B.x;  // objects.zig:126, as the compact nodes
    uint4* e = W.tl + 2u * ((size_t)tile * RTW_TL_MAX + rank);
    e[0] = make_uint4(fbits(A.x), fbits(A.y), fbits(A.z), fbits(rr));
    e[1] = make_uint4(id, fbits(me), 0u, 0u);
}

// small trees: one 64-lane block per tile scans every leaf of ordering 0
__global__ __launch_bounds__(64) void wf_tile_lists(rtw_launch L, rtw_wf W) {
    __shared__ float s_t[RTW_TL_MAX];
    __shared__ uint32_t s_id[RTW_TL_MAX];
    const uint32_t tile = blockIdx.x, lane = threadIdx.x;
    float x0, x1, y0, y1;
    if (!tile_bounds(L, W, tile * 64u + lane, x0, x1, y0, y1)) {  // no pixel of the tile is rendered
        if (lane == 0) W.tl_count[tile] = 0;
        return;
    }
    const TileFrustum F = tile_frustum(L, x0, x1, y0, y1);
    uint32_t count = 0;
    bool over = !F.ok;
    for (uint32_t base = 0; base < L.n_nodes && !over; base += 64u) {
        const uint32_t k = base + lane;
        bool cand = false;
        float tlow = 0.0f;
        if (k < L.n_nodes) {
            const uint4 c = L.cnodes[k * cn_quads(L)];  // ordering 0 (the 32-B form: leaf flag in the second uint4)
            const bool leaf = L.cnode32 ? (L.cnodes[2u * k + 1u].z & RTW_LEAF_BIT) != 0 : (c.w & RTW_LEAF_BIT) != 0;
            if (leaf)
                cand = tile_reach(F, mk(ubits(c.x), ubits(c.y), ubits(c.z)), __builtin_sqrtf(ubits(c.w & ~RTW_LEAF_BIT)),
                                  tlow);
        }
        const uint64_t m = __ballot(cand);
        const uint32_t n = (uint32_t)__popcll(m);
        if (count + n > L.tile_lists) {
            over = true;
            break;
        }
        if (cand) {
            const uint32_t at = count + (uint32_t)__popcll(m & ((lane == 0) ? 0ull : (~0ull >> (64 - lane))));
            s_t[at] = tlow;
            s_id[at] = k;
        }
        count += n;
    }
    if (over) {
        if (lane == 0) W.tl_count[tile] = RTW_TL_WALK;
        return;
    }
    __syncthreads();
    tile_emit(L, W, tile, s_t, s_id, count, lane);
    if (lane == 0) W.tl_count[tile] = count;
}

// large trees: a 64-lane block builds 64 tiles' lists, lane j walking tile j's frustum down the
// ordering-0 tree (32-B nodes; an inner box is kept when its bounding sphere is reachable)
__global__ __launch_bounds__(64) void wf_tile_lists_walk(rtw_launch L, rtw_wf W) {
    __shared__ float s_t[64][RTW_TL_MAX + 1];
    __shared__ uint32_t s_id[64][RTW_TL_MAX + 1];
    const uint32_t lane = threadIdx.x, t0 = blockIdx.x * 64u, n_tiles = W.n_pix >> 6;
    uint32_t count = 0;
    bool over = false, empty = false;
    TileFrustum F;
    for (uint32_t j = 0; j < 64; j++) {  // the bounds of tile t0 + j, wave-wide; lane j keeps them
        float x0 = 0, x1 = 0, y0 = 0, y1 = 0;
        bool any = false;
        if (t0 + j < n_tiles) any = tile_bounds(L, W, (t0 + j) * 64u + lane, x0, x1, y0, y1);
        if (lane == j) {
            empty = !any;
            F = tile_frustum(L, x0, x1, y0, y1);
        }
    }
    const uint32_t tile = t0 + lane;
    if (tile < n_tiles && !empty) {
        over = !F.ok;
        uint32_t i = 0;
        while (i < L.n_nodes && !over) {
            const float4 A = L.nodes[2u * i], B = L.nodes[2u * i + 1u];
            const uint32_t w = fbits(A.w);
            float tlow;
            if (w & RTW_LEAF_BIT) {
                if (tile_reach(F, mk(A.x, A.y, A.z), __builtin_fabsf(B.x), tlow)) {
                    if (count == L.tile_lists) over = true;
                    else {
                        s_t[lane][count] = tlow;
                        s_id[lane][count] = i;
                        count++;
                    }
                }
                i = w & RTW_SKIP_MASK;
            } else {
                const f3 lo = mk(A.x, A.y, A.z), hi = mk(B.x, B.y, B.z);
                const f3 m = (lo + hi) * splat(0.5f);
                const float rad = __builtin_sqrtf(length_squared(hi - lo)) * 0.5001f + 1e-5f;
                i = tile_reach(F, m, rad, tlow) ? i + 1u : (w & RTW_SKIP_MASK);
            }
        }
    }
    __syncthreads();
    if (tile >= n_tiles) return;
    if (empty) {
        W.tl_count[tile] = 0;
        return;
    }
    if (over) {
        W.tl_count[tile] = RTW_TL_WALK;
        return;
    }
    for (uint32_t k = 0; k < count; k++) tile_emit(L, W, tile, s_t[lane], s_id[lane], count, k);
    W.tl_count[tile] = count;
}

// The closest hit of a camera ray from its tile's list (wave-uniform: every lane of
// the wave is a ray of `tile`); RTW_TL_WALK -> false (walk the tree)
template <bool COUNT>
__device__ __forceinline__ bool wf_tile_hit(const rtw_launch& L, const rtw_wf& W, uint32_t tile, const Ray& r, int& hit,
                                            float& t_out, Counters& cnt) {
    tile = __builtin_amdgcn_readfirstlane(tile);
    const uint32_t n = W.tl_count[tile];
#if defined(RTW_DIAG_WALK) && defined(__HIP_DEVICE_COMPILE__)
    const bool dlead = dg_leader();
    if (dlead) atomicAdd(&rtw_diag_walk[n == RTW_TL_WALK ? 10 : 8], 1ull);
#endif
    if (n == RTW_TL_WALK) return false;
    const RayTrav rt = ray_trav(r, true);
    const uint4* __restrict__ e = W.tl + 2u * (size_t)tile * RTW_TL_MAX;
    float closest = kInf;
    hit = -1;
#if defined(RTW_DIAG_WALK) && defined(__HIP_DEVICE_COMPILE__)
    uint32_t tested = 0, exact = 0;
#endif
    for (uint32_t k = 0; k < n; k++) {
        const uint4 a = e[2u * k], b = e[2u * k + 1u];
        if (!__ballot(!(closest < ubits(b.y)))) break;  // every lane's hit is nearer than the rest can be
        if constexpr (COUNT) cnt.leaves++;
#if defined(RTW_DIAG_WALK) && defined(__HIP_DEVICE_COMPILE__)
        WalkDiag dgl;
        sphere_leaf(L, r, rt, mk(ubits(a.x), ubits(a.y), ubits(a.z)), ubits(a.w), b.x, closest, hit, &dgl);
        tested++;
        exact += __ballot(dgl.lexact != 0) ? 1u : 0u;
#else
        sphere_leaf(L, r, rt, mk(ubits(a.x), ubits(a.y), ubits(a.z)), ubits(a.w), b.x, closest, hit);
#endif
    }
#if defined(RTW_DIAG_WALK) && defined(__HIP_DEVICE_COMPILE__)
    if (dlead) {
        atomicAdd(&rtw_diag_walk[9], (unsigned long long)tested);
        atomicAdd(&rtw_diag_walk[11], (unsigned long long)exact);
    }
#endif
    t_out = closest;
    return true;
}

// trace: closest hit per ray of the input set (no shading state in registers)
template <uint32_t FEAT, bool LDS, bool CAM = false>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(wf_split_wpe<FEAT>(RTW_WPE_TRACE)))) void wf_trace(rtw_launch L, rtw_wf W, uint32_t it) {
    // the stripes shade(it) appends to start empty (they were iteration it-1's input)
    if (blockIdx.x == 0) W.len[(it + 1u) % 3u][threadIdx.x * RTW_WF_LEN_STRIDE] = 0;
    static_assert(RTW_WF_STRIPES == 256, "one block zeroes the stripe counters");
    const rtw_wf_set& S = W.set[it & 1u];
    Counters cnt;
    if constexpr (LDS) {
        // the node array(s) staged in LDS: the walk's loads become ds_read_b128
        extern __shared__ float4 wf_lds_nodes[];
        const uint32_t n4 = 2u * L.n_nodes * L.n_orders;
        for (uint32_t k = threadIdx.x; k < n4; k += 256u) wf_lds_nodes[k] = L.nodes[k];
        auto run = [&](const rtw_launch& G) {  // G: geometry statically in LDS or not
            for (WfIter e(W, it); e.more(); e.next()) {
                uint32_t slot;
                if (e.get(W, slot)) {
                    uint32_t depth;
                    rtw_rng rng;
                    float2 txy;
                    const Ray r = wf_input_ray<FEAT, CAM>(G, W, S, slot, it, depth, rng, txy, true);
                    if (depth) {
                        float t;
                        const int h = traverse<FEAT>(wf_lds_nodes, G, r, t, cnt, CAM ? rng.s : wf_mkey<FEAT>(S, slot));
                        W.hit[slot] = make_float2(t, __int_as_float(h));
                        cnt.rays++;
                    }
                }
            }
        };
        if constexpr ((FEAT & RTW_F_GEOM) != 0) {
            if (L.geom_lds) {
                const rtw_launch G = stage_geom(L, wf_lds_nodes + n4);
                __syncthreads();
                run(G);
                flush_counters(L, cnt, 0);
                return;
            }
        }
        __syncthreads();
        run(L);
        flush_counters(L, cnt, 0);
        return;
    }
    for (WfIter e(W, it); e.more(); e.next()) {
        uint32_t slot;
        if (e.get(W, slot)) {
            uint32_t depth;
            rtw_rng rng;
            float2 txy;
            const Ray r = wf_input_ray<FEAT, CAM>(L, W, S, slot, it, depth, rng, txy, true);
            if (depth) {
                float t = kInf;
                int h = -1;
                bool listed = false;
                if constexpr ((FEAT & (RTW_F_GEOM | RTW_F_MEDIUM | RTW_F_MOVING)) == 0) {
                    if (it == 0 && W.tl_count) {  // camera rays (slot = path id): the tile's candidate list
                        const uint32_t tile = (slot >> 6) / W.n_s;
                        listed = L.counters ? wf_tile_hit<true>(L, W, tile, r, h, t, cnt)
                                            : wf_tile_hit<false>(L, W, tile, r, h, t, cnt);
                    }
                }
                if (!listed) h = wf_traverse_global<FEAT>(L, r, t, cnt, CAM ? rng.s : wf_mkey<FEAT>(S, slot));
                W.hit[slot] = make_float2(t, __int_as_float(h));
                cnt.rays++;
            }
        }
    }
    flush_counters(L, cnt, 0);
}

// trace over the compact nodes staged in LDS (all octant copies of a small tree,
// e.g. BASELINE config 2: 8 x 969 x 16 B = 124 KB): 1024-thread blocks share one
// copy (one block per CU), ds_read_b128 instead of vector-memory gathers
template <uint32_t FEAT, bool CAM = false, int CN = CN_F16_8>
__global__ __launch_bounds__(1024) void wf_trace_clds(rtw_launch L, rtw_wf W, uint32_t it) {
    static_assert((FEAT & (RTW_F_GEOM | RTW_F_MEDIUM | RTW_F_MOVING)) == 0, "static sphere scenes");
    if (blockIdx.x == 0 && threadIdx.x < RTW_WF_STRIPES) W.len[(it + 1u) % 3u][threadIdx.x * RTW_WF_LEN_STRIDE] = 0;
    extern __shared__ uint4 wf_clds[];
    stage_clds(L, wf_clds);
    const rtw_wf_set& S = W.set[it & 1u];
    Counters cnt;
    for (WfIter e(W, it); e.more(); e.next()) {
        uint32_t slot;
        if (e.get(W, slot)) {
            uint32_t depth;
            rtw_rng rng;
            float2 txy;
            const Ray r = wf_input_ray<FEAT, CAM>(L, W, S, slot, it, depth, rng, txy, true);
            if (depth) {
                float t;
                const int h = L.counters ? walk_compact<true, true, CN>(L, wf_clds, r, t, cnt)
                                         : walk_compact<false, true, CN>(L, wf_clds, r, t, cnt);
                W.hit[slot] = make_float2(t, __int_as_float(h));
                cnt.rays++;
            }
        }
    }
    flush_counters(L, cnt, 0);
}

// shade: emission / background and Material.scatter; a surviving path's state
// moves to its slot in the other set; an ending path stores its radiance by id
template <uint32_t FEAT, bool CAM>
__device__ __forceinline__ void wf_shade_body(const rtw_launch& L, const rtw_wf& W, uint32_t it);

template <uint32_t FEAT, bool CAM = false>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(wf_split_wpe<FEAT>(RTW_WPE_SHADE)))) void wf_shade(rtw_launch L, rtw_wf W, uint32_t it) {
    if constexpr ((FEAT & RTW_F_GEOM) != 0) {
        if (L.geom_lds) {  // quads / members / instances in LDS (hit records of object scenes)
            extern __shared__ float4 wf_shade_geom[];
            const rtw_launch G = stage_geom(L, wf_shade_geom);
            __syncthreads();
            wf_shade_body<FEAT, CAM>(G, W, it);
            return;
        }
    }
    wf_shade_body<FEAT, CAM>(L, W, it);
}

template <uint32_t FEAT, bool CAM>
__device__ __forceinline__ void wf_shade_body(const rtw_launch& L, const rtw_wf& W, uint32_t it) {
    const rtw_wf_set& S = W.set[it & 1u];
    const rtw_wf_set& O = W.set[(it + 1u) & 1u];
    const bool bucketed = it < W.sort_iters;
    uint32_t bb = 0, bf = 64;  // lane b: bucket b's open block (wf_push_bucketed)
    for (WfIter e(W, it); e.more(); e.next()) {
        bool push = false;
        uint32_t slot = 0, pid = 0, depth = 0;
        f3 thr = mk(0, 0, 0), acc = mk(0, 0, 0);
        rtw_rng rng;
        rng.s = 0;
        Ray sc, rin;
        HitPrep hp;
        bool hitp = false, need_uv = false;
        if (e.get(W, slot)) {
            float2 txy;
            const Ray r = wf_input_ray<FEAT, CAM>(L, W, S, slot, it, depth, rng, txy, true);
            if (depth) {
                const float2 h = W.hit[slot];
                const int hit = __float_as_int(h.y);
                if (CAM) {
                    pid = slot;
                    thr = mk(1, 1, 1);
                    acc = mk(0, 0, 0);
                } else {
                    uint64_t rs;
                    wf_load_rest<FEAT>(L, S, slot, depth, txy, thr, acc, rs, pid, true);
                    rng.s = rs;
                }
                if (hit < 0) {
                    acc = acc + thr * background(L, r);
                } else {
                    if constexpr ((FEAT & (RTW_F_GEOM | RTW_F_MEDIUM)) == 0) {
                        // sphere scenes: the split form of the fused step (hit record, then one
                        // randomUnitVector rejection loop for the wave, then the material)
                        hp = hit_prep<FEAT>(L.nodes, L, r, hit, h.x);
                        hitp = true;
                        need_uv = needs_unit_vector<FEAT>(hp.m.kind);
                        rin = r;
                    } else {
                        f3 att;
                        if (shade<FEAT>(L.nodes, L, r, hit, h.x, rng, thr, acc, att, sc) && depth > 1) {
                            thr = thr * att;
                            push = true;
                        }
                    }
                }
            }
        }
        if constexpr ((FEAT & (RTW_F_GEOM | RTW_F_MEDIUM)) == 0) {
            float uv3[3] = {0.0f, 0.0f, 0.0f};
            if (need_uv) seq_reject<3>(rng, uv3);
            if (hitp) {
                const f3 ruv = need_uv ? unit_vector(mk(uv3[0], uv3[1], uv3[2])) : mk(0, 0, 0);
                f3 att;
                if (scatter_finish<FEAT>(L, rin, hp, ruv, rng, thr, acc, att, sc) && depth > 1) {
                    thr = thr * att;
                    push = true;
                }
            }
        }
        if (depth && !push) W.ls[pid] = rtw_rgb{acc.x, acc.y, acc.z};
        if (CAM && !depth) W.ls[slot] = rtw_rgb{0.0f, 0.0f, 0.0f};  // padding, rayColor(r, 0) = 0
        const uint32_t out = bucketed ? wf_push_bucketed(W, it, push, push ? wf_bucket(sc.d) & W.sort_mask : 0u, bb, bf)
                                      : wf_push(W, it, push);
        if (push) wf_store_path<FEAT>(O, out, sc, depth - 1, thr, rng.s, pid, acc, true);
    }
    if (bucketed) wf_close_blocks<FEAT>(W, it, bb, bf, true);
}

// tail: the paths still queued after the last wavefront iteration, each to
// completion; a lane whose path ends takes the wave's next path at once.
// CLDS: the walk reads the compact nodes staged in LDS (`lds`) instead of L1/L2.
// CNT (every kernel with a counted form): 0 = no device counters (the product launches: their registers and
// atomics compile away), 1 = the counted pass (rtw_render_opts.counters), 2 = decided per launch by L.counters
// PARK (`park`: 2 x 256 float4 of LDS, 256-thread blocks): the path's throughput, radiance, id and depth wait in
// LDS while its ray walks, so their registers are free for the walk (object scenes' LDS tail)
template <uint32_t FEAT, bool CLDS, int CN = CN_F16_8, int CNT = 2, bool PARK = false>
__device__ __forceinline__ void wf_tail_body(const rtw_launch& L, const rtw_wf& W, uint32_t it, const uint4* lds,
                                             const float4* nodes = nullptr, float4* park = nullptr) {
    const uint32_t lane = __lane_id();
    const uint64_t lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
    const rtw_wf_set& S = W.set[it & 1u];
    Counters cnt;
    uint32_t cursor = 0, pid = 0, depth = 0;
    bool active = false, exhausted = false;
    Ray r;
    f3 thr = mk(0, 0, 0), acc = mk(0, 0, 0);
    rtw_rng rng;
    rng.s = 0;
    // Dynamic input (W.deal, rtw_tuning.deal bit 2): the wave claims 64-slot chunks of the input stripes from one
    // counter as its lanes run dry, one claim issued a chunk ahead, so the tail's end is set by its longest
    // paths, not by a wave whose static share held more of them (C4: tail 56.7 -> 45.3 ms): chunk g of the
    // counter is chunk g / 256 of stripe g % 256.  (Claims per stripe group and a two-launch tail lost their
    // A/Bs: diag/deal_tail_modes.patch.)
    const uint32_t* lens = W.len[it % 3u];
    uint32_t gcur = 0, gnext = 0, limit = 0;  // wave-uniform; gnext lane 0's
    const bool dyn = W.deal && (W.deal_mode & 2u);
    uint32_t* ctr = W.deal;
    if (dyn) {
        uint32_t mx = 0;
        for (uint32_t k = lane; k < RTW_WF_STRIPES; k += 64u) mx = max(mx, lens[k * RTW_WF_LEN_STRIDE]);
        for (int o = 32; o > 0; o >>= 1) mx = max(mx, (uint32_t)__shfl_xor((int)mx, o));
        limit = ((mx + 63u) >> 6) * RTW_WF_STRIPES;
        gcur = __builtin_amdgcn_readfirstlane(wf_claim(ctr));
        gnext = wf_claim(ctr);
        exhausted = gcur >= limit;
    }
    for (;;) {
        const uint64_t need = __ballot(!active);
        if (need && !exhausted && dyn) {
            const uint32_t m = cursor + (uint32_t)__popcll(need & lt);  // element m of the wave's claimed chunks
            const uint32_t n_need = (uint32_t)__popcll(need);
            const uint32_t gn = __builtin_amdgcn_readfirstlane(gnext);
            if (!active) {
                const uint32_t g = (m >> 6) == (cursor >> 6) ? gcur : gn;
                const uint32_t s = g % RTW_WF_STRIPES;
                const uint32_t e = ((g / RTW_WF_STRIPES) << 6) | (m & 63u);
                if (g < limit && e < lens[s * RTW_WF_LEN_STRIDE]) {
                    float2 txy;
                    const uint32_t slot = s * W.stripe_cap + e;
                    r = wf_load_ray_it<FEAT>(L, S, slot, it, depth, txy, W.packed != 0u);
                    uint64_t rs = 0;
                    if (depth) wf_load_rest<FEAT>(L, S, slot, depth, txy, thr, acc, rs, pid, W.packed != 0u);
                    rng.s = rs;
                    active = depth != 0;
                }
            }
            if (((cursor + n_need) >> 6) != (cursor >> 6)) {  // the current chunk is used up: the next one
                gcur = gn;
                gnext = wf_claim(ctr);
            }
            cursor += n_need;
            exhausted = gcur >= limit;
        } else if (need && !exhausted) {
            const uint32_t m = cursor + (uint32_t)__popcll(need & lt);
            cursor += (uint32_t)__popcll(need);
            bool end = false;
            uint32_t slot = 0;
            const bool ok = wf_nth(W, it, m, slot, end);
            exhausted = __ballot(end && !active) == need;
            if (!active && ok) {  // (the tail's input is iteration it >= 1's: wf_iters >= 1)
                float2 txy;
                r = wf_load_ray_it<FEAT>(L, S, slot, it, depth, txy, W.packed != 0u);
                uint64_t rs = 0;
                if (depth) wf_load_rest<FEAT>(L, S, slot, depth, txy, thr, acc, rs, pid, W.packed != 0u);
                rng.s = rs;
                active = depth != 0;
            }
        }
        if (!__ballot(active)) {
            if (exhausted) break;
            continue;
        }
        bool done = true, hitp = false, need_uv = false;
        HitPrep hp;
        int ohit = -1;  // object scenes: the hit shaded after the wave's rejection loop
        float ot = 0.0f;
        if (active) {  // one more iteration of rayColor
            if constexpr (CNT != 0) {
                cnt.rays++;
                cnt.tail_rays++;
            }
            if constexpr (PARK) {
                park[threadIdx.x] = make_float4(thr.x, thr.y, thr.z, acc.x);
                park[256u + threadIdx.x] = make_float4(acc.y, acc.z, __uint_as_float(pid), __uint_as_float(depth));
            }
            float t;
            int hit;
            if constexpr (CLDS && CNT == 2)
                hit = L.counters ? walk_compact<true, true, CN>(L, lds, r, t, cnt)
                                 : walk_compact<false, true, CN>(L, lds, r, t, cnt);
            else if constexpr (CLDS)
                hit = walk_compact<CNT == 1, true, CN>(L, lds, r, t, cnt);
            else
                hit = nodes ? traverse<FEAT, false>(nodes, L, r, t, cnt, rng.s)  // the LDS stage
                            : wf_traverse_global<FEAT>(L, r, t, cnt, rng.s);
            if constexpr (PARK) {
                asm volatile("" ::: "memory");  // (no forwarding of the stores past the walk: the reload is real)
                const float4 p0 = park[threadIdx.x], p1 = park[256u + threadIdx.x];
                thr = mk(p0.x, p0.y, p0.z);
                acc = mk(p0.w, p1.x, p1.y);
                pid = fbits(p1.z);
                depth = fbits(p1.w);
            }
            if (hit < 0) {
                acc = acc + thr * background(L, r);
            } else if constexpr ((FEAT & ~RTW_F_CHECKER) == 0) {
                // untextured static sphere scenes: the fused step's split form (C2 tail -10 %, C4 -5 % over the
                // nested form; the textured C5 tail +5 %: nested form there), in the fused step's order -- the
                // material kind, the wave's rejection loop, then the hit record: the compact-LDS tail (C2) -0.9 %
                // tail time and no scratch left; the two-wide tail (C4), once at 6 waves, -2.1 % (at 5 waves it had
                // lost 1.2 %: profiles/r6_late_rest/f/, profiles/r6_waves/k/)
                hitp = true;
                ohit = hit;
                ot = t;
                need_uv = needs_unit_vector<FEAT>(hit_material_kind<FEAT>(L.nodes, L, hit));
            } else if constexpr ((FEAT & RTW_F_GEOM) != 0) {
                // object scenes: as the fused step's object path, the wave's shared rejection loop
                // (wf_reject3) before the hit record, on the material kind alone
                ohit = hit;
                ot = t;
                need_uv = needs_unit_vector<FEAT>(hit_material_kind<FEAT>(L.nodes, L, hit));
            } else {
                f3 att;
                Ray sc;
                if (shade<FEAT>(L.nodes, L, r, hit, t, rng, thr, acc, att, sc) && depth > 1) {
                    thr = thr * att;
                    r = sc;
                    depth--;
                    done = false;
                }
            }
        }
        if constexpr ((FEAT & RTW_F_GEOM) != 0) {
            float uv3[3] = {0.0f, 0.0f, 0.0f};
            wf_reject3(need_uv, rng, uv3);  // the whole wave
            if (ohit >= 0) {
                const HitPrep h = hit_prep<FEAT>(L.nodes, L, r, ohit, ot);
                const f3 ruv = need_uv ? unit_vector(mk(uv3[0], uv3[1], uv3[2])) : mk(0, 0, 0);
                f3 att;
                Ray sc;
                if (scatter_finish<FEAT>(L, r, h, ruv, rng, thr, acc, att, sc) && depth > 1) {
                    thr = thr * att;
                    r = sc;
                    depth--;
                    done = false;
                }
            }
        }
        if constexpr ((FEAT & ~RTW_F_CHECKER) == 0) {
            float uv3[3] = {0.0f, 0.0f, 0.0f};
            // the wave-cooperative loop (same candidates, same RNG states as seq_reject<3>): C2 +1.4 %
            if constexpr (CLDS) wf_reject3(need_uv, rng, uv3);
            else if (need_uv) seq_reject<3>(rng, uv3);  // (the cooperative loop here: +-0, profiles/r6_waves/k/)
            if (hitp) hp = hit_prep<FEAT>(L.nodes, L, r, ohit, ot);
            if (hitp) {
                const f3 ruv = need_uv ? unit_vector(mk(uv3[0], uv3[1], uv3[2])) : mk(0, 0, 0);
                f3 att;
                Ray sc;
                if (scatter_finish<FEAT>(L, r, hp, ruv, rng, thr, acc, att, sc) && depth > 1) {
                    thr = thr * att;
                    r = sc;
                    depth--;
                    done = false;
                }
            }
        }
        if (active && done) {
            W.ls[pid] = rtw_rgb{acc.x, acc.y, acc.z};
            active = false;
        }
    }
    if constexpr (CNT != 0) flush_counters(L, cnt, 0);
}

template <uint32_t FEAT>
__global__ __launch_bounds__(256) void wf_tail(rtw_launch L, rtw_wf W, uint32_t it) {
    wf_tail_body<FEAT, false>(L, W, it, nullptr);
}
// untextured static sphere scenes: capped at 96 VGPRs for 5 waves/SIMD (no spills there; the
// split shading form took it to 98 = 4 waves: C4 tail +3 %); other scene classes would spill
template <uint32_t FEAT, int CNT = 2>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(RTW_WPE_TAIL_W5))) void wf_tail_w5(rtw_launch L, rtw_wf W, uint32_t it) {
    wf_tail_body<FEAT, false, CN_F16_8, CNT>(L, W, it, nullptr);
}

// L.shade_lds: the same for the materials | textures | image records (small scenes)
__device__ __forceinline__ rtw_launch stage_shade(const rtw_launch& L, float4* lds) {
    const float4* src = reinterpret_cast<const float4*>(L.mats);
    for (uint32_t k = threadIdx.x; k < L.shade_lds / 16u; k += blockDim.x) lds[k] = src[k];
    rtw_launch G = L;
    const char* base = reinterpret_cast<const char*>(L.mats);
    char* lb = reinterpret_cast<char*>(lds);
    G.mats = reinterpret_cast<const rtw_dev_material*>(lb);
    G.texs = reinterpret_cast<const rtw_dev_texture*>(lb + (reinterpret_cast<const char*>(L.texs) - base));
    G.img_info = reinterpret_cast<const rtw_dev_image*>(lb + (reinterpret_cast<const char*>(L.img_info) - base));
    return G;
}

// the 32-B node array(s) staged in LDS (small object scenes: Cornell), + L.geom_lds bytes of geometry
template <uint32_t FEAT, int CNT = 2>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(wf_tail_lds_wpe<FEAT>()))) void wf_tail_lds(rtw_launch L, rtw_wf W, uint32_t it) {
    extern __shared__ float4 wf_tail_nodes[];
    // (the media class only: the all-features class of simple_light carries the medium bit too, and lost with it)
    constexpr bool kPark = RTW_TAIL_PARK && (FEAT & RTW_F_MEDIUM) != 0 &&
                           (FEAT & (RTW_F_IMAGE | RTW_F_NOISE | RTW_F_MOVING)) == 0;
    __shared__ float4 park_lds[kPark ? 512 : 1];
    float4* park = park_lds;
    const uint32_t n4 = 2u * L.n_nodes * L.n_orders;
    for (uint32_t k = threadIdx.x; k < n4; k += 256u) wf_tail_nodes[k] = L.nodes[k];
    // then materials, then geometry: one call per combination (statically LDS pointers)
    const bool sl = L.shade_lds != 0, gl = (FEAT & RTW_F_GEOM) != 0 && L.geom_lds != 0;
    if (sl && gl) {
        const rtw_launch G = stage_geom(stage_shade(L, wf_tail_nodes + n4), wf_tail_nodes + n4 + L.shade_lds / 16u);
        __syncthreads();
        wf_tail_body<FEAT, false, CN_F16_8, CNT, kPark>(G, W, it, nullptr, wf_tail_nodes, park);
        return;
    }
    if (sl) {
        const rtw_launch G = stage_shade(L, wf_tail_nodes + n4);
        __syncthreads();
        wf_tail_body<FEAT, false, CN_F16_8, CNT, kPark>(G, W, it, nullptr, wf_tail_nodes, park);
        return;
    }
    if constexpr ((FEAT & RTW_F_GEOM) != 0) {
        if (gl) {
            const rtw_launch G = stage_geom(L, wf_tail_nodes + n4);
            __syncthreads();
            wf_tail_body<FEAT, false, CN_F16_8, CNT, kPark>(G, W, it, nullptr, wf_tail_nodes, park);
            return;
        }
    }
    __syncthreads();
    wf_tail_body<FEAT, false, CN_F16_8, CNT, kPark>(L, W, it, nullptr, wf_tail_nodes, park);
}


template <uint32_t FEAT, int CN = CN_F16_8>
__global__ __launch_bounds__(1024) void wf_tail_clds(rtw_launch L, rtw_wf W, uint32_t it) {
    static_assert((FEAT & (RTW_F_GEOM | RTW_F_MEDIUM | RTW_F_MOVING)) == 0, "static sphere scenes");
    extern __shared__ uint4 wf_clds[];
    stage_clds(L, wf_clds);
    wf_tail_body<FEAT, true, CN>(L, W, it, wf_clds);
}
// the 4-copy stage (half the LDS) at two blocks of T threads per CU: 2T / 256 waves per SIMD
template <uint32_t FEAT, uint32_t T, int CNT = 2>
__global__ __launch_bounds__(T) __attribute__((amdgpu_waves_per_eu(2 * T / 256)))
void wf_tail_clds2(rtw_launch L, rtw_wf W, uint32_t it) {
    static_assert((FEAT & (RTW_F_GEOM | RTW_F_MEDIUM | RTW_F_MOVING)) == 0, "static sphere scenes");
    extern __shared__ uint4 wf_clds[];
    stage_clds(L, wf_clds);
    wf_tail_body<FEAT, true, CN_F16_4, CNT>(L, W, it, wf_clds);
}

// Where the fused step's walk reads the tree:
//   WALK_CLDS   the compact nodes of every octant copy staged in LDS (small static sphere SAH trees, C2)
//   WALK_LDS    the 32-B node array of one ordering staged in LDS (small object scenes: Cornell)
//   WALK_GLOBAL L.cnodes / L.nodes through L1/L2 (large trees: C4)
//   WALK_CLDS4  the compact nodes of the 4 (x, z)-sign copies staged in LDS (traverse_compact<.., Y4>)
//   WALK_CLDS32 the 32-B fp32-box nodes of the 4 copies staged in LDS (traverse_compact<.., Y4, F32>)
enum { WALK_CLDS = 0, WALK_LDS = 1, WALK_GLOBAL = 2, WALK_CLDS4 = 3, WALK_CLDS32 = 4 };
template <int WALK>
constexpr int walk_cn() { return WALK == WALK_CLDS32 ? CN_F32_4 : WALK == WALK_CLDS4 ? CN_F16_4 : CN_F16_8; }

template <uint32_t FEAT, int WALK, int CNT = 2>
__device__ __forceinline__ int wf_walk(const rtw_launch& L, const void* lds, const Ray& r, float& t, Counters& cnt,
                                       uint64_t mkey) {
    if constexpr (WALK == WALK_CLDS || WALK == WALK_CLDS4 || WALK == WALK_CLDS32) {
        const uint4* cn = static_cast<const uint4*>(lds);
        if constexpr (CNT != 2) return walk_compact<CNT == 1, true, walk_cn<WALK>()>(L, cn, r, t, cnt);
        return L.counters ? walk_compact<true, true, walk_cn<WALK>()>(L, cn, r, t, cnt)
                          : walk_compact<false, true, walk_cn<WALK>()>(L, cn, r, t, cnt);
    } else if constexpr (WALK == WALK_LDS) {
        return traverse<FEAT, false>(static_cast<const float4*>(lds), L, r, t, cnt, mkey);  // the LDS stage
    } else {
        return wf_traverse_global<FEAT>(L, r, t, cnt, mkey);
    }
}

// One fused wavefront iteration: iteration 0 generates the camera ray of path
// p = slot in registers (wf_camera), every iteration walks the tree (wf_trace) and
// shades (wf_shade) in the same kernel, appending the survivors to the next set.
// The ray never round-trips through HBM between trace and shade (no hit records:
// 48 B/ray less traffic, no gen pass), and the state streams of one wave overlap
// the walks of the others.  Same operations in the same order as
// gen/trace/shade: bit-identical.
// The stripe counters: this kernel appends to len[(it+1)%3] (zeroed by the
// previous iteration, or by the host for it = 0) and zeroes len[(it+2)%3],
// iteration it-1's input, for the next iteration.
// the fused step loads a path's throughput / id / RNG state after its walk (late_rest in wf_step_body): every
// scene class whose walk does not key media draws on the RNG state (object scenes: RTW_OBJ_LATE, an A/B switch)
#ifndef RTW_OBJ_LATE
#define RTW_OBJ_LATE 0
#endif
template <uint32_t FEAT>
constexpr bool wf_late_rest() {
    return (FEAT & RTW_F_MEDIUM) == 0 && ((FEAT & RTW_F_GEOM) == 0 || RTW_OBJ_LATE);
}

// IT0: 1 = the launch of iteration 0 (camera rays), 0 = a launch of iteration >= 1, 2 = either (runtime `it`)
template <uint32_t FEAT, int WALK, int CNT = 2, int IT0 = 2>
__device__ __forceinline__ void wf_step_body(const rtw_launch& L, const rtw_wf& W, uint32_t it, const void* lds) {
    if constexpr (IT0 == 1) it = 0;  // (the compiler then drops the other iterations' code)
    const bool first = IT0 == 2 ? it == 0 : IT0 == 1;
    const rtw_wf_set& S = W.set[it & 1u];
    const rtw_wf_set& O = W.set[(it + 1u) & 1u];
    Counters cnt;
    const bool bucketed = it < W.sort_iters;
    uint32_t bb = 0, bf = 64;  // lane b: bucket b's open block (wf_push_bucketed)
    for (WfIter e(W, it); e.more(); e.next()) {  // wave-uniform: the body starts converged
        bool live = false, push = false;
        uint32_t slot = 0, pid = 0, depth = 0;
        Ray r;
        r.o = r.d = mk(0, 0, 0);
        r.time = 0;
        rtw_rng rng;
        rng.s = 0;
        f3 thr = mk(1, 1, 1), acc = mk(0, 0, 0);
        const bool got = e.get(W, slot);
        if (first) {  // the camera ray in registers (wf_camera)
            pid = slot;
            live = wf_camera<FEAT>(L, W, got, slot, r, rng);
            if (got && !live) W.ls[slot] = rtw_rgb{0.0f, 0.0f, 0.0f};  // rayColor(r, 0) = 0
            depth = live ? L.max_depth : 0;
        } else if (got) {
            float2 txy;
            r = wf_load_ray_it<FEAT>(L, S, slot, it, depth, txy, true);
            live = depth != 0;
            if constexpr (!wf_late_rest<FEAT>()) {
                if (live) {  // media: the RNG state keys the ConstantMedium draws during the walk
                    uint64_t rs;
                    wf_load_rest<FEAT>(L, S, slot, depth, txy, thr, acc, rs, pid, true);
                    rng.s = rs;
                }
            }
        }
        // Sphere scenes load the rest of the path state (throughput, path id, RNG state) after the walk, not
        // before it: its six registers are not live across the walk, which took the fused step's spills from 156
        // to 140 B/lane at its 80-VGPR cap and C2 +3.5 % (two same-box rounds, profiles/r6_late_rest/); the
        // loads' latency is now exposed, but five other waves per SIMD cover it
        auto late_rest = [&]() {
            if constexpr (wf_late_rest<FEAT>()) {
                if (!first && live) {
                    float2 txy;
                    uint32_t d2;
                    (void)wf_load_ray_it<FEAT>(L, S, slot, it, d2, txy, true);
                    uint64_t rs;
                    wf_load_rest<FEAT>(L, S, slot, depth, txy, thr, acc, rs, pid, true);
                    rng.s = rs;
                }
            }
        };
        Ray sc;
        if constexpr ((FEAT & (RTW_F_GEOM | RTW_F_MEDIUM)) == 0) {
            // sphere scenes: the split form (C2 +6 %, C5 +3 % over the nested form of wf_shade)
            // The material kind, then the randomUnitVector draw of every lane that needs one (one rejection loop
            // for the wave), then the hit record and the material.  Building the hit record before the loop (the
            // form of rounds 2-5, C2 +6 % then over the nested form) kept its ~20 registers live across the loop:
            // at the 6-wave, 80-VGPR cap that spilled, and this order took the fused step's scratch from 124 to
            // 64 B/lane -- C2 +2.9 %, C5 +2.3 % (same box, profiles/r6_late_rest/).  The same draws in the same
            // order: bit-identical.
            HitPrep hp;
            bool hitp = false, need_uv = false;
            int hhit = -1;
            float ht = 0.0f;
            if (live) {
                float t;
                int hit = -1;
                bool listed = false;
                if constexpr (WALK != WALK_GLOBAL && (FEAT & (RTW_F_GEOM | RTW_F_MEDIUM | RTW_F_MOVING)) == 0) {
                    // camera rays: the tile's candidate list
                    if (first && W.tl_count) {
                        const uint32_t tile = (slot >> 6) / W.n_s;
                        if constexpr (CNT != 2) listed = wf_tile_hit<CNT == 1>(L, W, tile, r, hit, t, cnt);
                        else listed = L.counters ? wf_tile_hit<true>(L, W, tile, r, hit, t, cnt)
                                                 : wf_tile_hit<false>(L, W, tile, r, hit, t, cnt);
                    }
                }
                if (!listed) hit = wf_walk<FEAT, WALK, CNT>(L, lds, r, t, cnt, rng.s);
#if defined(RTW_ABLATE_WALK2)
                if (!listed) {  // timing ablation only: the walk twice (the second result is the same)
                    float t2;
                    if (wf_walk<FEAT, WALK>(L, lds, r, t2, cnt, rng.s) != hit) t = t2;
                }
#endif
#if defined(RTW_DIAG_WALK) && defined(__HIP_DEVICE_COMPILE__)
                if (!listed && it == rtw_diag_rec_it && rtw_diag_rec && slot < rtw_diag_rec_cap) {
                    rtw_diag_rec[2u * slot] = make_uint4(cnt.dsteps | (cnt.dleaves << 16), fbits(r.d.x), fbits(r.d.y),
                                                         fbits(r.d.z));
                    rtw_diag_rec[2u * slot + 1u] = make_uint4(fbits(r.o.x), fbits(r.o.y), fbits(r.o.z), pid + 1u);
                }
#endif
                if constexpr (CNT != 0) cnt.rays++;
                late_rest();
                if (hit < 0) {
                    acc = acc + thr * background(L, r);
                } else {
                    hhit = hit;
                    ht = t;
                    hitp = true;
                    need_uv = needs_unit_vector<FEAT>(hit_material_kind<FEAT>(L.nodes, L, hit));
                }
            }
            float uv3[3] = {0.0f, 0.0f, 0.0f};
            // the wave-cooperative loop (same candidates, same RNG states as seq_reject<3>): C2 +1.4 %, C5 +0.6 %
            if constexpr ((FEAT & (RTW_F_IMAGE | RTW_F_NOISE)) == 0 || RTW_COOP_TEXTURED) wf_reject3(need_uv, rng, uv3);
            else if (need_uv) seq_reject<3>(rng, uv3);
            if (hitp) hp = hit_prep<FEAT>(L.nodes, L, r, hhit, ht);
            if (hitp) {
                const f3 ruv = need_uv ? unit_vector(mk(uv3[0], uv3[1], uv3[2])) : mk(0, 0, 0);
                f3 att;
                if (scatter_finish<FEAT>(L, r, hp, ruv, rng, thr, acc, att, sc) && depth > 1) {
                    thr = thr * att;
                    push = true;
                }
            }
        } else {
            // object scenes: the walk, then the randomUnitVector draw of every lane whose material
            // starts with one (wf_reject3: the wave's lanes share the rejection loop; it only needs the
            // material kind, so no hit record is live across it), then the hit record and the material
            float t = 0.0f;
            int hit = -1;
            if (live) {
                hit = wf_walk<FEAT, WALK, CNT>(L, lds, r, t, cnt, rng.s);
#if defined(RTW_ABLATE_WALK2)
                {   // timing ablation only: the walk twice (the second result is the same)
                    float t2;
                    if (wf_walk<FEAT, WALK, CNT>(L, lds, r, t2, cnt, rng.s) != hit) t = t2;
                }
#endif
                if constexpr (CNT != 0) cnt.rays++;
                late_rest();
            }
            const bool need_uv = hit >= 0 && needs_unit_vector<FEAT>(hit_material_kind<FEAT>(L.nodes, L, hit));
            float uv3[3] = {0.0f, 0.0f, 0.0f};
            wf_reject3(need_uv, rng, uv3);
            if (live) {
                if (hit < 0) {
                    acc = acc + thr * background(L, r);
                } else {
                    const HitPrep hp = hit_prep<FEAT>(L.nodes, L, r, hit, t);
                    const f3 ruv = need_uv ? unit_vector(mk(uv3[0], uv3[1], uv3[2])) : mk(0, 0, 0);
                    f3 att;
                    if (scatter_finish<FEAT>(L, r, hp, ruv, rng, thr, acc, att, sc) && depth > 1) {
                        thr = thr * att;
                        push = true;
                    }
                }
            }
        }
        if (live && !push) W.ls[pid] = rtw_rgb{acc.x, acc.y, acc.z};
        const uint32_t out = bucketed ? wf_push_bucketed(W, it, push, push ? wf_bucket(sc.d) & W.sort_mask : 0u, bb, bf)
                                      : wf_push(W, it, push);
        if (push) wf_store_path<FEAT>(O, out, sc, depth - 1, thr, rng.s, pid, acc, true);
    }
    if (bucketed) wf_close_blocks<FEAT>(W, it, bb, bf, true);
    if constexpr (CNT != 0) flush_counters(L, cnt, 0);
}

__device__ __forceinline__ void wf_step_zero_next(const rtw_wf& W, uint32_t it) {
    if (blockIdx.x == 0 && threadIdx.x < RTW_WF_STRIPES) W.len[(it + 2u) % 3u][threadIdx.x * RTW_WF_LEN_STRIDE] = 0;
}

// compact nodes of every copy in LDS, then the materials when they fit
template <uint32_t FEAT, int WALK, int CNT = 2, int IT0 = 2>
__device__ __forceinline__ void wf_step_clds_body(const rtw_launch& L, const rtw_wf& W, uint32_t it) {
    wf_step_zero_next(W, it);
    extern __shared__ uint4 wf_clds[];
    stage_clds(L, wf_clds);
    if (L.mat_lds) {  // the materials after the nodes (the host checked that they fit)
        uint4* ml = wf_clds + L.n_nodes * L.n_orders * cn_quads(L);
        const uint4* src = reinterpret_cast<const uint4*>(L.mats);
        for (uint32_t k = threadIdx.x; k < L.mat_lds / 16u; k += blockDim.x) ml[k] = src[k];
        __syncthreads();
        rtw_launch Lm = L;
        Lm.mats = reinterpret_cast<const rtw_dev_material*>(ml);
        wf_step_body<FEAT, WALK, CNT, IT0>(Lm, W, it, wf_clds);
        return;
    }
    wf_step_body<FEAT, WALK, CNT, IT0>(L, W, it, wf_clds);
}

// one 1024-thread block per CU (the 8-copy stage, 124 KB for C2, allows no second block)
template <uint32_t FEAT, int CN = CN_F16_8>
__global__ __launch_bounds__(1024) void wf_step_clds(rtw_launch L, rtw_wf W, uint32_t it) {
    static_assert((FEAT & (RTW_F_GEOM | RTW_F_MEDIUM | RTW_F_MOVING)) == 0, "static sphere scenes");
    wf_step_clds_body<FEAT, CN == CN_F32_4 ? WALK_CLDS32 : CN == CN_F16_4 ? WALK_CLDS4 : WALK_CLDS>(L, W, it);
}

// The 4-copy stage (C2: 62 KB + 15.5 KB of materials) at two blocks of T = 768 threads per CU (rtw_tuning.clds_shape
// 4, the default): 6 waves per SIMD at <= 80 VGPRs (MI355X_MICROARCH.md: 80 allocated -> 6).  The fused step waits on
// its dependent ds_read_b128 41 % of the cycles at 4 waves (profiles/r4_stall/): the fifth and sixth waves have
// ready work to issue in those waits.  (Two blocks of 512 or 640 threads lost their A/Bs -- profiles/r5_occupancy/,
// diag/walk_variants.patch -- and were removed in round 6.)
// Iteration 0 (camera rays: wf_camera, the tile lists) and the later iterations (late_rest) of the fused steps in
// separate instantiations, so that neither pays for the other's registers: C2's step scratch 64 -> 44 / 28 B,
// C2 +1.8 % (same box, profiles/r6_waves/i/; C5, Cornell, smoke +-0.6 %).  0 = one instantiation (A/B).
#ifndef RTW_STEP_IT0
#define RTW_STEP_IT0 1
#endif
template <uint32_t FEAT, uint32_t T, int CNT = 2, int IT0 = 2>
__global__ __launch_bounds__(T) __attribute__((amdgpu_waves_per_eu(2 * T / 256)))
void wf_step_clds2(rtw_launch L, rtw_wf W, uint32_t it) {
    static_assert((FEAT & (RTW_F_GEOM | RTW_F_MEDIUM | RTW_F_MOVING)) == 0, "static sphere scenes");
    wf_step_clds_body<FEAT, WALK_CLDS4, CNT, IT0>(L, W, it);
}

// wf_step's LDS extras by mask (bit 0 Perlin tables, 1 materials/textures, 2 geometry); masks a
// scene class cannot use compile to nothing
template <uint32_t FEAT, uint32_t MASK, int CNT, int IT0>
__device__ __forceinline__ void wf_step_staged(const rtw_launch& L, const rtw_wf& W, uint32_t it, float4* nodes,
                                               float4* extra) {
    constexpr bool P = (MASK & 1u) && (FEAT & RTW_F_NOISE), S = (MASK & 2u) != 0, G = (MASK & 4u) && (FEAT & RTW_F_GEOM);
    if constexpr (P || S || G) {
        rtw_launch Lp = L;
        if constexpr (P) {  // noise gathers from LDS
            const uint32_t np4 = L.n_perlin * (RTW_PERLIN_BYTES / 16u);
            for (uint32_t k = threadIdx.x; k < np4; k += 256u) extra[k] = L.perlin[k];
            Lp.perlin = extra;
            extra += np4;
        }
        if constexpr (S) {
            Lp = stage_shade(Lp, extra);
            extra += L.shade_lds / 16u;
        }
        if constexpr (G) Lp = stage_geom(Lp, extra);
        __syncthreads();
        wf_step_body<FEAT, WALK_LDS, CNT, IT0>(Lp, W, it, nodes);
    }
}

// the 32-B node array (one ordering) in LDS, or the tree through L1/L2
template <uint32_t FEAT, bool LDS, int CNT = 2, int IT0 = 2>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(RTW_WPE_STEP))) void wf_step(rtw_launch L, rtw_wf W, uint32_t it) {
    wf_step_zero_next(W, it);
    extern __shared__ float4 wf_lds_nodes[];
    const uint32_t n4 = LDS ? 2u * L.n_nodes * L.n_orders : 0u;
    if constexpr (LDS) {
        for (uint32_t k = threadIdx.x; k < n4; k += 256u) wf_lds_nodes[k] = L.nodes[k];
        // after the nodes: Perlin tables, materials, geometry -- one call per staging mask, so
        // every pointer the body reads is statically LDS or global (no flat loads)
        const uint32_t mask = (((FEAT & RTW_F_NOISE) && L.perlin_lds) ? 1u : 0u) | (L.shade_lds ? 2u : 0u) |
                              (((FEAT & RTW_F_GEOM) && L.geom_lds) ? 4u : 0u);
        float4* extra = wf_lds_nodes + n4;
        switch (mask) {
            case 1: return wf_step_staged<FEAT, 1, CNT, IT0>(L, W, it, wf_lds_nodes, extra);
            case 2: return wf_step_staged<FEAT, 2, CNT, IT0>(L, W, it, wf_lds_nodes, extra);
            case 3: return wf_step_staged<FEAT, 3, CNT, IT0>(L, W, it, wf_lds_nodes, extra);
            case 4: return wf_step_staged<FEAT, 4, CNT, IT0>(L, W, it, wf_lds_nodes, extra);
            case 5: return wf_step_staged<FEAT, 5, CNT, IT0>(L, W, it, wf_lds_nodes, extra);
            case 6: return wf_step_staged<FEAT, 6, CNT, IT0>(L, W, it, wf_lds_nodes, extra);
            case 7: return wf_step_staged<FEAT, 7, CNT, IT0>(L, W, it, wf_lds_nodes, extra);
            default: break;
        }
        __syncthreads();
        wf_step_body<FEAT, WALK_LDS, CNT, IT0>(L, W, it, wf_lds_nodes);
    } else {
        wf_step_body<FEAT, WALK_GLOBAL, CNT, IT0>(L, W, it, nullptr);
    }
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
            // the samples' radiances in groups of R loads issued together, then added in sample order (the same
            // sums): one memory latency per group instead of per sample -- a shard of a multi-GPU render has too
            // few pixels (waves) per SIMD to hide a latency per sample (C2 at 8 ranks: 2.2x the N = 1 time / 8)
            constexpr uint32_t R = 8;
            const rtw_rgb* __restrict__ ls = W.ls + (((size_t)(q >> 6) * W.n_s) << 6) + (q & 63u);  // wf_path
            uint32_t s = 0;
            for (; s + R <= W.n_s; s += R) {
                rtw_rgb c[R];
#pragma unroll
                for (uint32_t k = 0; k < R; k++) c[k] = ls[(size_t)(s + k) << 6];
#pragma unroll
                for (uint32_t k = 0; k < R; k++) {
                    if (is_nan3(mk(c[k].x, c[k].y, c[k].z))) cnt.nans++;
                    a.x += c[k].x;
                    a.y += c[k].y;
                    a.z += c[k].z;
                }
            }
            for (; s < W.n_s; s++) {
                const rtw_rgb c = ls[(size_t)s << 6];
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

// resident blocks of `kernel`, rounded down to whole stripes of waves
template <typename K>
uint32_t wf_grid(K kernel, int n_cu, size_t lds = 0, uint32_t threads = 256) {
    int b = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, kernel, (int)threads, lds) != hipSuccess || b < 1) b = 1;
    uint32_t g = (uint32_t)(b * n_cu);
    // whole sets of stripes: the grid's waves a multiple of RTW_WF_STRIPES (every stripe the same number of
    // waves, WfIter), i.e. blocks a multiple of 256 / gcd(256, waves per block)
    uint32_t wpb = threads / 64, gcd = RTW_WF_STRIPES;
    for (uint32_t a = wpb; a;) {
        const uint32_t t = gcd % a;
        gcd = a;
        a = t;
    }
    const uint32_t per = RTW_WF_STRIPES / gcd;
    g -= g % per;
    return g ? g : per;
}

// grid-cache key of a launch shape on a device of n_cu CUs (never 0: an empty cache misses).  Every cache is
// per host thread and keyed by the CU count too: a grid larger than the device's would overflow the stripes
// that rtw_wavefront_max_waves(n_cu) sized.
inline uint64_t wf_key(int n_cu, uint64_t shape) { return ((uint64_t)(uint32_t)n_cu << 40) | (shape + 1u); }

// the same, cached per host thread for one dynamic LDS size (c = {grid, key})
template <typename K>
uint32_t wf_grid_cached(K kernel, int n_cu, size_t lds, uint64_t (&c)[2]) {
    if (c[1] != wf_key(n_cu, lds)) {
        c[0] = wf_grid(kernel, n_cu, lds);
        c[1] = wf_key(n_cu, lds);
    }
    return (uint32_t)c[0];
}

// the global tail launch of either form
template <uint32_t FEAT>
void wf_launch_tail(const rtw_launch& L, const rtw_wf& W, hipStream_t st, int n_cu, size_t lds, uint64_t (&cache)[2],
                    uint32_t it) {
    if constexpr ((FEAT & ~RTW_F_CHECKER) == 0)
        { if (L.counters) hipLaunchKernelGGL((wf_tail_w5<FEAT, 1>), dim3(wf_grid_cached(wf_tail_w5<FEAT, 0>, n_cu, lds, cache)), dim3(256),
                                        lds, st, L, W, it); else hipLaunchKernelGGL((wf_tail_w5<FEAT, 0>), dim3(wf_grid_cached(wf_tail_w5<FEAT, 0>, n_cu, lds, cache)), dim3(256),
                                        lds, st, L, W, it); }
    else
        hipLaunchKernelGGL(wf_tail<FEAT>, dim3(wf_grid_cached(wf_tail<FEAT>, n_cu, lds, cache)), dim3(256), lds, st, L,
                           W, it);
}

// dynamic LDS of the kernels that walk through L1/L2: the two-wide walk's per-lane stacks
template <uint32_t FEAT>
size_t wf_w2_lds(const rtw_launch& L) {
    if constexpr ((FEAT & (RTW_F_GEOM | RTW_F_MEDIUM | RTW_F_MOVING)) == 0) {
        if (L.w2nodes && L.fast_box) return (size_t)256u * 4u * L.w2_stack;
    }
    return 0;
}

// The camera-ray candidate lists of a batch (static sphere scenes with the compact nodes): the
// flat scan for small trees, the frustum walk for large ones.  Returns W with tl_count null when off.
template <uint32_t FEAT>
rtw_wf wf_lists(const rtw_launch& L, const rtw_wf& W, hipStream_t st) {
    rtw_wf Wt = W;
    if (!W.tl_count || !L.cnodes || (FEAT & (RTW_F_GEOM | RTW_F_MEDIUM | RTW_F_MOVING)) || L.max_depth == 0) {
        Wt.tl_count = nullptr;
        return Wt;
    }
    const uint32_t tiles = W.n_pix / 64u;
    if (L.n_nodes <= 4096u)
        hipLaunchKernelGGL(wf_tile_lists, dim3(tiles), dim3(64), 0, st, L, Wt);
    else
        hipLaunchKernelGGL(wf_tile_lists_walk, dim3((tiles + 63u) / 64u), dim3(64), 0, st, L, Wt);
    return Wt;
}

// Coherent-queue settings of a launch whose grid has nw waves.  Iteration 0 deals runs of
// up to 16 samples per tile, shorter when a wave would get fewer than 64 runs (a small batch: whole runs
// would leave the waves' shares of work uneven); direction bucketing only when a wave's iteration 0 has at
// least RTW_WF_SORT_MIN_CHUNKS chunks -- each open block ends its iteration partly dead, which only a large
// share of survivors per wave amortises (simple_light, 137 chunks per wave: -10 % with bucketing).  Deal bit 128
// (RTW_DEAL_SMALL_SORT) lifts that gate, so the tests run the bucketed queues of the large benched batches on small
// images (tests/test_gpu_parity.py, test_gpu_objects.py).
#define RTW_WF_SORT_MIN_CHUNKS 192u
rtw_wf wf_coherence(const rtw_wf& W, uint32_t nw, uint32_t sort_iters) {
    rtw_wf C = W;
    const uint32_t per_wave = nw ? (W.n_paths >> 6) / nw : 0u;
    uint32_t lg = 0;
    while (lg < 4 && (per_wave >> (lg + 1)) >= 64u) lg++;
    // the dynamic deal only where the waves have enough work to share: a small batch (simple_light, 137 chunks per
    // wave) ran 6 % slower with it -- its tail's claims cost more than they balance (profiles/r5_deal/)
    if (per_wave < RTW_WF_SORT_MIN_CHUNKS && !(C.deal_mode & 8u)) C.deal = nullptr;  // (bit 8: tests force it)
    if (C.deal && (C.deal_mode & 1u)) lg = 4;  // dynamic deal: the waves balance themselves, runs keep 16 samples
    C.run_log2 = lg;
    C.sort_iters = (per_wave >= RTW_WF_SORT_MIN_CHUNKS || (C.deal_mode & 128u)) ? sort_iters : 0u;
    return C;
}

template <uint32_t FEAT>
struct WfGrids {
    uint32_t shade = 0, shade0 = 0;  // shade0: iteration 0's instantiation (wf_camera)
    WfGrids() = default;
    explicit WfGrids(int n_cu)
        : shade(wf_grid(wf_shade<FEAT>, n_cu)), shade0(wf_grid(wf_shade<FEAT, true>, n_cu)) {}
};

// largest LDS stage of the wavefront trace (bytes); larger trees read L1/L2
#define RTW_WF_LDS_MAX (64u * 1024u)
#define RTW_WF_CLDS_MAX (150u * 1024u)  // compact-node LDS stage (one 1024-thread block per CU)

template <uint32_t FEAT, bool CAM>
uint32_t wf_lds_grid(int n_cu, size_t lds) {
    thread_local uint32_t cache[(RTW_WF_LDS_MAX + 16384) / 512 + 1] = {0};  // + geometry (L.geom_lds)
    thread_local int cache_cu = 0;
    if (cache_cu != n_cu) {
        for (uint32_t& c : cache) c = 0;
        cache_cu = n_cu;
    }
    uint32_t& g = cache[lds / 512];
    if (!g) g = wf_grid(wf_trace<FEAT, true, CAM>, n_cu, lds);
    return g;
}

// per CU count (a process may render on devices or partitions of different sizes), process-wide: the 8
// Tasks of a render (main.zig:314-326) share one set instead of each thread querying the occupancy API again
template <uint32_t FEAT>
WfGrids<FEAT> wf_grids(int n_cu) {
    static std::mutex mu;
    static std::map<int, WfGrids<FEAT>> cache;
    std::lock_guard<std::mutex> lk(mu);
    auto it = cache.find(n_cu);
    if (it == cache.end()) it = cache.emplace(n_cu, WfGrids<FEAT>(n_cu)).first;
    return it->second;
}

// (Grid sizes are cached per host thread: rtw_render may be called from several threads at once.)
// Fused path (L.wf_fuse & 1): one wf_step* kernel per iteration, then the tail
// (on the compact LDS stage when L.wf_fuse & 2) and the reduce.
//   clds > 0: compact nodes of all orders in LDS (wf_step_clds, 1024 threads)
//   lds  > 0: the 32-B node array in LDS (wf_step<FEAT, true>)
//   else    : the tree through L1/L2 (wf_step<FEAT, false>)
// dynamic LDS of the fused kernels: tree stage + what is staged after it

// scene classes whose fused step never runs on the compact LDS stage (wf_run: textured scenes keep the 32-B
// stage), so wf_run_fused instantiates no compact-LDS kernel for them
#define RTW_WF_NO_CLDS (RTW_F_GEOM | RTW_F_MEDIUM | RTW_F_MOVING | RTW_F_IMAGE | RTW_F_NOISE)
template <uint32_t FEAT>
void wf_run_fused(const rtw_launch& L, const rtw_wf& W0, hipStream_t st, int n_cu, size_t clds, size_t lds,
                  rtw_timer* T) {
    const size_t cdyn0 = clds,
                 cdyn = cdyn0 + L.mat_lds <= 160u * 1024u ? cdyn0 + L.mat_lds : cdyn0,
                 ldyn = lds + (L.perlin_lds ? (size_t)L.n_perlin * RTW_PERLIN_BYTES : 0) +
                        ((FEAT & RTW_F_GEOM) ? L.geom_lds : 0u) + L.shade_lds,
                 tdyn = lds + ((FEAT & RTW_F_GEOM) ? L.geom_lds : 0u) + L.shade_lds,
                 gdyn = wf_w2_lds<FEAT>(L);
    thread_local uint64_t cgrid[2] = {0, 0}, tgrid[2] = {0, 0}, lgrid[2] = {0, 0}, ggrid[2] = {0, 0}, wtail[2] = {0, 0};
    uint32_t grid = 0;
    // The compact stage's block shape: the 8-copy stage (C2: 124 KB) leaves room for one 1024-thread block
    // per CU; the 4-copy stage (L.n_orders == 4, 62 KB) for two 768-thread blocks (rtw_tuning.clds_shape 4)
    // when it fits half the LDS
    const bool y4 = L.n_orders == 4;
    const int cn = L.cnode32 ? CN_F32_4 : y4 ? CN_F16_4 : CN_F16_8;
    const uint32_t shape = clds && cn == CN_F16_4 && cdyn0 <= RTW_WF_CLDS2_MAX && L.clds_shape == 4u ? 4u : 1u;
    const bool two = shape == 4u;
    const size_t cdyn2 = two && cdyn > RTW_WF_CLDS2_MAX ? cdyn0 : cdyn;  // materials only if they fit too
    const uint32_t cthreads = two ? 768u : 1024u;
    if constexpr ((FEAT & RTW_WF_NO_CLDS) == 0) {
        const uint64_t key = wf_key(n_cu, (uint32_t)cdyn2 | (shape << 24) | ((uint32_t)cn << 28));
        if (clds && cgrid[1] != key) {
            if (two) {
                cgrid[0] = wf_grid(wf_step_clds2<FEAT, 768, 0>, n_cu, cdyn2, 768);
                tgrid[0] = wf_grid(wf_tail_clds2<FEAT, 768, 0>, n_cu, clds, 768);
            } else if (cn == CN_F32_4) {
                cgrid[0] = wf_grid(wf_step_clds<FEAT, CN_F32_4>, n_cu, cdyn2, 1024);
                tgrid[0] = wf_grid(wf_tail_clds<FEAT, CN_F32_4>, n_cu, clds, 1024);
            } else if (cn == CN_F16_4) {
                cgrid[0] = wf_grid(wf_step_clds<FEAT, CN_F16_4>, n_cu, cdyn2, 1024);
                tgrid[0] = wf_grid(wf_tail_clds<FEAT, CN_F16_4>, n_cu, clds, 1024);
            } else {
                cgrid[0] = wf_grid(wf_step_clds<FEAT, CN_F16_8>, n_cu, cdyn2, 1024);
                tgrid[0] = wf_grid(wf_tail_clds<FEAT, CN_F16_8>, n_cu, clds, 1024);
            }
            cgrid[1] = tgrid[1] = key;
        }
    }
    if (clds) {
        grid = (uint32_t)cgrid[0];
    } else if (lds) {
        if (lgrid[1] != wf_key(n_cu, ldyn)) {
            lgrid[0] = wf_grid(wf_step<FEAT, true, 0>, n_cu, ldyn);
            lgrid[1] = wf_key(n_cu, ldyn);
        }
        grid = (uint32_t)lgrid[0];
    } else {
        grid = wf_grid_cached(wf_step<FEAT, false, 0>, n_cu, gdyn, ggrid);
    }
    // iteration 0 appends to len[1]; every later iteration's output counters are
    // zeroed by the kernel two iterations before (wf_step_zero_next)
    (void)hipMemsetAsync(W0.len[1], 0, RTW_WF_STRIPES * RTW_WF_LEN_STRIDE * 4, st);
    if (W0.deal) (void)hipMemsetAsync(W0.deal, 0, RTW_WF_DEAL_COUNTERS * 4, st);
    rtw_wf W = wf_coherence(W0, grid * (clds ? cthreads / 64u : 4u), W0.sort_iters);
    W.packed = wf_packed<FEAT>() ? 1u : 0u;  // the fused step and its tail: always the packed state
    const uint32_t iters = L.max_depth < W.iters ? L.max_depth : W.iters;
    rtw_wf Wt = W;  // the camera-ray lists serve the LDS-staged steps of static sphere scenes
    if ((clds || lds) && iters) Wt = wf_lists<FEAT>(L, W, st);
    else Wt.tl_count = nullptr;
    // rayColor(depth <= 0) = 0 (camera.zig:183-185): no iteration writes W.ls, which holds the
    // previous render's radiance, so the reduce must add zeros
    if (iters == 0) (void)hipMemsetAsync(W.ls, 0, (size_t)W.n_paths * sizeof(rtw_rgb), st);
    for (uint32_t it = 0; it < iters; it++) {
        RTW_TIME_BEGIN(T, RTW_K_TRACE)
        Wt.deal = W.deal;  // (only iteration 0 deals from it: counters 0 .. 511)
        // deal bit 16: iteration it >= 1 claims its stripes' chunks from counters of its own
        Wt.deal_it = (W.deal && (W.deal_mode & 16u) && it) ? W.deal + RTW_WF_DEAL_COUNTERS0 + it * RTW_WF_STRIPES
                                                           : nullptr;
        if constexpr ((FEAT & RTW_WF_NO_CLDS) == 0) {
            if (clds) {
                rtw_launch Lc = L;  // the materials are staged only when they fit
                if (cdyn2 == cdyn0) Lc.mat_lds = 0;
                if (two)
                    {
                        if (L.counters) hipLaunchKernelGGL((wf_step_clds2<FEAT, 768, 1>), dim3(grid), dim3(768), cdyn2, st, Lc, Wt, it);
                        else if (RTW_STEP_IT0 && it == 0) hipLaunchKernelGGL((wf_step_clds2<FEAT, 768, 0, RTW_STEP_IT0 ? 1 : 2>), dim3(grid), dim3(768), cdyn2, st, Lc, Wt, it);
                        else if (RTW_STEP_IT0) hipLaunchKernelGGL((wf_step_clds2<FEAT, 768, 0, RTW_STEP_IT0 ? 0 : 2>), dim3(grid), dim3(768), cdyn2, st, Lc, Wt, it);
                        else hipLaunchKernelGGL((wf_step_clds2<FEAT, 768, 0>), dim3(grid), dim3(768), cdyn2, st, Lc, Wt, it);
                    }
                else if (cn == CN_F32_4)
                    hipLaunchKernelGGL((wf_step_clds<FEAT, CN_F32_4>), dim3(grid), dim3(1024), cdyn2, st, Lc, Wt, it);
                else if (cn == CN_F16_4)
                    hipLaunchKernelGGL((wf_step_clds<FEAT, CN_F16_4>), dim3(grid), dim3(1024), cdyn2, st, Lc, Wt, it);
                else
                    hipLaunchKernelGGL((wf_step_clds<FEAT, CN_F16_8>), dim3(grid), dim3(1024), cdyn2, st, Lc, Wt, it);
                RTW_TIME_END(T)
                continue;
            }
        }
        if (lds)
            {
                if (L.counters) hipLaunchKernelGGL((wf_step<FEAT, true, 1>), dim3(grid), dim3(256), ldyn, st, L, Wt, it);
                else if (RTW_STEP_IT0 && it == 0) hipLaunchKernelGGL((wf_step<FEAT, true, 0, RTW_STEP_IT0 ? 1 : 2>), dim3(grid), dim3(256), ldyn, st, L, Wt, it);
                else if (RTW_STEP_IT0) hipLaunchKernelGGL((wf_step<FEAT, true, 0, RTW_STEP_IT0 ? 0 : 2>), dim3(grid), dim3(256), ldyn, st, L, Wt, it);
                else hipLaunchKernelGGL((wf_step<FEAT, true, 0>), dim3(grid), dim3(256), ldyn, st, L, Wt, it);
            }
        else
            { if (L.counters) hipLaunchKernelGGL((wf_step<FEAT, false, 1>), dim3(grid), dim3(256), gdyn, st, L, W, it); else hipLaunchKernelGGL((wf_step<FEAT, false, 0>), dim3(grid), dim3(256), gdyn, st, L, W, it); }
        RTW_TIME_END(T)
    }
    if (iters < L.max_depth) {
        RTW_TIME_BEGIN(T, RTW_K_TAIL)
        // one tail launch over iteration itx's queue (W's counters: the launch's own)
        auto tail = [&](const rtw_wf& Wd, uint32_t itx) {
            if constexpr ((FEAT & RTW_WF_NO_CLDS) == 0) {
                if (clds && (L.wf_fuse & 2u)) {
                    const rtw_wf& W = Wd;
                    if (two)
                        { if (L.counters) hipLaunchKernelGGL((wf_tail_clds2<FEAT, 768, 1>), dim3((uint32_t)tgrid[0]), dim3(768), clds, st, L, W, itx); else hipLaunchKernelGGL((wf_tail_clds2<FEAT, 768, 0>), dim3((uint32_t)tgrid[0]), dim3(768), clds, st, L, W, itx); }
                    else if (cn == CN_F32_4)
                        hipLaunchKernelGGL((wf_tail_clds<FEAT, CN_F32_4>), dim3((uint32_t)tgrid[0]), dim3(1024), clds, st, L, W, itx);
                    else if (cn == CN_F16_4)
                        hipLaunchKernelGGL((wf_tail_clds<FEAT, CN_F16_4>), dim3((uint32_t)tgrid[0]), dim3(1024), clds, st, L, W, itx);
                    else
                        hipLaunchKernelGGL((wf_tail_clds<FEAT, CN_F16_8>), dim3((uint32_t)tgrid[0]), dim3(1024), clds, st, L, W, itx);
                    return;
                }
            }
            if (lds && (L.wf_fuse & 2u)) {  // the node array in LDS for the tail too
                thread_local uint64_t tl[2] = {0, 0};
                if (tl[1] != wf_key(n_cu, tdyn)) {
                    tl[0] = wf_grid(wf_tail_lds<FEAT, 0>, n_cu, tdyn);
                    tl[1] = wf_key(n_cu, tdyn);
                }
                { if (L.counters) hipLaunchKernelGGL((wf_tail_lds<FEAT, 1>), dim3((uint32_t)tl[0]), dim3(256), tdyn, st, L, Wd, itx); else hipLaunchKernelGGL((wf_tail_lds<FEAT, 0>), dim3((uint32_t)tl[0]), dim3(256), tdyn, st, L, Wd, itx); }
                return;
            }
            wf_launch_tail<FEAT>(L, Wd, st, n_cu, gdyn, wtail, itx);
        };
        rtw_wf Wd = W;  // the tail's input claims: counter 512 (iteration 0 took 0 .. 511)
        if (W.deal) Wd.deal = W.deal + RTW_WF_DEAL_LAUNCH;
        tail(Wd, iters);
        RTW_TIME_END(T)
    }
    RTW_TIME_BEGIN(T, RTW_K_REDUCE)
    hipLaunchKernelGGL(wf_reduce, dim3((W.n_pix + 255u) / 256u), dim3(256), 0, st, L, W);
    RTW_TIME_END(T)
}

template <uint32_t FEAT>
void wf_run(const rtw_launch& L, const rtw_wf& W0, hipStream_t st, int n_cu, rtw_timer* T) {
    const WfGrids<FEAT> g = wf_grids<FEAT>(n_cu);
    if (L.wf_fuse & 1u) {
        size_t fclds = 0, flds = 0;
        // (textured scenes keep the 32-B node stage: it leaves LDS for the Perlin tables and the
        // 1024-thread compact kernel would spill at its 128-VGPR cap -- C5 -20 % measured)
        if constexpr ((FEAT & (RTW_F_GEOM | RTW_F_MEDIUM | RTW_F_MOVING | RTW_F_IMAGE | RTW_F_NOISE)) == 0) {
            const size_t c = (size_t)L.n_nodes * L.n_orders * (L.cnode32 ? 32u : 16u);
            if (L.cnodes && L.fast_box && L.wf_clds && c <= RTW_WF_CLDS_MAX) fclds = c;
        }
        const size_t need = (size_t)L.n_nodes * L.n_orders * 32u;
        if (!fclds && L.wf_lds && need <= RTW_WF_LDS_MAX) flds = (need + 511u) / 512u * 512u;
        // measured: fused wins on C2 (+8.5 %), C5 (+24 %), Cornell (+2 %) and, since the
        // round-3 queues and object trees, Cornell smoke (media: +23 %); through L1/L2 (C4, RTW_WF_FUSE
        // bit 2) it loses (-13 %)
        if ((fclds || flds) || (L.wf_fuse & 4u)) {
            wf_run_fused<FEAT>(L, W0, st, n_cu, fclds, flds, T);
            return;
        }
    }
    rtw_wf W = wf_coherence(W0, g.shade * 4u, W0.sort_iters_split);  // the split kernels' queues
    W.packed = wf_packed<FEAT>() ? 1u : 0u;  // the split kernels (and their tail) use the packed state too
    const rtw_wf W1 = W;
    // dynamic deal: iteration 0's trace deals from counters 0 .. 511, its shade from 512 .. 1023
    if (W0.deal) (void)hipMemsetAsync(W0.deal, 0, RTW_WF_DEAL_COUNTERS * 4, st);
    const uint32_t iters = L.max_depth < W.iters ? L.max_depth : W.iters;
    // iteration 0's trace and shade generate the camera rays themselves (wf_camera); with no
    // iteration (max_depth 0) nothing writes W.ls and the reduce must add zeros
    if (iters == 0) (void)hipMemsetAsync(W.ls, 0, (size_t)W.n_paths * sizeof(rtw_rgb), st);
    const rtw_wf Wt = iters ? wf_lists<FEAT>(L, W, st) : W;  // camera rays: iteration 0 of wf_trace (L1/L2)
    rtw_wf Ws0 = W;  // iteration 0's shade: its own counters
    if (W.deal) Ws0.deal = W.deal + RTW_WF_DEAL_LAUNCH;
    const size_t w2l = wf_w2_lds<FEAT>(L);  // the two-wide walk's stacks (trace / tail through L1/L2)
    thread_local uint64_t wtrace[2] = {0, 0}, wtrace0[2] = {0, 0}, wtail[2] = {0, 0};
    const size_t lds_need = (size_t)L.n_nodes * L.n_orders * 32u;
    const size_t lds = (L.wf_lds && lds_need <= RTW_WF_LDS_MAX)
                           ? (lds_need + 511u) / 512u * 512u : 0;
    const size_t tlds = lds ? lds + ((FEAT & RTW_F_GEOM) ? L.geom_lds : 0u) : 0;  // + quads/members/instances
    const uint32_t lds_grid = lds ? wf_lds_grid<FEAT, false>(n_cu, tlds) : 0,
                   lds_grid0 = lds ? wf_lds_grid<FEAT, true>(n_cu, tlds) : 0;
    // compact nodes of every octant copy in LDS (small static sphere trees)
    const size_t clds = (L.cnodes && L.fast_box && L.wf_clds)
                            ? (size_t)L.n_nodes * L.n_orders * (L.cnode32 ? 32u : 16u) : 0;
    thread_local uint64_t clds_grid_cache[3] = {0, 0, 0};
    uint32_t clds_grid = 0, clds_grid0 = 0;
    constexpr uint32_t clds_threads = 1024;  // one block per CU shares the stage (256 / 512: slower)
    if constexpr ((FEAT & (RTW_F_GEOM | RTW_F_MEDIUM | RTW_F_MOVING)) == 0) {
        if (clds && clds <= RTW_WF_CLDS_MAX) {
            if (clds_grid_cache[1] != wf_key(n_cu, clds)) {  // (the Y4 forms: the same registers)
                clds_grid_cache[0] = wf_grid(wf_trace_clds<FEAT>, n_cu, clds, clds_threads);
                clds_grid_cache[2] = wf_grid(wf_trace_clds<FEAT, true>, n_cu, clds, clds_threads);
                clds_grid_cache[1] = wf_key(n_cu, clds);
            }
            clds_grid = (uint32_t)clds_grid_cache[0];
            clds_grid0 = (uint32_t)clds_grid_cache[2];
        }
    }
    for (uint32_t it = 0; it < iters; it++) {
        RTW_TIME_BEGIN(T, RTW_K_TRACE)
        // deal bit 16: iteration it >= 1's trace and shade claim their stripes' chunks from counters of their own
        rtw_wf W = W1;
        rtw_wf Ws = W1;
        if (W1.deal && (W1.deal_mode & 16u) && it) {
            W.deal_it = W1.deal + RTW_WF_DEAL_COUNTERS0 + it * RTW_WF_STRIPES;
            Ws.deal_it = W1.deal + RTW_WF_DEAL_SHADE + it * RTW_WF_STRIPES;
        }
        if constexpr ((FEAT & (RTW_F_GEOM | RTW_F_MEDIUM | RTW_F_MOVING)) == 0) {
            if (clds_grid) {
                const int cn = L.cnode32 ? CN_F32_4 : L.n_orders == 4 ? CN_F16_4 : CN_F16_8;
                const dim3 g(it == 0 ? clds_grid0 : clds_grid), b(clds_threads);
                if (it == 0 && cn == CN_F32_4) hipLaunchKernelGGL((wf_trace_clds<FEAT, true, CN_F32_4>), g, b, clds, st, L, W, it);
                else if (it == 0 && cn == CN_F16_4) hipLaunchKernelGGL((wf_trace_clds<FEAT, true, CN_F16_4>), g, b, clds, st, L, W, it);
                else if (it == 0) hipLaunchKernelGGL((wf_trace_clds<FEAT, true, CN_F16_8>), g, b, clds, st, L, W, it);
                else if (cn == CN_F32_4) hipLaunchKernelGGL((wf_trace_clds<FEAT, false, CN_F32_4>), g, b, clds, st, L, W, it);
                else if (cn == CN_F16_4) hipLaunchKernelGGL((wf_trace_clds<FEAT, false, CN_F16_4>), g, b, clds, st, L, W, it);
                else hipLaunchKernelGGL((wf_trace_clds<FEAT, false, CN_F16_8>), g, b, clds, st, L, W, it);
                RTW_TIME_END(T)
                goto shade_step;
            }
        }
        if (lds && it == 0)
            hipLaunchKernelGGL((wf_trace<FEAT, true, true>), dim3(lds_grid0), dim3(256), tlds, st, L, W, it);
        else if (lds)
            hipLaunchKernelGGL((wf_trace<FEAT, true>), dim3(lds_grid), dim3(256), tlds, st, L, W, it);
        else if (it == 0)
            hipLaunchKernelGGL((wf_trace<FEAT, false, true>),
                               dim3(wf_grid_cached(wf_trace<FEAT, false, true>, n_cu, w2l, wtrace0)), dim3(256), w2l, st,
                               L, Wt, it);
        else
            hipLaunchKernelGGL((wf_trace<FEAT, false>), dim3(wf_grid_cached(wf_trace<FEAT, false>, n_cu, w2l, wtrace)),
                               dim3(256), w2l, st, L, W, it);
        RTW_TIME_END(T)
    shade_step:
        RTW_TIME_BEGIN(T, RTW_K_SHADE)
        if (it == 0)
            hipLaunchKernelGGL((wf_shade<FEAT, true>), dim3(g.shade0), dim3(256), (FEAT & RTW_F_GEOM) ? L.geom_lds : 0u,
                               st, L, Ws0, it);
        else
            hipLaunchKernelGGL(wf_shade<FEAT>, dim3(g.shade), dim3(256), (FEAT & RTW_F_GEOM) ? L.geom_lds : 0u, st, L,
                               Ws, it);
        RTW_TIME_END(T)
    }
    if (iters < L.max_depth) {
        RTW_TIME_BEGIN(T, RTW_K_TAIL)
        rtw_wf Wd = W;  // the tail's input claims: counter 1024 (iteration 0's trace and shade took 0 .. 1023)
        if (W.deal) Wd.deal = W.deal + 2 * RTW_WF_DEAL_LAUNCH;
        auto tail = [&](const rtw_wf& Wx, uint32_t itx) {
            if (lds && (L.wf_fuse & 2u)) {  // the node array (+ geometry) in LDS for the tail (smoke +5 %)
                thread_local uint64_t tl[2] = {0, 0};
                const size_t tdyn = tlds + L.shade_lds;  // wf_tail_lds stages the materials too
                if (tl[1] != wf_key(n_cu, tdyn)) {
                    tl[0] = wf_grid(wf_tail_lds<FEAT, 0>, n_cu, tdyn);
                    tl[1] = wf_key(n_cu, tdyn);
                }
                { if (L.counters) hipLaunchKernelGGL((wf_tail_lds<FEAT, 1>), dim3((uint32_t)tl[0]), dim3(256), tdyn, st, L, Wx, itx); else hipLaunchKernelGGL((wf_tail_lds<FEAT, 0>), dim3((uint32_t)tl[0]), dim3(256), tdyn, st, L, Wx, itx); }
            } else {
                wf_launch_tail<FEAT>(L, Wx, st, n_cu, w2l, wtail, itx);
            }
        };
        tail(Wd, iters);
        RTW_TIME_END(T)
    }
    RTW_TIME_BEGIN(T, RTW_K_REDUCE)
    hipLaunchKernelGGL(wf_reduce, dim3((W.n_pix + 255u) / 256u), dim3(256), 0, st, L, W);
    RTW_TIME_END(T)
}

// Object scenes without media, image / noise textures or motion (quads, instances, lights,
// solid / checker textures: the Cornell box, HEAD's default scene) get their own
// instantiation: without the unused code paths the fused step needs fewer registers.
// Likewise static, unlit sphere scenes with image / noise textures (BASELINE config 5) and
// object scenes with media but no image / noise textures or motion (Cornell smoke).
#define RTW_F_OBJECTS (RTW_F_GEOM | RTW_F_LIGHT | RTW_F_CHECKER)
#define RTW_F_TEXTURED (RTW_F_CHECKER | RTW_F_IMAGE | RTW_F_NOISE)
#define RTW_F_MEDIA (RTW_F_GEOM | RTW_F_MEDIUM | RTW_F_LIGHT | RTW_F_CHECKER)
uint32_t wf_pick_feat(uint32_t f) {
    if ((f & ~RTW_F_CHECKER) == 0) return f ? RTW_F_CHECKER : 0u;
    if ((f & RTW_F_GEOM) && (f & ~RTW_F_OBJECTS) == 0) return RTW_F_OBJECTS;
    if ((f & ~RTW_F_TEXTURED) == 0) return RTW_F_TEXTURED;
    if ((f & RTW_F_MEDIUM) && (f & ~RTW_F_MEDIA) == 0) return RTW_F_MEDIA;
    return (f & (RTW_F_GEOM | RTW_F_MEDIUM)) ? RTW_F_ALL : RTW_F_SPHERES;
}

}  // namespace

#if !defined(RTW_WF_SPHERES_TU)
// untextured static sphere scenes (FEAT 0 / CHECKER: BASELINE C2, C3, C4) run from rtw_wavefront_spheres.hip,
// this code compiled with 64-B loop alignment (csrc/Makefile): C2 +0.8 %, C3 +0.7 %; the other scene classes
// gained nothing from the flag (C5 -0.3 %, Cornell -0.4 %), so they keep the default placement
void rtw_wf_run_spheres(const rtw_launch& L, const rtw_wf& W, hipStream_t st, int n_cu, rtw_timer* T, uint32_t feat);
uint32_t rtw_wf_spheres_max_waves(int n_cu);

void rtw_wavefront_batch(const rtw_launch& L, const rtw_wf& W, void* stream, int n_cu, rtw_timer* T) {
    hipStream_t st = (hipStream_t)stream;
    switch (wf_pick_feat(L.feat)) {
    case 0u: rtw_wf_run_spheres(L, W, st, n_cu, T, 0u); break;
    case RTW_F_CHECKER: rtw_wf_run_spheres(L, W, st, n_cu, T, RTW_F_CHECKER); break;
    case RTW_F_SPHERES: wf_run<RTW_F_SPHERES>(L, W, st, n_cu, T); break;
    case RTW_F_OBJECTS: wf_run<RTW_F_OBJECTS>(L, W, st, n_cu, T); break;
    case RTW_F_TEXTURED: wf_run<RTW_F_TEXTURED>(L, W, st, n_cu, T); break;
    case RTW_F_MEDIA: wf_run<RTW_F_MEDIA>(L, W, st, n_cu, T); break;
    default: wf_run<RTW_F_ALL>(L, W, st, n_cu, T); break;
    }
}

uint32_t rtw_wavefront_max_waves(int n_cu) {
    uint32_t m = 0;
    auto mx = [&m](uint32_t a, uint32_t b) { m = std::max({m, a, b}); };
    mx(wf_grids<RTW_F_SPHERES>(n_cu).shade, wf_grids<RTW_F_SPHERES>(n_cu).shade0);
    mx(wf_grids<RTW_F_OBJECTS>(n_cu).shade, wf_grids<RTW_F_OBJECTS>(n_cu).shade0);
    mx(wf_grids<RTW_F_TEXTURED>(n_cu).shade, wf_grids<RTW_F_TEXTURED>(n_cu).shade0);
    mx(wf_grids<RTW_F_MEDIA>(n_cu).shade, wf_grids<RTW_F_MEDIA>(n_cu).shade0);
    mx(wf_grids<RTW_F_ALL>(n_cu).shade, wf_grids<RTW_F_ALL>(n_cu).shade0);
    return std::max(4 * m, rtw_wf_spheres_max_waves(n_cu));
}
#else
void rtw_wf_run_spheres(const rtw_launch& L, const rtw_wf& W, hipStream_t st, int n_cu, rtw_timer* T, uint32_t feat) {
    if (feat) wf_run<RTW_F_CHECKER>(L, W, st, n_cu, T);
    else wf_run<0u>(L, W, st, n_cu, T);
}

// (waves: the 256-thread shade grids and the compact-LDS kernels' grids, whichever launches more; computed per
// CU count -- it sizes the stripes, which the kernels do not bound-check)
uint32_t rtw_wf_spheres_max_waves(int n_cu) {
    static std::mutex mu;
    static std::map<int, uint32_t> cache;
    std::lock_guard<std::mutex> lk(mu);
    if (auto it = cache.find(n_cu); it != cache.end()) return it->second;
    const uint32_t b = std::max({wf_grids<0u>(n_cu).shade, wf_grids<0u>(n_cu).shade0, wf_grids<RTW_F_CHECKER>(n_cu).shade,
                                 wf_grids<RTW_F_CHECKER>(n_cu).shade0});
    const uint32_t c2 = std::max(wf_grid(wf_step_clds2<0u, 768, 0>, n_cu, 0, 768), wf_grid(wf_step_clds2<RTW_F_CHECKER, 768, 0>, n_cu, 0, 768)) * 12u;
    const uint32_t c1 = std::max(wf_grid(wf_step_clds<0u>, n_cu, 0, 1024), wf_grid(wf_step_clds<RTW_F_CHECKER>, n_cu, 0, 1024)) * 16u;
    const uint32_t val = std::max({4u * b, c2, c1});
    cache[n_cu] = val;
    return val;
}

#if defined(RTW_DIAG_WALK)  // (the sphere-scene kernels' records and counters: this translation unit's)
// diagnostic build only: where the per-slot walk records of iteration `it` go (null: off)
extern "C" int rtw_debug_walk_records(void* d_rec, uint32_t cap_slots, uint32_t it) {
    uint4* p = static_cast<uint4*>(d_rec);
    if (hipMemcpyToSymbol(HIP_SYMBOL(rtw_diag_rec), &p, sizeof p) != hipSuccess) return RTW_E_HIP;
    if (hipMemcpyToSymbol(HIP_SYMBOL(rtw_diag_rec_cap), &cap_slots, 4) != hipSuccess) return RTW_E_HIP;
    if (hipMemcpyToSymbol(HIP_SYMBOL(rtw_diag_rec_it), &it, 4) != hipSuccess) return RTW_E_HIP;
    return RTW_OK;
}
// diagnostic build only: the compact walk's step counters (rtw_device.h WalkDiag), read and optionally reset
extern "C" int rtw_debug_walk_counters(uint64_t* out, int reset) {
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(rtw_diag_walk), 16 * sizeof(uint64_t)) != hipSuccess) return RTW_E_HIP;
    if (reset) {
        const uint64_t z[16] = {0};
        if (hipMemcpyToSymbol(HIP_SYMBOL(rtw_diag_walk), z, sizeof z) != hipSuccess) return RTW_E_HIP;
    }
    return RTW_OK;
}
#endif
#endif  // RTW_WF_SPHERES_TU
