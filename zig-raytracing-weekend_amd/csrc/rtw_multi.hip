// rtw_multi.hip -- one process driving N devices (include/rtw_gpu.h rtw_multi_*):
// row-interleaved shard renders (rtw_render_rows_device) + grouped RCCL
// send/recv of the compact tiles to device 0.
//
// Replaces startRender's split of one frame over 8 RenderThreads
// (src/main.zig:314-326, each running Camera.render, src/camera.zig:93-116).
// Shard k of N owns the row blocks b = k, k + N, ... (rows_per_block rows each);
// its tile row r is image row ((r / rpb) * N + k) * rpb + r % rpb (map_row in
// rtw_device.h).  Every tile is cap = ceil(blocks / N) * rpb rows (the unused
// tail of a short shard is never read back), so device 0 holds the N tiles in one
// stacked buffer and moves them with one ncclSend / ncclRecv pair per device in
// one group -- the only data-path exchange of the algorithm.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/rtw_gpu.h"
#include "rtw_internal.h"

struct rtw_multi {
    std::vector<rtw_ctx*> ctx;
    std::vector<int> dev;
    std::vector<ncclComm_t> comm;
    std::vector<float4*> tile;     // per device: cap * W float4
    size_t tile_elems = 0;         // float4 per tile (allocated)
    float4* stacked = nullptr;     // device 0: N tiles
    float4* frame = nullptr;       // device 0: host-API staging of the frame
    size_t frame_elems = 0;
    hipEvent_t ev_in = nullptr, ev_out = nullptr;
    std::mutex mu;
};

namespace {

int mfail(int code, const std::string& msg) {
    rtw_set_error(msg.c_str());  // rtw_last_error()
    return code;
}

#define MHIP(expr)                                                                           \
    do {                                                                                     \
        hipError_t _e = (expr);                                                              \
        if (_e != hipSuccess)                                                                \
            return mfail(_e == hipErrorOutOfMemory ? RTW_E_OOM : RTW_E_HIP,                  \
                         std::string(#expr) + ": " + hipGetErrorString(_e));                 \
    } while (0)
#define MNCCL(expr)                                                                          \
    do {                                                                                     \
        ncclResult_t _r = (expr);                                                            \
        if (_r != ncclSuccess) return mfail(RTW_E_HIP, std::string(#expr) + ": " + ncclGetErrorString(_r)); \
    } while (0)

// The calls of one RCCL group: the first failure is kept and the group is always closed (an open
// group would defer every later RCCL call of this thread).
struct NcclGroup {
    ncclResult_t first = ncclSuccess;
    const char* what = "";
    void add(ncclResult_t r, const char* w) {
        if (first == ncclSuccess && r != ncclSuccess) {
            first = r;
            what = w;
        }
    }
    bool ok() const { return first == ncclSuccess; }
    int end() {
        const ncclResult_t e = ncclGroupEnd();
        if (first != ncclSuccess) return mfail(RTW_E_HIP, std::string(what) + ": " + ncclGetErrorString(first));
        if (e != ncclSuccess) return mfail(RTW_E_HIP, std::string("ncclGroupEnd: ") + ncclGetErrorString(e));
        return RTW_OK;
    }
};

// dir 0: frame rows -> stacked tiles (pack); dir 1: stacked tiles -> frame rows (unpack).
// One thread per float4; x fastest, so both sides are contiguous runs of W.
__global__ __launch_bounds__(256) void shard_rows_copy(float4* __restrict__ frame, float4* __restrict__ stacked,
                                                       uint32_t W, uint32_t H, uint32_t rpb, uint32_t n,
                                                       uint32_t cap, uint32_t dir) {
    const uint64_t i = (uint64_t)blockIdx.x * 256u + threadIdx.x;
    const uint64_t per = (uint64_t)cap * W;
    if (i >= per * n) return;
    const uint32_t k = (uint32_t)(i / per);
    const uint32_t rem = (uint32_t)(i - (uint64_t)k * per);
    const uint32_t r = rem / W, x = rem - r * W;
    const uint32_t y = rtw_shard_row(H, rpb, n, k, r);
    if (y >= H) return;
    float4* f = frame + (size_t)y * W + x;
    if (dir == 0) stacked[i] = *f;
    else *f = stacked[i];
}

int ensure_buffers(rtw_multi* m, size_t tile_elems, size_t frame_elems) {
    const uint32_t n = (uint32_t)m->ctx.size();
    if (m->tile_elems < tile_elems) {
        for (uint32_t k = 0; k < n; k++) {
            MHIP(hipSetDevice(m->dev[k]));
            MHIP(hipStreamSynchronize(m->ctx[k]->stream));
            if (m->tile[k]) (void)hipFree(m->tile[k]);
            m->tile[k] = nullptr;
        }
        MHIP(hipSetDevice(m->dev[0]));
        if (m->stacked) (void)hipFree(m->stacked);
        m->stacked = nullptr;
        m->tile_elems = 0;
        for (uint32_t k = 0; k < n; k++) {
            MHIP(hipSetDevice(m->dev[k]));
            MHIP(hipMalloc(&m->tile[k], tile_elems * sizeof(float4)));
        }
        MHIP(hipSetDevice(m->dev[0]));
        MHIP(hipMalloc(&m->stacked, tile_elems * n * sizeof(float4)));
        m->tile_elems = tile_elems;
    }
    if (frame_elems && m->frame_elems < frame_elems) {
        MHIP(hipSetDevice(m->dev[0]));
        MHIP(hipStreamSynchronize(m->ctx[0]->stream));
        if (m->frame) (void)hipFree(m->frame);
        m->frame = nullptr;
        m->frame_elems = 0;
        MHIP(hipMalloc(&m->frame, frame_elems * sizeof(float4)));
        m->frame_elems = frame_elems;
    }
    return RTW_OK;
}

// The device-side frame render; the caller holds m->mu.  Streams: every device's work
// runs on its context's own stream; `stream` (device 0) is joined in and out by events.
// Samples in batches of spp_batch (0: one batch unless the caller polls); when ctl polls, every
// device finishes batch b before progress and the stop flags are read, and a stop ends the loop
// after the last finished batch -- the gather below then brings the finished batches to the frame.
int multi_render(rtw_multi* m, const rtw_camera* cam, uint32_t rpb, uint32_t s0, uint32_t s1, uint64_t seed,
                 float4* frame, hipStream_t stream, uint32_t spp_batch, uint32_t flags, const rtw_render_opts* ctl) {
    const uint32_t n = (uint32_t)m->ctx.size();
    const uint32_t W = cam->image_width, H = cam->image_height;
    const uint32_t cap = rtw_shard_capacity(H, rpb, n);
    const size_t per = (size_t)cap * W;
    if (rtw_stop_requested(ctl)) return mfail(RTW_E_CANCELLED, "cancelled");  // nothing touched
    if (int rc = ensure_buffers(m, per, 0)) return rc;
    hipStream_t s_root = m->ctx[0]->stream;
    MHIP(hipSetDevice(m->dev[0]));
    if (stream && stream != s_root) {  // the caller's prior work on its stream (e.g. zero fills) first
        MHIP(hipEventRecord(m->ev_in, stream));
        MHIP(hipStreamWaitEvent(s_root, m->ev_in, 0));
    }
    const uint64_t total = (uint64_t)per * n;
    const uint32_t blocks = (uint32_t)((total + 255) / 256);
    const size_t count = per * 4;  // floats per tile
    if (flags & RTW_RENDER_FRESH) {
        for (uint32_t k = 0; k < n; k++) {
            MHIP(hipSetDevice(m->dev[k]));
            MHIP(hipMemsetAsync(m->tile[k], 0, per * sizeof(float4), m->ctx[k]->stream));
        }
    } else {  // the frame's current rows to their shards: pack on device 0, then one grouped send/recv
        MHIP(hipSetDevice(m->dev[0]));
        hipLaunchKernelGGL(shard_rows_copy, dim3(blocks), dim3(256), 0, s_root, frame, m->stacked, W, H, rpb, n,
                           cap, 0u);
        MHIP(hipGetLastError());
        MNCCL(ncclGroupStart());
        NcclGroup g;
        for (uint32_t k = 0; k < n && g.ok(); k++) {
            g.add(ncclSend(m->stacked + k * per, count, ncclFloat32, (int)k, m->comm[0], s_root), "ncclSend");
            if (g.ok()) g.add(ncclRecv(m->tile[k], count, ncclFloat32, 0, m->comm[k], m->ctx[k]->stream), "ncclRecv");
        }
        if (int rc = g.end()) return rc;
    }
    const bool polled = rtw_polled(ctl);
    const uint64_t pixels = (uint64_t)W * H;
    uint32_t batch = spp_batch ? spp_batch : s1 - s0;
    if (!spp_batch && polled) {  // the single-context auto batch of the largest shard
        const uint64_t target = m->ctx[0]->variant == 2 ? m->ctx[0]->wf_max_paths : (64ull << 20);
        const uint64_t b = target / std::max<uint64_t>(1, per);
        batch = (uint32_t)std::min<uint64_t>(std::max<uint64_t>(b, 1), s1 - s0);
    }
    int stop = RTW_OK;
    rtw_render_opts o{};
    o.flags = RTW_RENDER_NO_SYNC;
    for (uint32_t b0 = s0; b0 < s1 && stop == RTW_OK; b0 += batch) {
        const uint32_t b1 = (s1 - b0 < batch) ? s1 : b0 + batch;
        o.spp_batch = b1 - b0;
        for (uint32_t k = 0; k < n; k++) {  // enqueue only: the N devices render concurrently
            const int rc = rtw_render_rows_device(m->ctx[k], cam, rpb, n, k, b0, b1, seed,
                                                  reinterpret_cast<float*>(m->tile[k]), nullptr, &o);
            if (rc) return mfail(rc, std::string("shard render: ") + rtw_last_error());
        }
        if (polled) {
            for (uint32_t k = 0; k < n; k++) {
                MHIP(hipSetDevice(m->dev[k]));
                MHIP(hipStreamSynchronize(m->ctx[k]->stream));
            }
            if (ctl->progress && ctl->progress(pixels * (uint64_t)(b1 - s0), pixels * (uint64_t)(s1 - s0), ctl->user))
                stop = mfail(RTW_E_CANCELLED, "cancelled by progress callback");
            else if (b1 < s1 && rtw_stop_requested(ctl))
                stop = mfail(RTW_E_CANCELLED, "cancelled");
        }
    }
    MNCCL(ncclGroupStart());  // the tiles to device 0 (the gather)
    NcclGroup g;
    for (uint32_t k = 0; k < n && g.ok(); k++) {
        g.add(ncclSend(m->tile[k], count, ncclFloat32, 0, m->comm[k], m->ctx[k]->stream), "ncclSend");
        if (g.ok()) g.add(ncclRecv(m->stacked + k * per, count, ncclFloat32, (int)k, m->comm[0], s_root), "ncclRecv");
    }
    if (int rc = g.end()) return rc;
    MHIP(hipSetDevice(m->dev[0]));
    hipLaunchKernelGGL(shard_rows_copy, dim3(blocks), dim3(256), 0, s_root, frame, m->stacked, W, H, rpb, n, cap,
                       1u);
    MHIP(hipGetLastError());
    if (stream && stream != s_root) {
        MHIP(hipEventRecord(m->ev_out, s_root));
        MHIP(hipStreamWaitEvent(stream, m->ev_out, 0));
    }
    return stop;
}

int check_args(rtw_multi* m, const rtw_camera* cam, uint32_t rpb, uint32_t s0, uint32_t s1) {
    if (!m) return mfail(RTW_E_INVALID, "null rtw_multi");
    if (!cam || cam->image_width == 0 || cam->image_height == 0) return mfail(RTW_E_INVALID, "camera not initialised");
    if ((uint64_t)cam->image_width * cam->image_height > 0xFFFFFFFFull) return mfail(RTW_E_INVALID, "image too large");
    if ((rpb & ~RTW_ROWS_FLAGS) == 0) return mfail(RTW_E_INVALID, "rows_per_block == 0");
    if (s0 > s1) return mfail(RTW_E_INVALID, "bad sample range");
    return RTW_OK;
}

}  // namespace

extern "C" {

int rtw_multi_create(rtw_ctx* const* ctxs, uint32_t n, rtw_multi** out) {
    if (!out) return mfail(RTW_E_INVALID, "null out");
    *out = nullptr;
    if (!ctxs || n == 0) return mfail(RTW_E_INVALID, "no contexts");
    rtw_multi* m = new rtw_multi();
    for (uint32_t k = 0; k < n; k++) {
        if (!ctxs[k] || ctxs[k]->device == RTW_DEVICE_CPU) {
            delete m;
            return mfail(RTW_E_INVALID, "null or host context");
        }
        for (uint32_t j = 0; j < k; j++)
            if (ctxs[j]->device == ctxs[k]->device) {
                delete m;
                return mfail(RTW_E_INVALID, "two contexts on one device (one context per device)");
            }
        m->ctx.push_back(ctxs[k]);
        m->dev.push_back(ctxs[k]->device);
    }
    m->comm.assign(n, nullptr);
    m->tile.assign(n, nullptr);
    const ncclResult_t r = ncclCommInitAll(m->comm.data(), (int)n, m->dev.data());
    if (r != ncclSuccess) {
        delete m;
        return mfail(RTW_E_HIP, std::string("ncclCommInitAll: ") + ncclGetErrorString(r));
    }
    hipError_t e = hipSetDevice(m->dev[0]);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&m->ev_in, hipEventDisableTiming);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&m->ev_out, hipEventDisableTiming);
    if (e != hipSuccess) {
        rtw_multi_destroy(m);
        return mfail(RTW_E_HIP, std::string("rtw_multi_create: ") + hipGetErrorString(e));
    }
    *out = m;
    return RTW_OK;
}

void rtw_multi_destroy(rtw_multi* m) {
    if (!m) return;
    for (size_t k = 0; k < m->ctx.size(); k++) {
        (void)hipSetDevice(m->dev[k]);
        (void)hipStreamSynchronize(m->ctx[k]->stream);
        if (m->tile[k]) (void)hipFree(m->tile[k]);
        if (m->comm[k]) (void)ncclCommDestroy(m->comm[k]);
    }
    if (!m->dev.empty()) (void)hipSetDevice(m->dev[0]);
    if (m->stacked) (void)hipFree(m->stacked);
    if (m->frame) (void)hipFree(m->frame);
    if (m->ev_in) (void)hipEventDestroy(m->ev_in);
    if (m->ev_out) (void)hipEventDestroy(m->ev_out);
    delete m;
}

int rtw_render_multi_device(rtw_multi* m, const rtw_camera* cam, uint32_t rpb, uint32_t s0, uint32_t s1,
                            uint64_t seed, float* d_accum, void* stream, const rtw_render_opts* opts) {
    if (int rc = check_args(m, cam, rpb, s0, s1)) return rc;
    if (!d_accum) return mfail(RTW_E_INVALID, "null accum");
    if (opts && (opts->counters || opts->timing)) return mfail(RTW_E_INVALID, "counters/timing are per context");
    if (s0 == s1) return RTW_OK;
    std::lock_guard<std::mutex> lock(m->mu);
    const uint32_t flags = opts ? opts->flags : 0u;
    int rc = multi_render(m, cam, rpb, s0, s1, seed, reinterpret_cast<float4*>(d_accum), (hipStream_t)stream,
                          opts ? opts->spp_batch : 0u, flags, opts);
    if (rc && rc != RTW_E_CANCELLED) return rc;
    if (!(flags & RTW_RENDER_NO_SYNC)) {
        MHIP(hipSetDevice(m->dev[0]));
        MHIP(hipStreamSynchronize(stream ? (hipStream_t)stream : m->ctx[0]->stream));
    }
    return rc;
}

int rtw_render_multi_ex(rtw_multi* m, const rtw_camera* cam, uint32_t rpb, uint32_t s0, uint32_t s1, uint64_t seed,
                        float* accum, const rtw_render_opts* opts) {
    if (int rc = check_args(m, cam, rpb, s0, s1)) return rc;
    if (!accum) return mfail(RTW_E_INVALID, "null accum");
    if (opts && (opts->flags || opts->counters || opts->timing))
        return mfail(RTW_E_INVALID, "host-buffer render: flags, counters and timing must be 0/NULL");
    if (s0 == s1) return RTW_OK;
    if (rtw_stop_requested(opts)) return mfail(RTW_E_CANCELLED, "cancelled");
    std::lock_guard<std::mutex> lock(m->mu);
    const size_t px = (size_t)cam->image_width * cam->image_height;
    if (int rc = ensure_buffers(m, 0, px)) return rc;
    hipStream_t s = m->ctx[0]->stream;
    MHIP(hipSetDevice(m->dev[0]));
    MHIP(hipMemcpyAsync(m->frame, accum, px * sizeof(float4), hipMemcpyHostToDevice, s));
    const int rc = multi_render(m, cam, rpb, s0, s1, seed, m->frame, nullptr, opts ? opts->spp_batch : 0u, 0u, opts);
    if (rc && rc != RTW_E_CANCELLED) return rc;
    MHIP(hipSetDevice(m->dev[0]));
    MHIP(hipMemcpyAsync(accum, m->frame, px * sizeof(float4), hipMemcpyDeviceToHost, s));
    MHIP(hipStreamSynchronize(s));
    return rc;  // RTW_E_CANCELLED: accum holds the finished batches
}

int rtw_render_multi(rtw_multi* m, const rtw_camera* cam, uint32_t rpb, uint32_t s0, uint32_t s1, uint64_t seed,
                     float* accum, const volatile int32_t* cancel) {
    rtw_render_opts o{};
    o.cancel = cancel;
    return rtw_render_multi_ex(m, cam, rpb, s0, s1, seed, accum, &o);
}

int rtw_multi_info(rtw_multi* m, uint32_t* n_devices, int* rccl_ranks) {
    if (!m) return mfail(RTW_E_INVALID, "null rtw_multi");
    if (n_devices) *n_devices = (uint32_t)m->ctx.size();
    if (rccl_ranks) {
        int c = 0;
        MNCCL(ncclCommCount(m->comm[0], &c));
        *rccl_ranks = c;
    }
    return RTW_OK;
}

}  // extern "C"
