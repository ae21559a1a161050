// rtw_output.hip -- output formats and checkpoints over the float4 accumulator
// (SURVEY §8f rows 3-4).  Output:
// the two P3 PPM writers of the reference (color.zig:64-69 writeColor,
// stdout.zig:5-18 printPpmToStdout), an RGBA8 PNG encoder for the
// SharedStateImageWriter texture (the reference's "save to file" TODO,
// main.zig:47), and the texel update of camera.zig:58-65 as a device kernel.
// Progress/resume: countSamples (main.zig:470-477) and a CRC-checked checkpoint
// file of the accumulator + the camera, seed, scene hash and samples done.
#include <hip/hip_runtime.h>
#include <unistd.h>

#include <cmath>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/rtw_gpu.h"

#pragma STDC FP_CONTRACT OFF

namespace {

// color.zig:21-41 toGamma: c / n, sqrt, clamp to [0, 0.999] (interval.zig:16-20)
inline void to_gamma(const float* px, float g[3]) {
    const float scale = 1.0f / px[3];
    for (int k = 0; k < 3; k++) {
        float x = std::sqrt(px[k] * scale);
        if (x < 0.0f) x = 0.0f;
        if (x > 0.999f) x = 0.999f;
        g[k] = x;
    }
}

// Zig's "{d}" of a whole-valued f32 in [0, 256]; "nan" for NaN
inline int put_value(char* dst, float v) {
    if (!(v == v)) {
        std::memcpy(dst, "nan", 3);
        return 3;
    }
    return std::snprintf(dst, 8, "%d", (int)v);
}

uint32_t crc_table[256];
void crc_fill() {
    for (uint32_t n = 0; n < 256; n++) {
        uint32_t c = n;
        for (int k = 0; k < 8; k++) c = (c & 1) ? 0xEDB88320u ^ (c >> 1) : c >> 1;
        crc_table[n] = c;
    }
}
void crc_init() {
    static const bool once = (crc_fill(), true);  // thread-safe one-time init
    (void)once;
}
uint32_t crc32(const uint8_t* p, size_t n, uint32_t c = 0xFFFFFFFFu) {
    for (size_t i = 0; i < n; i++) c = crc_table[(c ^ p[i]) & 0xFF] ^ (c >> 8);
    return c;
}

struct Sink {
    uint8_t* out;
    size_t cap, n = 0;
    void put(const void* src, size_t k) {
        if (out && n + k <= cap) std::memcpy(out + n, src, k);
        n += k;
    }
    void be32(uint32_t v) {
        const uint8_t b[4] = {(uint8_t)(v >> 24), (uint8_t)(v >> 16), (uint8_t)(v >> 8), (uint8_t)v};
        put(b, 4);
    }
};

__global__ void texels_kernel(const float4* __restrict__ acc, uint32_t n, uchar4* __restrict__ out) {
    const uint32_t i = blockIdx.x * 256u + threadIdx.x;
    if (i >= n) return;
    const float4 c = acc[i];
    const float scale = 1.0f / c.w;
    const float v[3] = {c.x, c.y, c.z};
    uint8_t b[3];
    for (int k = 0; k < 3; k++) {
        float x = __builtin_sqrtf(v[k] * scale);
        if (x < 0.0f) x = 0.0f;
        if (x > 0.999f) x = 0.999f;
        b[k] = (x == x) ? (uint8_t)(256 * x) : 0;  // NaN (UB in the reference): 0
    }
    out[i] = make_uchar4(b[0], b[1], b[2], 255);
}

}  // namespace

extern "C" {

int rtw_texture_from_accum_device(const float* d_accum, uint32_t n, uint8_t* d_rgba, void* stream) {
    if (!d_accum || !d_rgba) return RTW_E_INVALID;
    if (n == 0) return RTW_OK;
    hipLaunchKernelGGL(texels_kernel, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)stream,
                       reinterpret_cast<const float4*>(d_accum), n, reinterpret_cast<uchar4*>(d_rgba));
    return hipGetLastError() == hipSuccess ? RTW_OK : RTW_E_HIP;
}

int rtw_encode_ppm(const float* accum, uint32_t width, uint32_t height, uint32_t style, char* out, size_t cap,
                   size_t* len) {
    if (!accum || !len || style > RTW_PPM_STDOUT) return RTW_E_INVALID;
    Sink s{reinterpret_cast<uint8_t*>(out), out ? cap : 0};
    char line[64];
    int k = std::snprintf(line, sizeof line, "P3\n%u %u\n255\n", width, height);
    s.put(line, (size_t)k);
    const char sep = style == RTW_PPM_WRITECOLOR ? '\n' : '\t';
    for (uint64_t i = 0; i < (uint64_t)width * height; i++) {
        float g[3];
        to_gamma(accum + 4 * i, g);
        int p = 0;
        for (int c = 0; c < 3; c++) {
            const float v = style == RTW_PPM_WRITECOLOR ? std::round(256 * g[c])      // color.zig:68
                                                        : std::floor(g[c] * 255.999f);  // stdout.zig:15
            p += put_value(line + p, v);
            line[p++] = c < 2 ? ' ' : sep;
        }
        s.put(line, (size_t)p);
    }
    *len = s.n;
    if (out && s.n > cap) return RTW_E_INVALID;
    return RTW_OK;
}

float rtw_count_samples(const float* accum, uint64_t n) {
    float samples = 0;  // main.zig:471-476: f32, index order
    if (!accum) return 0;
    for (uint64_t i = 0; i < n; i++) samples += accum[4 * i + 3];
    return samples;
}

int rtw_checkpoint_write(const char* path, const rtw_camera* cam, uint64_t seed, uint64_t scene_hash,
                         uint32_t spp_done, const float* accum) {
    if (!path || !cam || !accum) return RTW_E_INVALID;
    crc_init();
    // write path.tmp, flush it to disk, then rename it over path: a crash mid-write (the case
    // resume exists for) leaves the previous checkpoint intact
    const std::string tmp_path = std::string(path) + ".tmp";
    FILE* f = std::fopen(tmp_path.c_str(), "wb");
    if (!f) return RTW_E_INVALID;
    uint32_t crc = 0xFFFFFFFFu;
    bool ok = true;
    auto put = [&](const void* p, size_t n) {
        crc = crc32(static_cast<const uint8_t*>(p), n, crc);
        ok = ok && std::fwrite(p, 1, n, f) == n;
    };
    const uint32_t version = 1;
    const uint64_t n_pix = cam->size;
    put("RTWCKPT1", 8);
    put(&version, 4);
    put(&spp_done, 4);
    put(&seed, 8);
    put(&scene_hash, 8);
    put(cam, sizeof *cam);
    put(&n_pix, 8);
    put(accum, n_pix * 16);
    const uint32_t c = crc ^ 0xFFFFFFFFu;
    ok = ok && std::fwrite(&c, 1, 4, f) == 4;
    ok = ok && std::fflush(f) == 0 && ::fsync(::fileno(f)) == 0;
    ok = (std::fclose(f) == 0) && ok;
    ok = ok && std::rename(tmp_path.c_str(), path) == 0;
    if (!ok) std::remove(tmp_path.c_str());
    return ok ? RTW_OK : RTW_E_INVALID;
}

int rtw_checkpoint_read(const char* path, rtw_camera* cam, uint64_t* seed, uint64_t* scene_hash,
                        uint32_t* spp_done, float* accum, uint64_t cap_pixels) {
    if (!path) return RTW_E_INVALID;
    crc_init();
    FILE* f = std::fopen(path, "rb");
    if (!f) return RTW_E_INVALID;
    uint32_t crc = 0xFFFFFFFFu;
    bool ok = true;
    auto get = [&](void* p, size_t n) {
        ok = ok && std::fread(p, 1, n, f) == n;
        if (ok) crc = crc32(static_cast<const uint8_t*>(p), n, crc);
    };
    char magic[8];
    uint32_t version = 0, done = 0;
    uint64_t sd = 0, hash = 0, n_pix = 0;
    rtw_camera c{};
    get(magic, 8);
    get(&version, 4);
    get(&done, 4);
    get(&sd, 8);
    get(&hash, 8);
    get(&c, sizeof c);
    get(&n_pix, 8);
    ok = ok && std::memcmp(magic, "RTWCKPT1", 8) == 0 && version == 1 && n_pix == c.size &&
         (!accum || n_pix == cap_pixels);
    std::vector<float> tmp;
    if (ok) {
        tmp.resize(n_pix * 4);
        get(tmp.data(), n_pix * 16);
    }
    uint32_t stored = 0;
    ok = ok && std::fread(&stored, 1, 4, f) == 4 && stored == (crc ^ 0xFFFFFFFFu);
    std::fclose(f);
    if (!ok) return RTW_E_INVALID;
    if (cam) *cam = c;
    if (seed) *seed = sd;
    if (scene_hash) *scene_hash = hash;
    if (spp_done) *spp_done = done;
    if (accum) std::memcpy(accum, tmp.data(), n_pix * 16);
    return RTW_OK;
}

int rtw_encode_png(const uint8_t* rgba, uint32_t width, uint32_t height, uint8_t* out, size_t cap, size_t* len) {
    if (!rgba || !len || width == 0 || height == 0) return RTW_E_INVALID;
    crc_init();
    Sink s{out, out ? cap : 0};
    static const uint8_t sig[8] = {0x89, 'P', 'N', 'G', '\r', '\n', 0x1A, '\n'};
    s.put(sig, 8);
    auto chunk = [&](const char* type, const std::string& data) {
        s.be32((uint32_t)data.size());
        s.put(type, 4);
        s.put(data.data(), data.size());
        uint32_t c = crc32(reinterpret_cast<const uint8_t*>(type), 4);
        c = crc32(reinterpret_cast<const uint8_t*>(data.data()), data.size(), c);
        s.be32(c ^ 0xFFFFFFFFu);
    };
    std::string ihdr(13, '\0');
    for (int k = 0; k < 4; k++) {
        ihdr[k] = (char)(width >> (24 - 8 * k));
        ihdr[4 + k] = (char)(height >> (24 - 8 * k));
    }
    ihdr[8] = 8;   // bit depth
    ihdr[9] = 6;   // RGBA
    chunk("IHDR", ihdr);
    // zlib stream of stored deflate blocks over (filter byte 0 + row) per row
    const size_t row = (size_t)width * 4;
    const size_t raw_n = (row + 1) * height;
    std::string z;
    z.reserve(raw_n + raw_n / 65535 * 5 + 16);
    z.push_back((char)0x78);
    z.push_back((char)0x01);
    uint32_t a1 = 1, a2 = 0;  // Adler-32
    std::string block;
    size_t done = 0;
    auto flush = [&](bool last) {
        const uint16_t n = (uint16_t)block.size();
        z.push_back((char)(last ? 1 : 0));
        z.push_back((char)(n & 0xFF));
        z.push_back((char)(n >> 8));
        z.push_back((char)(~n & 0xFF));
        z.push_back((char)((uint16_t)~n >> 8));
        z += block;
        block.clear();
    };
    for (uint32_t y = 0; y < height; y++) {
        for (size_t i = 0; i <= row; i++) {
            const uint8_t b = i == 0 ? 0 : rgba[(size_t)y * row + i - 1];
            a1 = (a1 + b) % 65521u;
            a2 = (a2 + a1) % 65521u;
            block.push_back((char)b);
            done++;
            if (block.size() == 65535) flush(done == raw_n);
        }
    }
    if (!block.empty() || done == 0) flush(true);
    const uint32_t ad = (a2 << 16) | a1;
    for (int k = 0; k < 4; k++) z.push_back((char)(ad >> (24 - 8 * k)));
    chunk("IDAT", z);
    chunk("IEND", std::string());
    *len = s.n;
    if (out && s.n > cap) return RTW_E_INVALID;
    return RTW_OK;
}

}  // extern "C"
