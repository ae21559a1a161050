// DIAGNOSTIC ONLY (not part of the product): the gfx950 VALU issue ceiling that bench.py's
// roofline divides by (VERDICT r3 "next round" item 1).
//
// Each lane runs NCH independent chains of one VALU instruction (inline asm, so the compiler can
// neither pack two v_fma_f32 into a v_pk_fma_f32 nor fold the chains), ITER times.  The number of
// waves per SIMD is set by the launch: 256-thread blocks put one wave on each of a CU's 4 SIMDs,
// and the block's dynamic LDS (160 KiB / w, rounded down so w blocks fit and w + 1 do not) allows
// exactly w resident blocks per CU -> w waves per SIMD.  The grid is ROUNDS x 256 CUs x w blocks,
// so the chip stays full for all but the last round.  One extra shape reproduces the product's
// fused step (wf_step_clds): 1024-thread blocks, 124 KiB of LDS -> one block per CU = 4 waves/SIMD.
//
// Output (one JSON line per case): wave-instructions, lane-ops, kernel ms (HIP events), lane-op/s,
// and the SIMD cycles per wave-instruction at the nominal 2.4 GHz.  Under rocprofv3 --pmc the same
// dispatches carry SQ_INSTS_VALU / SQ_ACTIVE_INST_VALU / GRBM_GUI_ACTIVE (tools/valu_peak.sh).
//
// Build: hipcc --offload-arch=gfx950 -O3 -o diag/valu_peak diag/valu_peak.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>

#define CK(x)                                                                              \
    do {                                                                                   \
        hipError_t e_ = (x);                                                               \
        if (e_ != hipSuccess) {                                                            \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(1);                                                                       \
        }                                                                                  \
    } while (0)

enum Op { OP_FMA = 0, OP_ADD = 1 };

template <int OP>
__device__ __forceinline__ void step(float& a, float b, float c) {
    if constexpr (OP == OP_FMA) {
        asm volatile("v_fma_f32 %0, %1, %2, %0" : "+v"(a) : "v"(b), "v"(c));
    } else if constexpr (OP == OP_ADD) {
        asm volatile("v_add_f32 %0, %1, %0" : "+v"(a) : "v"(b));
    }
}

// NCH independent chains of one op per lane, ITER trips of UNR rounds (UNR x NCH instructions per loop
// branch); out[] keeps the chains live
template <int OP, int NCH, int UNR = 1>
__global__ void valu_chains(float* out, int iters, float b, float c) {
    extern __shared__ float lds_pad[];   // only sizes occupancy; touched once so it is allocated
    float a[NCH];
#pragma unroll
    for (int i = 0; i < NCH; ++i) a[i] = (float)(threadIdx.x + i);
    for (int it = 0; it < iters; it += UNR) {
#pragma unroll
        for (int u = 0; u < UNR; ++u)
#pragma unroll
            for (int i = 0; i < NCH; ++i) step<OP>(a[i], b, c);
    }
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < NCH; ++i) s += a[i];
    if (threadIdx.x == 0) lds_pad[0] = s;
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

// packed form: one v_pk_fma_f32 = 2 lane-ops per lane
template <int NCH>
__global__ void valu_pk_chains(float* out, int iters, float b, float c) {
    extern __shared__ float lds_pad[];
    typedef float f2 __attribute__((ext_vector_type(2)));
    f2 a[NCH];
    f2 bb = {b, b}, cc = {c, c};
#pragma unroll
    for (int i = 0; i < NCH; ++i) a[i] = f2{(float)threadIdx.x, (float)i};
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int i = 0; i < NCH; ++i) asm volatile("v_pk_fma_f32 %0, %1, %2, %0" : "+v"(a[i]) : "v"(bb), "v"(cc));
    }
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < NCH; ++i) s += a[i].x + a[i].y;
    if (threadIdx.x == 0) lds_pad[0] = s;
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

// LDS pointer chase: each lane follows idx = lds[idx] (ds_read_b32, dependent), `iters` times; the
// table is a random cycle over the block's LDS words, so lanes conflict as a walk's node reads do
__global__ void lds_chase(float* out, int iters, float b, float c) {
    extern __shared__ uint32_t tab[];
    const uint32_t n = (uint32_t)(b);  // table words (a power of two)
    for (uint32_t k = threadIdx.x; k < n; k += blockDim.x) tab[k] = (k * 2654435761u + 12345u) & (n - 1u);
    __syncthreads();
    uint32_t i = (threadIdx.x * 97u) & (n - 1u);
    for (int it = 0; it < iters; ++it) i = tab[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = (float)i + c;
}

// the same chase with ds_read_b128 (16-B records, the compact walk's node read)
__global__ void lds_chase128(float* out, int iters, float b, float c) {
    extern __shared__ uint4 tab4[];
    const uint32_t n = (uint32_t)(b) / 4u;  // records
    for (uint32_t k = threadIdx.x; k < n; k += blockDim.x) {
        const uint32_t nx = (k * 2654435761u + 12345u) & (n - 1u);
        tab4[k] = make_uint4(nx, nx, nx, nx);
    }
    __syncthreads();
    uint32_t i = (threadIdx.x * 97u) & (n - 1u);
    for (int it = 0; it < iters; ++it) {
        const uint4 v = tab4[i];
        i = v.x ^ (v.y & 0u);
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = (float)i + c;
}

// where a block's waves run: HW_ID (s_getreg, hwreg 4: wave 3:0, SIMD 5:4, CU 11:8) per wave
__global__ void placement(uint32_t* out) {
    extern __shared__ float lds_pad[];
    const uint32_t id = __builtin_amdgcn_s_getreg((31 << 11) | (0 << 6) | 4);
    if ((threadIdx.x & 63u) == 0) out[blockIdx.x * (blockDim.x / 64u) + threadIdx.x / 64u] = id;
    if (threadIdx.x == 0) lds_pad[0] = 0.f;
}

struct Case {
    const char* name;
    const void* fn;
    int op_lane_ops;   // lane-ops per instruction per lane (2 for packed)
    int nch;
    int block;         // threads per block
    int waves_simd;    // intended resident waves per SIMD
    int lds;           // dynamic LDS bytes per block
};

static int lds_for(int w) {
    // w blocks of this size fit in 160 KiB, w + 1 do not
    return (160 * 1024) / w - 1024;
}

int main(int argc, char** argv) {
    int iters = argc > 1 ? atoi(argv[1]) : 50000;
    const int rounds = argc > 2 ? atoi(argv[2]) : 8;
    int dev = 0;
    CK(hipSetDevice(dev));
    hipDeviceProp_t p;
    CK(hipGetDeviceProperties(&p, dev));
    const int cus = p.multiProcessorCount;
    fprintf(stderr, "device %s, %d CUs, clock %d kHz, LDS/block max %zu\n", p.gcnArchName, cus, p.clockRate,
            p.sharedMemPerBlock);

    Case cases[64];
    int n = 0;
    const int waves[] = {1, 2, 4, 8};
    for (int w : waves) {
        cases[n++] = {"fma_ch16", (const void*)valu_chains<OP_FMA, 16>, 1, 16, 256, w, lds_for(w)};
    }
    for (int w : waves) {
        cases[n++] = {"fma_ch4", (const void*)valu_chains<OP_FMA, 4>, 1, 4, 256, w, lds_for(w)};
    }
    for (int w : waves) {
        cases[n++] = {"add_ch16", (const void*)valu_chains<OP_ADD, 16>, 1, 16, 256, w, lds_for(w)};
    }
    for (int w : waves) {
        cases[n++] = {"pkfma_ch16", (const void*)valu_pk_chains<16>, 2, 16, 256, w, lds_for(w)};
    }
    cases[n++] = {"fma_ch1", (const void*)valu_chains<OP_FMA, 1>, 1, 1, 256, 8, lds_for(8)};
    // the product's fused-step shape: 1024-thread block + 124 KiB stage -> 1 block / CU = 4 waves / SIMD
    cases[n++] = {"fma_ch16_wfstep_shape", (const void*)valu_chains<OP_FMA, 16>, 1, 16, 1024, 4, 124 * 1024};
    cases[n++] = {"fma_ch4_wfstep_shape", (const void*)valu_chains<OP_FMA, 4>, 1, 4, 1024, 4, 124 * 1024};
    cases[n++] = {"fma_ch8_wfstep_shape", (const void*)valu_chains<OP_FMA, 8>, 1, 8, 1024, 4, 124 * 1024};
    cases[n++] = {"fma_ch2_wfstep_shape", (const void*)valu_chains<OP_FMA, 2>, 1, 2, 1024, 4, 124 * 1024};
    cases[n++] = {"fma_ch1_wfstep_shape", (const void*)valu_chains<OP_FMA, 1>, 1, 1, 1024, 4, 124 * 1024};
    cases[n++] = {"fma_ch16_block1024_2pcu", (const void*)valu_chains<OP_FMA, 16>, 1, 16, 1024, 8, 60 * 1024};
    cases[n++] = {"fma_ch16_block512_w4", (const void*)valu_chains<OP_FMA, 16>, 1, 16, 512, 4, 60 * 1024};
    // the loop branch amortised over 256 instructions (a taken branch per 16 or fewer costs issue time)
    for (int w : waves) cases[n++] = {"fma_ch16_unr16", (const void*)valu_chains<OP_FMA, 16, 16>, 1, 16, 256, w, lds_for(w)};
    for (int w : waves) cases[n++] = {"fma_ch4_unr64", (const void*)valu_chains<OP_FMA, 4, 64>, 1, 4, 256, w, lds_for(w)};
    for (int w : waves) cases[n++] = {"fma_ch1_unr256", (const void*)valu_chains<OP_FMA, 1, 256>, 1, 1, 256, w, lds_for(w)};
    cases[n++] = {"fma_ch16_unr16_wfstep_shape", (const void*)valu_chains<OP_FMA, 16, 16>, 1, 16, 1024, 4, 124 * 1024};
    cases[n++] = {"fma_ch4_unr64_wfstep_shape", (const void*)valu_chains<OP_FMA, 4, 64>, 1, 4, 1024, 4, 124 * 1024};
    cases[n++] = {"fma_ch1_unr256_wfstep_shape", (const void*)valu_chains<OP_FMA, 1, 256>, 1, 1, 1024, 4, 124 * 1024};
    const int n_valu = n;
    // LDS dependent-read latency (lane-ops = reads): 16 KiB table, 1 chain per lane
    for (int w : waves) cases[n++] = {"lds_chase_b32", (const void*)lds_chase, 1, 1, 256, w, lds_for(w)};
    for (int w : waves) cases[n++] = {"lds_chase_b128", (const void*)lds_chase128, 1, 1, 256, w, lds_for(w)};
    cases[n++] = {"lds_chase_b128_wfstep_shape", (const void*)lds_chase128, 1, 1, 1024, 4, 124 * 1024};

    float* out;
    size_t max_threads = (size_t)rounds * cus * 8 * 256 + 1024 * cus * rounds;
    CK(hipMalloc(&out, max_threads * sizeof(float)));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int k = 0; k < n; ++k) {
        Case& c = cases[k];
        CK(hipFuncSetAttribute(c.fn, hipFuncAttributeMaxDynamicSharedMemorySize, c.lds));
        int blocks_per_cu = c.waves_simd * 256 / c.block;
        int grid = rounds * cus * blocks_per_cu;
        const bool chase = k >= n_valu;
        int it = chase ? iters / 8 : (c.nch >= 16 ? iters : iters * (16 / c.nch));
        float b = chase ? 4096.0f : 1.0000001f, cc = chase ? 0.0f : 1e-7f;
        void* args[] = {&out, &it, &b, &cc};
        // warm-up launch (clocks, code object load)
        CK(hipLaunchKernel(c.fn, dim3(grid), dim3(c.block), args, c.lds, 0));
        CK(hipDeviceSynchronize());
        int occ = 0;
        CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, c.fn, c.block, c.lds));
        float best = 1e30f;
        for (int rep = 0; rep < 3; ++rep) {
            CK(hipEventRecord(e0, 0));
            CK(hipLaunchKernel(c.fn, dim3(grid), dim3(c.block), args, c.lds, 0));
            CK(hipEventRecord(e1, 0));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            if (ms < best) best = ms;
        }
        double wave_insts = (double)grid * (c.block / 64) * it * c.nch;
        double lane_ops = wave_insts * 64 * c.op_lane_ops;
        double s = best * 1e-3;
        if (chase) {  // per-wave cycles of one dependent LDS read
            const double waves_per_simd_resident = c.waves_simd;
            printf("{\"case\": \"%s\", \"block\": %d, \"waves_per_simd\": %d, \"occupancy_blocks_per_cu\": %d, "
                   "\"grid\": %d, \"iters\": %d, \"ms\": %.4f, \"wave_reads\": %.6g, "
                   "\"cycles_per_dependent_read_per_wave_at_2p4GHz\": %.2f, \"simd_cycles_per_wave_read\": %.3f}\n",
                   c.name, c.block, c.waves_simd, occ, grid, it, best, wave_insts,
                   s * 2.4e9 * cus * 4.0 * waves_per_simd_resident / wave_insts, s * 2.4e9 * cus * 4.0 / wave_insts);
            fflush(stdout);
            continue;
        }
        double simds = cus * 4.0;
        double cyc_per_inst = s * 2.4e9 * simds / wave_insts;
        printf("{\"case\": \"%s\", \"block\": %d, \"waves_per_simd\": %d, \"occupancy_blocks_per_cu\": %d, "
               "\"lds\": %d, \"chains\": %d, \"grid\": %d, \"iters\": %d, \"wave_insts\": %.6g, "
               "\"lane_ops\": %.6g, \"ms\": %.4f, \"tlane_ops_per_s\": %.4f, \"simd_cycles_per_wave_inst_at_2p4GHz\": %.4f}\n",
               c.name, c.block, c.waves_simd, occ, c.lds, c.nch, grid, it, wave_insts, lane_ops, best,
               lane_ops / s / 1e12, cyc_per_inst);
        fflush(stdout);
    }
    // wave placement of a 256-thread block alone on its CU and of the fused step's 1024-thread shape
    uint32_t* ids;
    CK(hipMalloc(&ids, 4096 * 16 * sizeof(uint32_t)));
    const int shapes[2][2] = {{256, 159 * 1024}, {1024, 124 * 1024}};
    for (auto& sh : shapes) {
        CK(hipFuncSetAttribute((const void*)placement, hipFuncAttributeMaxDynamicSharedMemorySize, sh[1]));
        const int grid = cus, wpb = sh[0] / 64;
        hipLaunchKernelGGL(placement, dim3(grid), dim3(sh[0]), sh[1], 0, ids);
        CK(hipDeviceSynchronize());
        uint32_t* h = (uint32_t*)malloc(grid * wpb * 4);
        CK(hipMemcpy(h, ids, grid * wpb * 4, hipMemcpyDeviceToHost));
        int hist[5][17] = {{0}};  // [SIMD][waves of one block on it]
        for (int bI = 0; bI < grid; ++bI) {
            int per[4] = {0, 0, 0, 0};
            for (int w = 0; w < wpb; ++w) per[(h[bI * wpb + w] >> 4) & 3]++;
            for (int sI = 0; sI < 4; ++sI) hist[sI][per[sI] > 16 ? 16 : per[sI]]++;
        }
        printf("{\"case\": \"placement\", \"block\": %d, \"blocks\": %d, \"blocks_with_k_waves_on_simd\": [", sh[0], grid);
        for (int sI = 0; sI < 4; ++sI) {
            printf("%s{", sI ? ", " : "");
            int first = 1;
            for (int kk = 0; kk <= 16; ++kk)
                if (hist[sI][kk]) { printf("%s\"%d\": %d", first ? "" : ", ", kk, hist[sI][kk]); first = 0; }
            printf("}");
        }
        printf("]}\n");
        free(h);
    }
    CK(hipFree(ids));
    CK(hipFree(out));
    return 0;
}
