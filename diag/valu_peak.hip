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

// one instruction class per kernel (16 independent chains x UNR per loop branch): its issue cost and
// whether two waves' instances dual-issue (SQ_ACTIVE_INST_VALU2).  Operands are garbage; only timing counts.
enum Cls { C_CNDMASK = 0, C_MAX3, C_FMA_MIX, C_SQRT, C_RCP, C_ADD_U32, C_MUL_LO_U32, C_MOV, C_CMP_SGPR,
           C_FMA_SGPR, C_MUL_F32, C_CNDMASK_VCC, C_LSHL_ADD, C_BFE, C_XOR,
           C_MIN_F32, C_MAX_F32, C_MIN3, C_MED3, C_SUB_F32, C_ADD_ABS, C_SUB_NEG, C_CMP_VCC, C_CMP_VCC_CND,
           C_AND, C_OR, C_LSHL, C_LSHR, C_CVT_F16, C_PK_ADD, C_PK_MUL, C_PERM, C_MUL_HI, C_FMA_INLINE,
           C_ADD_LITERAL, C_FMAC, C_MUL_U24, C_CMP_SGPR_OPND, C_LDEXP,
           C_MAX_I32, C_MIN_U32, C_MAX3_I32, C_SUB_U32, C_ASHR_I32, C_ADD3_U32, C_LSHL_OR, C_BFI, C_CNDMASK_VGPR3,
           C_PK_MAX_F16, C_MUL_F32_SGPR, C_ADD_F32_SGPR, C_COUNT };
template <int K>
__device__ __forceinline__ void cls_step(float& a, float b, float c, uint64_t m, uint64_t& sm, float sc) {
    if constexpr (K == C_CNDMASK) asm volatile("v_cndmask_b32_e64 %0, %0, %1, %2" : "+v"(a) : "v"(b), "s"(m));
    if constexpr (K == C_MAX3) asm volatile("v_max3_f32 %0, %0, %1, %2" : "+v"(a) : "v"(b), "v"(c));
    if constexpr (K == C_FMA_MIX) asm volatile("v_fma_mix_f32 %0, %1, %2, %0 op_sel_hi:[1,0,0]" : "+v"(a) : "v"(b), "v"(c));
    if constexpr (K == C_SQRT) asm volatile("v_sqrt_f32 %0, %0" : "+v"(a));
    if constexpr (K == C_RCP) asm volatile("v_rcp_f32 %0, %0" : "+v"(a));
    if constexpr (K == C_ADD_U32) asm volatile("v_add_u32 %0, %0, %1" : "+v"(a) : "v"(b));
    if constexpr (K == C_MUL_LO_U32) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(a) : "v"(b));
    if constexpr (K == C_MOV) asm volatile("v_mov_b32 %0, %1" : "=v"(a) : "v"(b));
    if constexpr (K == C_CMP_SGPR) asm volatile("v_cmp_gt_f32_e64 %0, %1, %2" : "=s"(sm) : "v"(a), "v"(b));
    if constexpr (K == C_FMA_SGPR) asm volatile("v_fma_f32 %0, %1, %2, %0" : "+v"(a) : "v"(b), "s"(sc));
    if constexpr (K == C_MUL_F32) asm volatile("v_mul_f32 %0, %0, %1" : "+v"(a) : "v"(b));
    if constexpr (K == C_CNDMASK_VCC) asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(a) : "v"(b));
    if constexpr (K == C_LSHL_ADD) asm volatile("v_lshl_add_u32 %0, %0, 4, %1" : "+v"(a) : "v"(b));
    if constexpr (K == C_BFE) asm volatile("v_bfe_u32 %0, %0, 8, 8" : "+v"(a));
    if constexpr (K == C_XOR) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(a) : "v"(b));
    if constexpr (K == C_MIN_F32) asm volatile("v_min_f32 %0, %0, %1" : "+v"(a) : "v"(b));
    if constexpr (K == C_MAX_F32) asm volatile("v_max_f32 %0, %0, %1" : "+v"(a) : "v"(b));
    if constexpr (K == C_MIN3) asm volatile("v_min3_f32 %0, %0, %1, %2" : "+v"(a) : "v"(b), "v"(c));
    if constexpr (K == C_MED3) asm volatile("v_med3_f32 %0, %0, %1, %2" : "+v"(a) : "v"(b), "v"(c));
    if constexpr (K == C_SUB_F32) asm volatile("v_sub_f32 %0, %0, %1" : "+v"(a) : "v"(b));
    if constexpr (K == C_ADD_ABS) asm volatile("v_add_f32_e64 %0, %0, |%1|" : "+v"(a) : "v"(b));
    if constexpr (K == C_SUB_NEG) asm volatile("v_sub_f32_e64 %0, -%0, %1" : "+v"(a) : "v"(b));
    if constexpr (K == C_CMP_VCC) asm volatile("v_cmp_gt_f32 vcc, %0, %1" : : "v"(a), "v"(b) : "vcc");
    if constexpr (K == C_CMP_VCC_CND)
        asm volatile("v_cmp_gt_f32 vcc, %0, %1\n\ts_nop 0\n\tv_cndmask_b32 %0, %0, %1, vcc" : "+v"(a) : "v"(b) : "vcc");
    if constexpr (K == C_AND) asm volatile("v_and_b32 %0, %0, %1" : "+v"(a) : "v"(b));
    if constexpr (K == C_OR) asm volatile("v_or_b32 %0, %0, %1" : "+v"(a) : "v"(b));
    if constexpr (K == C_LSHL) asm volatile("v_lshlrev_b32 %0, 3, %0" : "+v"(a));
    if constexpr (K == C_LSHR) asm volatile("v_lshrrev_b32 %0, 3, %0" : "+v"(a));
    if constexpr (K == C_CVT_F16) asm volatile("v_cvt_f32_f16 %0, %1" : "=v"(a) : "v"(b));
    if constexpr (K == C_PERM) asm volatile("v_perm_b32 %0, %0, %1, %2" : "+v"(a) : "v"(b), "v"(c));
    if constexpr (K == C_MUL_HI) asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(a) : "v"(b));
    if constexpr (K == C_FMA_INLINE) asm volatile("v_fma_f32 %0, %0, %1, 1.0" : "+v"(a) : "v"(b));
    if constexpr (K == C_ADD_LITERAL) asm volatile("v_add_f32 %0, 0x35800000, %0" : "+v"(a));
    if constexpr (K == C_FMAC) asm volatile("v_fmac_f32 %0, %1, %2" : "+v"(a) : "v"(b), "v"(c));
    if constexpr (K == C_MUL_U24) asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(a) : "v"(b));
    if constexpr (K == C_CMP_SGPR_OPND) asm volatile("v_cmp_gt_f32 vcc, %0, %1" : : "s"(sc), "v"(a) : "vcc");
    if constexpr (K == C_LDEXP) asm volatile("v_ldexp_f32 %0, %0, %1" : "+v"(a) : "v"(b));
    if constexpr (K == C_MAX_I32) asm volatile("v_max_i32 %0, %0, %1" : "+v"(a) : "v"(b));
    if constexpr (K == C_MIN_U32) asm volatile("v_min_u32 %0, %0, %1" : "+v"(a) : "v"(b));
    if constexpr (K == C_MAX3_I32) asm volatile("v_max3_i32 %0, %0, %1, %2" : "+v"(a) : "v"(b), "v"(c));
    if constexpr (K == C_SUB_U32) asm volatile("v_sub_u32 %0, %0, %1" : "+v"(a) : "v"(b));
    if constexpr (K == C_ASHR_I32) asm volatile("v_ashrrev_i32 %0, 3, %0" : "+v"(a));
    if constexpr (K == C_ADD3_U32) asm volatile("v_add3_u32 %0, %0, %1, %2" : "+v"(a) : "v"(b), "v"(c));
    if constexpr (K == C_LSHL_OR) asm volatile("v_lshl_or_b32 %0, %0, 3, %1" : "+v"(a) : "v"(b));
    if constexpr (K == C_BFI) asm volatile("v_bfi_b32 %0, %0, %1, %2" : "+v"(a) : "v"(b), "v"(c));
    if constexpr (K == C_CNDMASK_VGPR3) asm volatile("v_cndmask_b32_e64 %0, %0, %1, %2" : "+v"(a) : "v"(b), "s"(m));
    if constexpr (K == C_PK_MAX_F16) asm volatile("v_pk_max_f16 %0, %0, %1" : "+v"(a) : "v"(b));
    if constexpr (K == C_MUL_F32_SGPR) asm volatile("v_mul_f32 %0, %1, %0" : "+v"(a) : "s"(sc));
    if constexpr (K == C_ADD_F32_SGPR) asm volatile("v_add_f32 %0, %1, %0" : "+v"(a) : "s"(sc));
}
// packed pairs (64-bit registers)
template <int K>
__global__ void cls_pk_chains(float* out, int iters, float b, float c) {
    extern __shared__ float lds_pad[];
    typedef float f2 __attribute__((ext_vector_type(2)));
    f2 a[16];
    const f2 bb = {b, c};
#pragma unroll
    for (int i = 0; i < 16; ++i) a[i] = f2{(float)threadIdx.x, (float)i};
    for (int it = 0; it < iters; it += 16) {
#pragma unroll
        for (int u = 0; u < 16; ++u)
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                if constexpr (K == C_PK_ADD) asm volatile("v_pk_add_f32 %0, %0, %1" : "+v"(a[i]) : "v"(bb));
                else asm volatile("v_pk_mul_f32 %0, %0, %1" : "+v"(a[i]) : "v"(bb));
            }
    }
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < 16; ++i) s += a[i].x + a[i].y;
    if (threadIdx.x == 0) lds_pad[0] = s;
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
template <int K>
__global__ void cls_chains(float* out, int iters, float b, float c) {
    extern __shared__ float lds_pad[];
    float a[16];
    uint64_t sm[16];
    const uint64_t m = __ballot(threadIdx.x & 1);
#pragma unroll
    for (int i = 0; i < 16; ++i) { a[i] = (float)(threadIdx.x + i); sm[i] = 0; }
    for (int it = 0; it < iters; it += 16) {
#pragma unroll
        for (int u = 0; u < 16; ++u)
#pragma unroll
            for (int i = 0; i < 16; ++i) cls_step<K>(a[i], b, c, m, sm[i], c);
    }
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < 16; ++i) s += a[i] + (float)(sm[i] & 1);
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

    Case cases[192];
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
    {
        static const char* cls_names[C_COUNT] = {"cndmask_sgpr", "max3", "fma_mix", "sqrt", "rcp", "add_u32",
                                                 "mul_lo_u32", "mov", "cmp_to_sgpr", "fma_sgpr_operand", "mul_f32",
                                                 "cndmask_vcc", "lshl_add_u32", "bfe_u32", "xor_b32",
                                                 "min_f32", "max_f32", "min3_f32", "med3_f32", "sub_f32", "add_abs_e64",
                                                 "sub_neg_e64", "cmp_to_vcc", "cmp_vcc_nop_cndmask_pair", "and_b32",
                                                 "or_b32", "lshlrev_b32", "lshrrev_b32", "cvt_f32_f16", "pk_add_f32",
                                                 "pk_mul_f32", "perm_b32", "mul_hi_u32", "fma_inline_const",
                                                 "add_literal", "fmac_f32", "mul_u32_u24", "cmp_sgpr_operand", "ldexp_f32",
                                                 "max_i32", "min_u32", "max3_i32", "sub_u32", "ashrrev_i32", "add3_u32",
                                                 "lshl_or_b32", "bfi_b32", "cndmask_sgpr_b", "pk_max_f16",
                                                 "mul_f32_sgpr_operand", "add_f32_sgpr_operand"};
#define CLS(k) (const void*)cls_chains<k>
        const void* fns[C_COUNT] = {CLS(0), CLS(1), CLS(2), CLS(3), CLS(4), CLS(5), CLS(6), CLS(7), CLS(8), CLS(9),
                                    CLS(10), CLS(11), CLS(12), CLS(13), CLS(14), CLS(15), CLS(16), CLS(17), CLS(18),
                                    CLS(19), CLS(20), CLS(21), CLS(22), CLS(23), CLS(24), CLS(25), CLS(26), CLS(27),
                                    CLS(28), (const void*)cls_pk_chains<C_PK_ADD>, (const void*)cls_pk_chains<C_PK_MUL>,
                                    CLS(31), CLS(32), CLS(33), CLS(34), CLS(35), CLS(36), CLS(37), CLS(38), CLS(39),
                                    CLS(40), CLS(41), CLS(42), CLS(43), CLS(44), CLS(45), CLS(46), CLS(47), CLS(48),
                                    CLS(49), CLS(50)};
#undef CLS
        static char names[C_COUNT][2][48];
        for (int kk = 0; kk < C_COUNT; ++kk) {
            const int wsel[2] = {4, 8};
            for (int j = 0; j < 2; ++j) {
                snprintf(names[kk][j], sizeof names[kk][j], "cls_%s", cls_names[kk]);
                cases[n++] = {names[kk][j], fns[kk], 1, 16, 256, wsel[j], lds_for(wsel[j])};
            }
        }
    }
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
