// valu_cost.hip — relative issue cost of single VALU instructions on gfx950 (experiment): 16
// independent chains per lane, 8 waves per SIMD; cost relative to v_fma_f32.
#include <hip/hip_runtime.h>
#include <cstdio>

#define BODY(asmstr)                                                                              \
    for (int it = 0; it < iters; ++it) {                                                          \
        _Pragma("unroll") for (int i = 0; i < 16; ++i) asm volatile(asmstr : "+v"(a[i]) : "v"(b), "v"(c)); \
    }
#define KERNEL(NAME, asmstr)                                                                      \
    __global__ __launch_bounds__(256) void NAME(unsigned *out, int iters) {                       \
        unsigned a[16];                                                                           \
        for (int i = 0; i < 16; ++i) a[i] = threadIdx.x * 77u + i;                                \
        const unsigned b = 0x3f800001u, c = 0x04030201u;                                          \
        BODY(asmstr)                                                                              \
        unsigned s = 0;                                                                           \
        for (int i = 0; i < 16; ++i) s += a[i];                                                   \
        out[blockIdx.x * blockDim.x + threadIdx.x] = s;                                           \
    }

#define LIST(X)                                                       \
    X(k_fma, "v_fma_f32 %0, %0, %1, %2")                              \
    X(k_add_f32, "v_add_f32 %0, %0, %1")                              \
    X(k_sub_f32, "v_sub_f32 %0, %0, %1")                              \
    X(k_mul_f32, "v_mul_f32 %0, %0, %1")                              \
    X(k_fmac, "v_fmac_f32 %0, %1, %2")                                \
    X(k_min_f32, "v_min_f32 %0, %0, %1")                              \
    X(k_max3_f32, "v_max3_f32 %0, %0, %1, %2")                        \
    X(k_med3_f32, "v_med3_f32 %0, %0, %1, %2")                        \
    X(k_add_u32, "v_add_u32 %0, %0, %1")                              \
    X(k_sub_u32, "v_sub_u32 %0, %0, %1")                              \
    X(k_add3_u32, "v_add3_u32 %0, %0, %1, %2")                        \
    X(k_and_b32, "v_and_b32 %0, %0, %1")                              \
    X(k_or_b32, "v_or_b32 %0, %0, %1")                                \
    X(k_xor_b32, "v_xor_b32 %0, %0, %1")                              \
    X(k_lshl, "v_lshlrev_b32 %0, 3, %0")                              \
    X(k_lshr, "v_lshrrev_b32 %0, 3, %0")                              \
    X(k_lshl_add, "v_lshl_add_u32 %0, %0, 2, %1")                     \
    X(k_bfe, "v_bfe_u32 %0, %0, 8, 8")                                \
    X(k_mul_lo, "v_mul_lo_u32 %0, %0, %1")                            \
    X(k_mul_u24, "v_mul_u32_u24 %0, %0, %1")                          \
    X(k_mad_u24, "v_mad_u32_u24 %0, %0, %1, %2")                      \
    X(k_min_u32, "v_min_u32 %0, %0, %1")                              \
    X(k_max_i32, "v_max_i32 %0, %0, %1")                              \
    X(k_cvt_f32_u32, "v_cvt_f32_u32 %0, %0")                          \
    X(k_cvt_ubyte, "v_cvt_f32_ubyte1 %0, %0")                         \
    X(k_mov, "v_mov_b32 %0, %1")                                      \
    X(k_cmp_cnd, "v_cmp_lt_f32 vcc, %0, %1\n v_cndmask_b32 %0, %0, %1, vcc") \
    X(k_cmp_cnd_s, "v_cmp_lt_f32 s[40:41], %0, %1\n v_cndmask_b32_e64 %0, %0, %1, s[40:41]") \
    X(k_cmp, "v_cmp_lt_f32 vcc, %0, %1")                              \
    X(k_rcp, "v_rcp_f32 %0, %0")                                      \
    X(k_sqrt, "v_sqrt_f32 %0, %0")                                    \
    X(k_perm, "v_perm_b32 %0, %0, %1, %2")                            \
    X(k_xad, "v_xad_u32 %0, %0, %1, %2")                              \
    X(k_dpp, "v_mov_b32_dpp %0, %1 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf") \
    X(k_fma_mix, "v_fma_mix_f32 %0, %2, %1, %0 op_sel_hi:[1,0,0]")   \
    X(k_fma_mix_hi, "v_fma_mix_f32 %0, %2, %1, %0 op_sel:[1,0,0] op_sel_hi:[1,0,0]") \
    X(k_cvt_f16, "v_cvt_f32_f16 %0, %0")                              \
    X(k_xor_sdwa, "v_xor_b32_sdwa %0, %0, %0 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:WORD_1 src1_sel:DWORD") \
    X(k_max_f16, "v_max_f16 %0, %0, %1")                              \
    X(k_pk_max_f16, "v_pk_max_f16 %0, %0, %1")                        \
    X(k_alignbit, "v_alignbit_b32 %0, %0, %0, 15")                    \
    X(k_mul_hi, "v_mul_hi_u32 %0, %0, %1")                           

#define DEF(NAME, S) KERNEL(NAME, S)
LIST(DEF)

int main() {
    const int blocks = 256 * 8, iters = 4096;
    unsigned *out;
    (void)hipMalloc(&out, blocks * 256 * 4);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    float base = 0;
#define RUN(NAME, S)                                                                            \
    {                                                                                           \
        float ms = 0;                                                                           \
        for (int rep = 0; rep < 2; ++rep) {                                                     \
            (void)hipEventRecord(e0);                                                           \
            NAME<<<blocks, 256>>>(out, iters);                                                  \
            (void)hipEventRecord(e1);                                                           \
            (void)hipEventSynchronize(e1);                                                      \
            (void)hipEventElapsedTime(&ms, e0, e1);                                             \
        }                                                                                       \
        if (base == 0) base = ms;                                                               \
        printf("%-14s %-60s %6.3f ms  cost %.2f\n", #NAME, S, ms, ms / base);                   \
    }
    LIST(RUN)
    return 0;
}
