// pkfma_bench.hip — relative issue cost of single VALU instructions on gfx950 (experiment for
// the quantized-BVH decode and the hash RNG): 16 independent chains per lane, 8 waves per SIMD.
#include <hip/hip_runtime.h>
#include <cstdio>

#define OP(asmstr) asm volatile(asmstr : "+v"(a[i]) : "v"(b), "v"(c))
template <int MODE>
__global__ __launch_bounds__(256) void bench(unsigned *out, int iters) {
    unsigned a[16];
    for (int i = 0; i < 16; ++i) a[i] = threadIdx.x * 77u + i;
    const unsigned b = 0x3f800001u, c = 0x04030201u;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            if (MODE == 0) OP("v_fma_f32 %0, %0, %1, %2");
            if (MODE == 1) OP("v_cvt_f32_ubyte1 %0, %0");
            if (MODE == 2) OP("v_perm_b32 %0, %0, %1, %2");
            if (MODE == 3) OP("v_mul_lo_u32 %0, %0, %1");
            if (MODE == 4) OP("v_cvt_f32_u32 %0, %0");
            if (MODE == 5) OP("v_bfe_u32 %0, %0, 8, 8");
            if (MODE == 6) OP("v_ldexp_f32 %0, %0, %2");
            if (MODE == 7) OP("v_xor_b32 %0, %0, %1");
            if (MODE == 9) OP("v_or_b32_sdwa %0, %1, %0 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_1");
            if (MODE == 10) OP("v_add_u32 %0, %0, %1");
            if (MODE == 11) OP("v_min_f32 %0, %0, %1");
            if (MODE == 12) OP("v_max3_f32 %0, %0, %1, %2");
            if (MODE == 13) OP("v_cndmask_b32 %0, %0, %1, vcc");
            if (MODE == 14) OP("v_lshlrev_b32 %0, 3, %0");
            if (MODE == 15) OP("v_mul_f32 %0, %0, %1");
        }
    }
    unsigned s = 0;
    for (int i = 0; i < 16; ++i) s += a[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <>
__global__ __launch_bounds__(256) void bench<8>(unsigned *out, int iters) {
    typedef float f2 __attribute__((ext_vector_type(2)));
    f2 a[8];
    for (int i = 0; i < 8; ++i) a[i] = f2{threadIdx.x * 0.01f + i, 1.0f};
    const f2 b = {1.0001f, 0.999f}, c = {0.5f, 0.25f};
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int i = 0; i < 8; ++i) asm volatile("v_pk_fma_f32 %0, %0, %1, %2" : "+v"(a[i]) : "v"(b), "v"(c));
        // 8 pk instructions per iteration: counted as 16 below (2 lanes' worth each) -> rate per pair
    }
    float s = 0;
    for (int i = 0; i < 8; ++i) s += a[i].x + a[i].y;
    out[blockIdx.x * blockDim.x + threadIdx.x] = __float_as_uint(s);
}

template <int MODE>
float run(unsigned *out, int blocks, int iters) {
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    float ms = 0;
    for (int rep = 0; rep < 2; ++rep) {
        (void)hipEventRecord(e0);
        bench<MODE><<<blocks, 256>>>(out, iters);
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        (void)hipEventElapsedTime(&ms, e0, e1);
    }
    return ms;
}

int main() {
    const int blocks = 256 * 8, iters = 8192;
    unsigned *out;
    (void)hipMalloc(&out, blocks * 256 * 4);
    const char *names[16] = {"v_fma_f32", "v_cvt_f32_ubyte1", "v_perm_b32", "v_mul_lo_u32", "v_cvt_f32_u32",
                             "v_bfe_u32", "v_ldexp_f32", "v_xor_b32", "v_pk_fma_f32 (x8/iter)", "v_or_b32_sdwa BYTE_1",
                             "v_add_u32", "v_min_f32", "v_max3_f32", "v_cndmask_b32", "v_lshlrev_b32", "v_mul_f32"};
    float ms[16];
    ms[0] = run<0>(out, blocks, iters);
    ms[1] = run<1>(out, blocks, iters);
    ms[2] = run<2>(out, blocks, iters);
    ms[3] = run<3>(out, blocks, iters);
    ms[4] = run<4>(out, blocks, iters);
    ms[5] = run<5>(out, blocks, iters);
    ms[6] = run<6>(out, blocks, iters);
    ms[7] = run<7>(out, blocks, iters);
    ms[8] = run<8>(out, blocks, iters);
    ms[9] = run<9>(out, blocks, iters);
    ms[10] = run<10>(out, blocks, iters);
    ms[11] = run<11>(out, blocks, iters);
    ms[12] = run<12>(out, blocks, iters);
    ms[13] = run<13>(out, blocks, iters);
    ms[14] = run<14>(out, blocks, iters);
    ms[15] = run<15>(out, blocks, iters);
    for (int m = 0; m < 16; ++m) {
        const double winst = double(blocks) * 4 * iters * (m == 8 ? 8 : 16);
        printf("%-24s %7.3f ms  %7.1f G wave-inst/s  cost %.2f x v_fma_f32\n", names[m], ms[m], winst / ms[m] / 1e6,
               (ms[m] / (m == 8 ? 8 : 16)) / (ms[0] / 16));
    }
    return 0;
}
