// rn_check.hip — exhaustive check of short correctly-rounded sqrt / reciprocal sequences against
// the compiler's IEEE sqrtf and 1.0f/x on gfx950 (experiment; run on the GPU box).  Every float
// bit pattern is checked; mismatches are counted per candidate and biased exponent of x.
//   c0 raw v_sqrt_f32                      vs sqrtf(x)
//   c1 v_sqrt_f32 + one-ulp fix-up         vs sqrtf(x)          (no denormal scaling / class test)
//   c2 raw v_rcp_f32                       vs 1.0f / x
//   c3 v_rcp_f32 + one Newton step (fma)   vs 1.0f / x
//   c4 c3(c1(x))                           vs 1.0f / sqrtf(x)
//   c5 raw v_rsq_f32                       vs 1.0f / sqrtf(x)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstring>

#pragma clang fp contract(off)

constexpr int kCand = 6;

__device__ __forceinline__ float sqrt_fix(float x) {
    const float s = __builtin_amdgcn_sqrtf(x);
    const float sm = __uint_as_float(__float_as_uint(s) - 1u);
    const float sp = __uint_as_float(__float_as_uint(s) + 1u);
    float r = s;
    if (fmaf(-sm, s, x) <= 0.0f) r = sm;
    if (fmaf(-sp, s, x) > 0.0f) r = sp;
    return r;
}

__device__ __forceinline__ float rcp_nr(float x) {
    const float y = __builtin_amdgcn_rcpf(x);
    const float e = fmaf(-x, y, 1.0f);
    return fmaf(e, y, y);
}

__device__ __forceinline__ bool same(float a, float b) {
    return __float_as_uint(a) == __float_as_uint(b) || (a != a && b != b);
}

__global__ __launch_bounds__(256) void check(unsigned long long *cnt, unsigned *first, unsigned long long base,
                                             unsigned long long n) {
    __shared__ unsigned local[kCand * 256];
    for (int i = threadIdx.x; i < kCand * 256; i += 256) local[i] = 0;
    __syncthreads();
    for (unsigned long long i = blockIdx.x * 256ull + threadIdx.x; i < n; i += gridDim.x * 256ull) {
        const unsigned u = unsigned(base + i);
        const float x = __uint_as_float(u);
        const unsigned e = (u >> 23) & 255u;
        const float sq = sqrtf(x), rc = 1.0f / x, isq = 1.0f / sqrtf(x);
        bool bad[kCand];
        bad[0] = !same(__builtin_amdgcn_sqrtf(x), sq);
        bad[1] = !same(sqrt_fix(x), sq);
        bad[2] = !same(__builtin_amdgcn_rcpf(x), rc);
        bad[3] = !same(rcp_nr(x), rc);
        bad[4] = !same(rcp_nr(sqrt_fix(x)), isq);
        bad[5] = !same(__builtin_amdgcn_rsqf(x), isq);
        for (int c = 0; c < kCand; ++c)
            if (bad[c]) {
                atomicAdd(&local[c * 256 + e], 1u);
                atomicMin(&first[c * 256 + e], u);
            }
    }
    __syncthreads();
    for (int i = threadIdx.x; i < kCand * 256; i += 256)
        if (local[i]) atomicAdd(&cnt[i], (unsigned long long)local[i]);
}

int main(int argc, char **argv) {
    // positive floats only by default (sign symmetric); "all" checks every pattern
    const bool all = argc > 1 && !strcmp(argv[1], "all");
    const unsigned long long total = all ? (1ull << 32) : (1ull << 31);
    unsigned long long *dCnt;
    unsigned *dFirst;
    hipMalloc(&dCnt, sizeof(unsigned long long) * kCand * 256);
    hipMalloc(&dFirst, sizeof(unsigned) * kCand * 256);
    hipMemset(dCnt, 0, sizeof(unsigned long long) * kCand * 256);
    hipMemset(dFirst, 0xff, sizeof(unsigned) * kCand * 256);
    const unsigned long long chunk = 1ull << 28;
    for (unsigned long long b = 0; b < total; b += chunk) hipLaunchKernelGGL(check, dim3(8192), dim3(256), 0, 0, dCnt, dFirst, b, chunk);
    if (hipDeviceSynchronize() != hipSuccess) {
        printf("kernel failed\n");
        return 1;
    }
    unsigned long long cnt[kCand * 256];
    unsigned first[kCand * 256];
    hipMemcpy(cnt, dCnt, sizeof(cnt), hipMemcpyDeviceToHost);
    hipMemcpy(first, dFirst, sizeof(first), hipMemcpyDeviceToHost);
    const char *names[kCand] = {"raw_sqrt", "sqrt_fix", "raw_rcp", "rcp_nr", "rcp_nr(sqrt_fix)", "raw_rsq"};
    for (int c = 0; c < kCand; ++c) {
        unsigned long long t = 0;
        for (int e = 0; e < 256; ++e) t += cnt[c * 256 + e];
        printf("%-18s mismatches %llu of %llu\n", names[c], t, total);
        for (int e = 0; e < 256; ++e)
            if (cnt[c * 256 + e]) printf("    exp %3d (2^%d): %llu  first 0x%08x\n", e, e - 127, cnt[c * 256 + e], first[c * 256 + e]);
    }
    return 0;
}
