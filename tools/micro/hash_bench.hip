// hash_bench.hip — throughput of the hash RNG's 32-bit multiply forms on gfx950 (experiment).
// Each thread runs a dependent chain of hashes; 4 independent chains per thread for ILP.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__device__ __forceinline__ uint32_t mul_lo(uint32_t x, uint32_t c) { return x * c; }

// x * c mod 2^32 from 16-bit halves with full-rate 24-bit multiplies
__device__ __forceinline__ uint32_t mul_split(uint32_t x, uint32_t c) {
    const uint32_t xl = x & 0xffffu, xh = x >> 16, cl = c & 0xffffu, ch = c >> 16;
    uint32_t lo, m1, mid;
    asm volatile("v_mul_u32_u24 %0, %1, %2" : "=v"(lo) : "v"(xl), "v"(cl));
    asm volatile("v_mul_u32_u24 %0, %1, %2" : "=v"(m1) : "v"(xl), "v"(ch));
    asm volatile("v_mad_u32_u24 %0, %1, %2, %3" : "=v"(mid) : "v"(xh), "v"(cl), "v"(m1));
    return lo + (mid << 16);
}

template <int MODE>
__device__ __forceinline__ uint32_t hash(uint32_t x) {
    x ^= x >> 16;
    x = MODE ? mul_split(x, 0x7feb352du) : mul_lo(x, 0x7feb352du);
    x ^= x >> 15;
    x = MODE ? mul_split(x, 0x846ca68bu) : mul_lo(x, 0x846ca68bu);
    x ^= x >> 16;
    return x;
}

template <int MODE>
__global__ void bench(uint32_t *out, int iters) {
    uint32_t a = blockIdx.x * 256 + threadIdx.x, b = a ^ 0x1234567u, c = a * 3u + 7u, d = ~a;
    for (int i = 0; i < iters; ++i) {
        a = hash<MODE>(a);
        b = hash<MODE>(b);
        c = hash<MODE>(c);
        d = hash<MODE>(d);
    }
    out[blockIdx.x * 256 + threadIdx.x] = a ^ b ^ c ^ d;
}

int main() {
    const int blocks = 256 * 32, iters = 4096;
    uint32_t *out;
    hipMalloc(&out, blocks * 256 * 4);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    uint32_t *h0 = new uint32_t[blocks * 256], *h1 = new uint32_t[blocks * 256];
    for (int mode = 0; mode < 2; ++mode) {
        for (int rep = 0; rep < 2; ++rep) {
            hipEventRecord(e0);
            if (mode == 0) hipLaunchKernelGGL(bench<0>, dim3(blocks), dim3(256), 0, 0, out, iters);
            else hipLaunchKernelGGL(bench<1>, dim3(blocks), dim3(256), 0, 0, out, iters);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            const double hashes = double(blocks) * 256 * iters * 4;
            if (rep == 1) printf("mode %d (%s): %.3f ms, %.1f Ghash/s\n", mode, mode ? "24-bit split" : "mul_lo_u32", ms,
                                 hashes / ms / 1e6);
        }
        hipMemcpy(mode ? h1 : h0, out, blocks * 256 * 4, hipMemcpyDeviceToHost);
    }
    int diff = 0;
    for (int i = 0; i < blocks * 256; ++i) diff += h0[i] != h1[i];
    printf("results differ in %d of %d\n", diff, blocks * 256);
    return 0;
}
