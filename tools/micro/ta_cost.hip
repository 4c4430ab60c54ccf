// ta_cost.hip — vector-memory address-unit (TA) cost of global loads on gfx950 (experiment):
// L2-resident buffer, many independent loads per lane; per-lane addresses scattered (each lane
// its own 64-B line), coalesced (consecutive lanes consecutive elements) or wave-uniform.
// Prints cycles per wave-load instruction per CU at the measured rate.  ACTIVE: lanes that take
// part (the others are masked off around the load), to see whether the TA's cost follows the
// exec mask or the instruction.
#include <hip/hip_runtime.h>
#include <cstdio>

template <typename T, int PATTERN, int ACTIVE = 64>
__global__ __launch_bounds__(256) void k(const T *buf, unsigned mask, float *out, int iters) {
    float acc = 0.0f;
    const unsigned lane = threadIdx.x & 63u;
    unsigned base = (blockIdx.x * 977u + (threadIdx.x >> 6) * 131u) * 64u;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            unsigned e;
            const unsigned step = base + unsigned(it * 8 + u) * 4099u;
            if (PATTERN == 0) e = (step + lane * 67u) & mask;        // scattered: one line per lane (64 B stride units)
            else if (PATTERN == 1) e = (step * 64u + lane) & mask;   // coalesced
            else e = step & mask;                                     // uniform
            if (ACTIVE == 64 || lane < unsigned(ACTIVE)) {
                const T v = buf[e];
                acc += *reinterpret_cast<const float *>(&v);
            }
        }
    }
    out[blockIdx.x * 256 + threadIdx.x] = acc;
}

template <typename T, int P, int A = 64>
void run(const char *name, void *buf, unsigned elems, float *out, int cus, double ghz) {
    const int blocks = cus * 8, iters = 512;
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    float ms = 0;
    for (int rep = 0; rep < 3; ++rep) {
        (void)hipEventRecord(a);
        k<T, P, A><<<blocks, 256>>>((const T *)buf, elems - 1, out, iters);
        (void)hipEventRecord(b);
        (void)hipEventSynchronize(b);
        (void)hipEventElapsedTime(&ms, a, b);
    }
    const double waveLoads = double(blocks) * 4 * iters * 8;
    const double perCu = waveLoads / cus;
    printf("%-22s %8.3f ms  %6.2f cycles/wave-load/CU  %7.1f GB/s\n", name, ms, ms * 1e-3 * ghz * 1e9 / perCu,
           waveLoads * 64 * sizeof(T) / (ms * 1e-3) / 1e9);
}

int main() {
    int cus = 0;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    const double ghz = 2.4;
    const unsigned bytes = 1u << 20;  // 1 MB: L2-resident
    void *buf;
    (void)hipMalloc(&buf, bytes);
    (void)hipMemset(buf, 0, bytes);
    float *out;
    (void)hipMalloc(&out, size_t(cus) * 8 * 256 * 4);
    run<float, 0>("dword scattered", buf, bytes / 4, out, cus, ghz);
    run<float2, 0>("dwordx2 scattered", buf, bytes / 8, out, cus, ghz);
    run<float3, 0>("dwordx3 scattered", buf, bytes / 12 & ~1u ? (bytes / 16) : 0, out, cus, ghz);
    run<float4, 0>("dwordx4 scattered", buf, bytes / 16, out, cus, ghz);
    run<float, 1>("dword coalesced", buf, bytes / 4, out, cus, ghz);
    run<float4, 1>("dwordx4 coalesced", buf, bytes / 16, out, cus, ghz);
    run<float4, 0, 32>("dwordx4 scattered 32", buf, bytes / 16, out, cus, ghz);
    run<float4, 0, 16>("dwordx4 scattered 16", buf, bytes / 16, out, cus, ghz);
    run<float4, 0, 4>("dwordx4 scattered 4", buf, bytes / 16, out, cus, ghz);
    run<float, 2>("dword uniform", buf, bytes / 4, out, cus, ghz);
    run<float4, 2>("dwordx4 uniform", buf, bytes / 16, out, cus, ghz);
    return 0;
}
