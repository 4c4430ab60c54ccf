// Probe: does a kernel on stream B, gated by hipStreamWaitValue32 on a word that a still-running
// kernel on stream A raises at its "drain", start while A's tail runs (its blocks taking the slots
// A's exiting blocks free), for three kinds of flag memory?  A's waves all finish their main part at
// ~base us and one wave in 8 runs a tail of `tail` us more; the first wave to finish its main part
// raises the flag (plus a stream-ordered hipStreamWriteValue32 after A as the backstop).  Prints A's
// flag time, A's end and B's first block start, in us from A's first block start.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                                \
    do {                                                                                     \
        hipError_t e_ = (x);                                                                 \
        if (e_ != hipSuccess) {                                                              \
            std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            std::exit(2);                                                                    \
        }                                                                                    \
    } while (0)

__device__ unsigned long long rt() { return __builtin_amdgcn_s_memrealtime(); }

// t[0] min start, t[1] first flag time, t[2] max end (A); t[3] min start (B)
__global__ __launch_bounds__(256) void kernA(unsigned *flag, unsigned ticket, unsigned long long *t, unsigned base,
                                             unsigned tail) {
    extern __shared__ int lds[];
    const unsigned long long s = rt();
    if (threadIdx.x == 0) atomicMin(&t[0], s);
    lds[threadIdx.x] = threadIdx.x;
    const unsigned wave = blockIdx.x * 4 + threadIdx.x / 64;
    while (rt() - s < base * 100ull) __builtin_amdgcn_s_sleep(2);
    if ((threadIdx.x & 63) == 0) {
        const unsigned long long f = rt();
        atomicMin(&t[1], f);
        __hip_atomic_fetch_max(flag, ticket, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    if (wave % 8 == 0)
        while (rt() - s < (base + tail) * 100ull) __builtin_amdgcn_s_sleep(2);
    if ((threadIdx.x & 63) == 0) atomicMax(&t[2], rt());
    if (lds[(threadIdx.x + 1) & 255] == 12345) t[4] = 1;
}

__global__ __launch_bounds__(256) void kernB(unsigned long long *t) {
    extern __shared__ int lds[];
    const unsigned long long s = rt();
    if (threadIdx.x == 0) atomicMin(&t[3], s);
    lds[threadIdx.x] = 1;
    while (rt() - s < 2000ull) __builtin_amdgcn_s_sleep(2);
    if (lds[(threadIdx.x + 1) & 255] == 12345) t[4] = 1;
}

int main(int argc, char **argv) {
    const unsigned base = argc > 1 ? unsigned(std::atoi(argv[1])) : 300, tail = argc > 2 ? unsigned(std::atoi(argv[2])) : 200;
    int canWait = 0, cus = 0;
    CK(hipDeviceGetAttribute(&canWait, hipDeviceAttributeCanUseStreamWaitValue, 0));
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    std::printf("{\"can_wait_value\": %d, \"cus\": %d}\n", canWait, cus);
    hipStream_t a, b;
    CK(hipStreamCreateWithFlags(&a, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&b, hipStreamNonBlocking));
    unsigned long long *t;
    CK(hipMalloc(&t, 8 * sizeof(unsigned long long)));
    const size_t ldsBytes = 64 * 1024;  // 2 blocks per CU
    const int blocks = cus * 2;
    for (int kind = 0; kind < 3; ++kind) {
        unsigned *flag = nullptr;
        if (kind == 0) CK(hipExtMallocWithFlags(reinterpret_cast<void **>(&flag), 8, hipMallocSignalMemory));
        if (kind == 1) CK(hipMalloc(&flag, 256));
        if (kind == 2) CK(hipHostMalloc(reinterpret_cast<void **>(&flag), 256, hipHostMallocCoherent));
        const char *name = kind == 0 ? "signal" : kind == 1 ? "device" : "host_coherent";
        if (kind != 2) CK(hipMemset(flag, 0, kind == 0 ? 8 : 256));
        else flag[0] = 0;
        CK(hipDeviceSynchronize());
        for (unsigned rep = 1; rep <= 3; ++rep) {
            unsigned long long init[8] = {~0ull, ~0ull, 0, ~0ull, 0, 0, 0, 0};
            CK(hipMemcpy(t, init, sizeof(init), hipMemcpyHostToDevice));
            const unsigned ticket = rep;
            hipLaunchKernelGGL(kernA, dim3(blocks), dim3(256), ldsBytes, a, flag, ticket, t, base, tail);
            CK(hipGetLastError());
            CK(hipStreamWriteValue32(a, flag, ticket, 0));
            CK(hipStreamWaitValue32(b, flag, ticket, hipStreamWaitValueGte, 0xffffffffu));
            hipLaunchKernelGGL(kernB, dim3(blocks), dim3(256), ldsBytes, b, t);
            CK(hipGetLastError());
            CK(hipDeviceSynchronize());
            unsigned long long r[8];
            CK(hipMemcpy(r, t, sizeof(r), hipMemcpyDeviceToHost));
            const double us = 0.01;
            std::printf("{\"flag\": \"%s\", \"rep\": %u, \"a_flag_us\": %.1f, \"a_end_us\": %.1f, \"b_start_us\": %.1f}\n",
                        name, rep, (r[1] - r[0]) * us, (r[2] - r[0]) * us, (double(r[3]) - double(r[0])) * us);
        }
        if (kind == 0 || kind == 1) CK(hipFree(flag));
        else CK(hipHostFree(flag));
    }
    return 0;
}
