// wf_sort_cost.hip — what a global coherence sort of the wavefront's extend queue costs on MI355X
// ("a key-only global sort of the extend queue").  One iteration of config 5 (blob70k
// 1080p/64 spp, every path in flight) holds up to N = 132.7 M paths in the queue layout of
// hippt_wavefront.hip (three float4 arrays, 48 B per path).  A global sort needs, per iteration:
//   sort   rocprim::radix_sort_pairs of (15-bit key: direction octant + 4x4x4 origin cell... here
//          random keys of that width) and the entry index, over the queue;
//   gather the extend kernel (or a copy pass) reading each path's 48 B through the sorted index.
// The program times both with HIP events for n = N, N/2, N/4 and prints one JSON line per size;
// their sum over config 5's iterations is the least a global sort adds to a step.
#include <hip/hip_runtime.h>
#include <cstring>
#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/iterator/counting_iterator.hpp>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHECK(x)                                                                              \
    do {                                                                                      \
        hipError_t e_ = (x);                                                                  \
        if (e_ != hipSuccess) {                                                               \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                     \
            std::exit(1);                                                                     \
        }                                                                                     \
    } while (0)

__global__ void init_keys(unsigned short *k, unsigned n, unsigned bits) {
    for (unsigned i = blockIdx.x * 256u + threadIdx.x; i < n; i += gridDim.x * 256u) {
        unsigned h = i * 2654435761u;
        h ^= h >> 15;
        h *= 2246822519u;
        h ^= h >> 13;
        k[i] = (unsigned short)(h & ((1u << bits) - 1u));
    }
}

__global__ void fill(float4 *a, unsigned n) {
    for (unsigned i = blockIdx.x * 256u + threadIdx.x; i < n; i += gridDim.x * 256u)
        a[i] = make_float4(float(i), 1.0f, 2.0f, 3.0f);
}

// the sorted order's 48-byte paths into a queue of their own, coalesced writes
__global__ void gather(const unsigned *idx, const float4 *ra, const float4 *rb, const float4 *rc, float4 *da,
                       float4 *db, float4 *dc, unsigned n) {
    for (unsigned j = blockIdx.x * 256u + threadIdx.x; j < n; j += gridDim.x * 256u) {
        const unsigned s = idx[j];
        da[j] = ra[s];
        db[j] = rb[s];
        dc[j] = rc[s];
    }
}

// the same copy in queue order (no sort): the pass's floor
__global__ void copy_in_order(const float4 *ra, const float4 *rb, const float4 *rc, float4 *da, float4 *db,
                              float4 *dc, unsigned n) {
    for (unsigned j = blockIdx.x * 256u + threadIdx.x; j < n; j += gridDim.x * 256u) {
        da[j] = ra[j];
        db[j] = rb[j];
        dc[j] = rc[j];
    }
}

int main() {
    const unsigned N = 1920u * 1080u * 64u;
    const unsigned bits = 15;
    int cus = 0;
    CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    const unsigned grid = unsigned(cus) * 16;
    unsigned short *k0, *k1;
    unsigned *v1;
    float4 *q[6];
    CHECK(hipMalloc(&k0, size_t(N) * 2));
    CHECK(hipMalloc(&k1, size_t(N) * 2));
    CHECK(hipMalloc(&v1, size_t(N) * 4));
    for (auto &p : q) CHECK(hipMalloc(&p, size_t(N) * 16));
    for (int i = 0; i < 3; ++i) hipLaunchKernelGGL(fill, dim3(grid), dim3(256), 0, 0, q[i], N);
    size_t tmpBytes = 0;
    rocprim::counting_iterator<unsigned> iota(0u);
    CHECK(rocprim::radix_sort_pairs(nullptr, tmpBytes, k0, k1, iota, v1, N, 0, bits));
    void *tmp = nullptr;
    CHECK(hipMalloc(&tmp, tmpBytes));
    hipEvent_t e[4];
    for (auto &x : e) CHECK(hipEventCreate(&x));
    for (unsigned n : {N, N / 2, N / 4}) {
        float sortMs = 0, gatherMs = 0, copyMs = 0;
        for (int rep = 0; rep < 4; ++rep) {  // rep 0 warms up
            hipLaunchKernelGGL(init_keys, dim3(grid), dim3(256), 0, 0, k0, n, bits);
            CHECK(hipEventRecord(e[0]));
            CHECK(rocprim::radix_sort_pairs(tmp, tmpBytes, k0, k1, iota, v1, n, 0, bits));
            CHECK(hipEventRecord(e[1]));
            hipLaunchKernelGGL(gather, dim3(grid), dim3(256), 0, 0, v1, q[0], q[1], q[2], q[3], q[4], q[5], n);
            CHECK(hipEventRecord(e[2]));
            hipLaunchKernelGGL(copy_in_order, dim3(grid), dim3(256), 0, 0, q[0], q[1], q[2], q[3], q[4], q[5], n);
            CHECK(hipEventRecord(e[3]));
            CHECK(hipEventSynchronize(e[3]));
            float a, b, c;
            CHECK(hipEventElapsedTime(&a, e[0], e[1]));
            CHECK(hipEventElapsedTime(&b, e[1], e[2]));
            CHECK(hipEventElapsedTime(&c, e[2], e[3]));
            if (rep) {
                sortMs += a / 3;
                gatherMs += b / 3;
                copyMs += c / 3;
            }
        }
        std::printf("{\"paths\": %u, \"key_bits\": %u, \"sort_ms\": %.4f, \"gather_ms\": %.4f, \"copy_in_order_ms\": %.4f}\n",
                    n, bits, sortMs, gatherMs, copyMs);
    }
    CHECK(hipGetLastError());
    return 0;
}
