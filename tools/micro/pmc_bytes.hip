// pmc_bytes.hip — calibration of rocprofv3's FETCH_SIZE / WRITE_SIZE on gfx950 for the access
// widths the path tracer uses (MI355X_MICROARCH.md §HBM: FETCH_SIZE reads half the
// bytes of a 16-B/lane streaming read, WRITE_SIZE exact for 16-B/lane streaming stores, other widths
// uncalibrated).  Every kernel moves a known byte count through buffers of 1 GiB each (4x the
// 256 MiB Infinity Cache, so that nothing is served on-die), one dispatch per pattern:
//   st_f3    12-B/lane stores, consecutive lanes consecutive items (mesh_kernel's store_radiance)
//   ld_f3    12-B/lane loads of the same layout (combine_pixel's scratch reads)
//   ld_f3_fr the combine's frame loop: 12-B/lane loads, item fl * bandPixels + p for fl = 0..63
//   ld_f4    16-B/lane loads (the guide's calibrated case)
//   st_f4    16-B/lane stores (the guide's calibrated case)
//   rmw_f4   a float4 read and written per lane (the accumulation update)
//   ld_row   16-B loads of rows of scattered 128-B nodes, one node per lane (a BVH node row read
//            from global memory): one distinct 128-B line per lane
// The program prints one JSON line per kernel (name, bytes moved); tools/micro/pmc_bytes.py joins
// them with the rocprofv3 counter CSVs into per-width factors (bytes / counter bytes).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CHECK(x)                                                                              \
    do {                                                                                      \
        hipError_t e_ = (x);                                                                  \
        if (e_ != hipSuccess) {                                                               \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                     \
            std::exit(1);                                                                     \
        }                                                                                     \
    } while (0)

constexpr size_t kBytes = size_t(1) << 30;

__global__ __launch_bounds__(256) void st_f3(float *dst, unsigned n) {
    for (unsigned i = blockIdx.x * 256u + threadIdx.x; i < n; i += gridDim.x * 256u)
        *reinterpret_cast<float3 *>(dst + 3 * size_t(i)) = make_float3(float(i), 1.0f, 2.0f);
}

__global__ __launch_bounds__(256) void ld_f3(const float *src, unsigned n, float *out) {
    float a = 0.0f;
    for (unsigned i = blockIdx.x * 256u + threadIdx.x; i < n; i += gridDim.x * 256u) {
        const float3 v = *reinterpret_cast<const float3 *>(src + 3 * size_t(i));
        a += v.x + v.y + v.z;
    }
    if (a == 12345.0f) out[0] = a;
}

// pixels p < px, frames fl < 64: item fl * px + p (every item once, frame-major per pixel)
__global__ __launch_bounds__(256) void ld_f3_fr(const float *src, unsigned px, float *out) {
    float a = 0.0f;
    for (unsigned p = blockIdx.x * 256u + threadIdx.x; p < px; p += gridDim.x * 256u)
        for (unsigned fl = 0; fl < 64; ++fl) {
            const float3 v = *reinterpret_cast<const float3 *>(src + 3 * (size_t(fl) * px + p));
            a = fmaf(a, 0.5f, v.x + v.y + v.z);
        }
    if (a == 12345.0f) out[0] = a;
}

__global__ __launch_bounds__(256) void ld_f4(const float4 *src, unsigned n, float *out) {
    float a = 0.0f;
    for (unsigned i = blockIdx.x * 256u + threadIdx.x; i < n; i += gridDim.x * 256u) {
        const float4 v = src[i];
        a += v.x + v.y + v.z + v.w;
    }
    if (a == 12345.0f) out[0] = a;
}

__global__ __launch_bounds__(256) void st_f4(float4 *dst, unsigned n) {
    for (unsigned i = blockIdx.x * 256u + threadIdx.x; i < n; i += gridDim.x * 256u)
        dst[i] = make_float4(float(i), 1.0f, 2.0f, 3.0f);
}

__global__ __launch_bounds__(256) void rmw_f4(float4 *buf, unsigned n) {
    for (unsigned i = blockIdx.x * 256u + threadIdx.x; i < n; i += gridDim.x * 256u) {
        float4 v = buf[i];
        v.x = v.x * 0.5f + 1.0f;
        buf[i] = v;
    }
}

// lane i reads the first 16-B row of node 8i (128-B nodes, 1 KiB apart): one distinct 128-B line
// per lane, each read once
__global__ __launch_bounds__(256) void ld_row(const float4 *nodes, unsigned reads, float *out) {
    float a = 0.0f;
    for (unsigned i = blockIdx.x * 256u + threadIdx.x; i < reads; i += gridDim.x * 256u) {
        const float4 v = nodes[size_t(i) * 64];
        a += v.x + v.w;
    }
    if (a == 12345.0f) out[0] = a;
}

int main() {
    int cus = 0;
    CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    const unsigned grid = unsigned(cus) * 8;
    float *a = nullptr, *b = nullptr, *out = nullptr;
    CHECK(hipMalloc(&a, kBytes));
    CHECK(hipMalloc(&b, kBytes));
    CHECK(hipMalloc(&out, 64));
    CHECK(hipMemset(a, 0, kBytes));
    CHECK(hipMemset(b, 0, kBytes));
    CHECK(hipDeviceSynchronize());
    const unsigned n3 = unsigned(kBytes / 12), n4 = unsigned(kBytes / 16);
    const unsigned px = n3 / 64;                 // ld_f3_fr: px pixels x 64 frames
    auto line = [](const char *k, double bytes, const char *what) {
        std::printf("{\"kernel\": \"%s\", \"bytes\": %.0f, \"what\": \"%s\"}\n", k, bytes, what);
    };
    hipLaunchKernelGGL(st_f3, dim3(grid), dim3(256), 0, 0, a, n3);
    line("st_f3", 12.0 * n3, "12-B/lane coalesced stores");
    hipLaunchKernelGGL(ld_f3, dim3(grid), dim3(256), 0, 0, a, n3, out);
    line("ld_f3", 12.0 * n3, "12-B/lane coalesced loads");
    hipLaunchKernelGGL(ld_f3_fr, dim3(grid), dim3(256), 0, 0, a, px, out);
    line("ld_f3_fr", 12.0 * 64 * px, "12-B/lane loads, 64 frames per pixel (combine)");
    hipLaunchKernelGGL(ld_f4, dim3(grid), dim3(256), 0, 0, reinterpret_cast<const float4 *>(b), n4, out);
    line("ld_f4", 16.0 * n4, "16-B/lane coalesced loads");
    hipLaunchKernelGGL(st_f4, dim3(grid), dim3(256), 0, 0, reinterpret_cast<float4 *>(b), n4);
    line("st_f4", 16.0 * n4, "16-B/lane coalesced stores");
    hipLaunchKernelGGL(rmw_f4, dim3(grid), dim3(256), 0, 0, reinterpret_cast<float4 *>(b), n4);
    line("rmw_f4", 32.0 * n4, "float4 read + write per lane");
    const unsigned reads = unsigned(kBytes / 1024);
    hipLaunchKernelGGL(ld_row, dim3(grid), dim3(256), 0, 0, reinterpret_cast<const float4 *>(a), reads, out);
    line("ld_row", 128.0 * reads, "scattered 16-B node rows, one 128-B line each (bytes = 128 per line)");
    CHECK(hipGetLastError());
    CHECK(hipDeviceSynchronize());
    CHECK(hipFree(a));
    CHECK(hipFree(b));
    CHECK(hipFree(out));
    return 0;
}
