// rn_selftest.hip — test helper (not product code): checks the kernels' short correctly-rounded
// sequences (qt-raytracer_amd/csrc/hippt_trace.h sqrt_fix, rcp_nr, rsqrt_rn, rsqrt_unit_draw)
// against hipcc's IEEE sqrtf / 1.0f/x on every float bit pattern, on the GPU.  Used by
// tests/test_gpu_rounding.py through ctypes.
#include <hip/hip_runtime.h>

#include "hippt_trace.h"

#pragma clang fp contract(off)

using namespace hippt::trace;

namespace {

__device__ __forceinline__ bool same(float a, float b) {
    return __float_as_uint(a) == __float_as_uint(b) || (a != a && b != b);
}

// counts[k]: mismatches of check k inside its claimed domain
//   0 rsqrt_rn(x)        == 1/sqrtf(x)   every x
//   1 rsqrt_unit_draw(x) == 1/sqrtf(x)   x = +0 or 2^-48 <= x < 1 (a sum of squares is never -0)
//   2 sqrt_fix(x)        == sqrtf(x)     x >= 2^-104
//   3 rcp_nr(x)          == 1.0f/x       2^-126 <= |x| < 2^126
__global__ __launch_bounds__(256) void check(unsigned long long *counts, unsigned long long base, unsigned long long n) {
    unsigned c[4] = {0, 0, 0, 0};
    for (unsigned long long i = blockIdx.x * 256ull + threadIdx.x; i < n; i += gridDim.x * 256ull) {
        const unsigned u = unsigned(base + i);
        const float x = __uint_as_float(u);
        const float ax = fabsf(x);
        const float isq = 1.0f / sqrtf(x);
        c[0] += !same(rsqrt_rn(x), isq);
        if (u == 0u || (x >= 0x1p-48f && x < 1.0f)) c[1] += !same(rsqrt_unit_draw(x), isq);
        if (x >= 0x1p-104f) c[2] += !same(sqrt_fix(x), sqrtf(x));
        if (ax >= 0x1p-126f && ax < 0x1p126f) c[3] += !same(rcp_nr(x), 1.0f / x);
    }
    for (int k = 0; k < 4; ++k)
        if (c[k]) atomicAdd(&counts[k], (unsigned long long)c[k]);
}

}  // namespace

extern "C" int rn_selftest(unsigned long long *hostCounts) {
    unsigned long long *d = nullptr;
    if (hipMalloc(&d, 4 * sizeof(unsigned long long)) != hipSuccess) return 1;
    (void)hipMemset(d, 0, 4 * sizeof(unsigned long long));
    const unsigned long long chunk = 1ull << 28;
    for (unsigned long long b = 0; b < (1ull << 32); b += chunk)
        hipLaunchKernelGGL(check, dim3(8192), dim3(256), 0, 0, d, b, chunk);
    const bool ok = hipDeviceSynchronize() == hipSuccess &&
                    hipMemcpy(hostCounts, d, 4 * sizeof(unsigned long long), hipMemcpyDeviceToHost) == hipSuccess;
    (void)hipFree(d);
    return ok ? 0 : 2;
}
