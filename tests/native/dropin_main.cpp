// dropin_main.cpp — TEST INFRASTRUCTURE (tests/test_dropin_reference.py).  A minimal caller of the
// reference's UNMODIFIED src/backends/CudaPathTracer.{h,cpp} (compiled from /root/reference with
// -DENABLE_CUDA_BACKEND against Qt 5 QtCore), linked against libhippt.so instead of the CUDA
// kernel: proves the drop-in at the link and call level (CudaPathTracer.cpp:4-8,20-57).
#include <cstdio>

#include "CudaPathTracer.h"

extern "C" const char *hipptLastError(void);

int main() {
    CudaPathTracer tracer;
    const bool ok = tracer.initialize(64, 48);
    std::printf("init=%d\n", ok ? 1 : 0);
    std::printf("lastError=%s\n", tracer.lastError().toUtf8().constData());
    std::printf("libError=%s\n", hipptLastError());
    if (ok) {
        bool r = true;
        for (int f = 0; f < 3 && r; ++f) r = tracer.renderFrame(8);
        std::printf("render=%d frames=%d pixels=%d\n", r ? 1 : 0, tracer.frameIndex(), tracer.hostPixels() ? 1 : 0);
        if (r) std::printf("pixel0=%u\n", tracer.hostPixels()[0]);
    }
    return 0;
}
