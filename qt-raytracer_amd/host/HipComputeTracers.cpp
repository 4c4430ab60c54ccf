// HipComputeTracers.cpp — see HipComputeTracers.h.
#include "HipComputeTracers.h"

#include <algorithm>

namespace {

// The GL / Vulkan shaders clamp the bounce count (GpuPathTracer.cpp:57, VulkanPathTracer.cpp:95)
int clamp_depth(int maxDepth) { return std::clamp(maxDepth, 1, 64); }

// A blocking render of RGBA8 words; the process-wide pixel format is restored afterwards, so other
// hipptRenderFrames* callers in the process keep theirs (the render has combined and copied its
// frames before it returns: nothing pending still reads the option).
bool rgba8_frames(int first, int count, int maxDepth, const unsigned int **pixels, std::string &error) {
    const char *err = nullptr;
    const long long saved = hipptGetOption(HIPPT_OPT_PIXEL_FORMAT);
    const bool ok = hipptSetOption(HIPPT_OPT_PIXEL_FORMAT, HIPPT_PIXEL_RGBA8) &&
                    hipptRenderFrames(first, count, maxDepth, pixels, &err);
    hipptSetOption(HIPPT_OPT_PIXEL_FORMAT, saved);
    if (!ok) {
        error = err ? err : "HIP render failed";
        return false;
    }
    return true;
}

}  // namespace

// ---- VulkanPathTracer interface ----------------------------------------------------------------

HipVulkanPathTracer::~HipVulkanPathTracer() {
    if (m_ready) cudaPathTracerShutdown();
}

bool HipVulkanPathTracer::initialize(int width, int height) {
    // VulkanPathTracer.cpp:67-81: the size and a zero frame index first, then the device side
    m_width = width;
    m_height = height;
    m_frameIndex = 0;
    m_hostPixels = nullptr;
    const char *err = nullptr;
    m_ready = cudaPathTracerInit(width, height, &err);
    if (!m_ready) {
        m_lastError = err ? err : "HIP initialization failed";
        return false;
    }
    // hostPixels() holds the cleared frame until the first render (the zeroed m_hostOutput, :71)
    if (!rgba8_frames(0, 0, 1, &m_hostPixels, m_lastError)) return m_ready = false;
    return true;
}

bool HipVulkanPathTracer::renderFrame(int maxDepth) {
    if (!m_ready) {  // VulkanPathTracer.cpp:85-88
        m_lastError = "HIP compute is not initialized";
        return false;
    }
    if (!rgba8_frames(m_frameIndex, 1, clamp_depth(maxDepth), &m_hostPixels, m_lastError)) return false;
    ++m_frameIndex;  // :257
    return true;
}

// ---- GpuPathTracer interface -------------------------------------------------------------------

HipGpuPathTracer::~HipGpuPathTracer() { release(); }

bool HipGpuPathTracer::initialize() {
    // GpuPathTracer.cpp:14-37 needs a current GL 4.3 context; this backend needs a HIP device
    if (hipptDeviceCount() < 1) {
        m_lastError = "No HIP device";
        return false;
    }
    m_ready = true;
    return true;
}

bool HipGpuPathTracer::resize(int width, int height) {
    if (width <= 0 || height <= 0) return false;  // :38-41
    if (m_sized && m_width == width && m_height == height) return true;
    m_width = width;
    m_height = height;
    m_frameIndex = 0;
    m_hostPixels = nullptr;
    const char *err = nullptr;
    m_sized = cudaPathTracerInit(width, height, &err);  // new, cleared images (ensureTextures)
    if (!m_sized) {
        m_lastError = err ? err : "HIP initialization failed";
        return false;
    }
    return rgba8_frames(0, 0, 1, &m_hostPixels, m_lastError);
}

bool HipGpuPathTracer::renderFrame(int samplesPerFrame, int maxDepth) {
    if (!m_ready || !m_sized) return false;  // :53-55
    samplesPerFrame = std::max(1, samplesPerFrame);
    if (!rgba8_frames(m_frameIndex, samplesPerFrame, clamp_depth(maxDepth), &m_hostPixels, m_lastError)) return false;
    m_frameIndex += samplesPerFrame;  // one dispatch per sample, each advancing the index (:68-74)
    return true;
}

void HipGpuPathTracer::resetAccumulation() {
    m_frameIndex = 0;  // :85-95
    if (!m_sized) return;
    const char *err = nullptr;
    if (!hipptResetAccumulation(&err)) m_lastError = err ? err : "HIP reset failed";
}

void HipGpuPathTracer::release() {
    if (m_sized) cudaPathTracerShutdown();
    m_sized = false;
    m_ready = false;
    m_hostPixels = nullptr;
}
