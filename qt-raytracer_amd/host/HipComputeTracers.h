// HipComputeTracers.h — the reference's two other GPU backend interfaces over libhippt.so's
// C ABI, so the Qt viewport's "vulkan" and GL compute branches can run on an MI355X unchanged
// apart from the class name.
//
//   HipVulkanPathTracer  VulkanPathTracer (src/backends/vulkan/VulkanPathTracer.h:7-16):
//                        initialize(w, h), renderFrame(maxDepth) = one frame at the current
//                        index (maxDepth clamped to 1..64, VulkanPathTracer.cpp:95), then the
//                        index advances; hostPixels() = the library-owned RGBA8 UNORM frame
//                        (bytes R, G, B, A, as the Vulkan staging copy, :252-255).
//   HipGpuPathTracer     GpuPathTracer (src/backends/GpuPathTracer.h:9-25): initialize(),
//                        resize(w, h) (a new size restarts the frame count, :38-50),
//                        renderFrame(samplesPerFrame, maxDepth) (samplesPerFrame >= 1 frames,
//                        maxDepth clamped to 1..64, :52-83), resetAccumulation() (:85-95), the
//                        accessors.  outputTextureId() becomes hostPixels(): the RGBA8 UNORM
//                        texels the GL_RGBA8 output image holds, which the GL host uploads with
//                        glTexSubImage2D (no GL context exists in this build).
//
// Both render the reference GPU kernels' built-in 4-sphere scene by default (the same one the
// GL and Vulkan shaders hard-code) or any uploaded scene (HipPathTracer's scene calls apply:
// the library holds one scene).  Qt-free: std::string instead of QString.
#pragma once

#include <string>

#include "hippt.h"

class HipVulkanPathTracer {
public:
    HipVulkanPathTracer() = default;
    ~HipVulkanPathTracer();
    HipVulkanPathTracer(const HipVulkanPathTracer &) = delete;
    HipVulkanPathTracer &operator=(const HipVulkanPathTracer &) = delete;

    bool initialize(int width, int height);
    bool renderFrame(int maxDepth);
    const unsigned int *hostPixels() const { return m_hostPixels; }
    int frameIndex() const { return m_frameIndex; }
    std::string lastError() const { return m_lastError; }

private:
    int m_width = 0;
    int m_height = 0;
    int m_frameIndex = 0;
    bool m_ready = false;
    const unsigned int *m_hostPixels = nullptr;
    std::string m_lastError;
};

class HipGpuPathTracer {
public:
    HipGpuPathTracer() = default;
    ~HipGpuPathTracer();
    HipGpuPathTracer(const HipGpuPathTracer &) = delete;
    HipGpuPathTracer &operator=(const HipGpuPathTracer &) = delete;

    bool initialize();
    bool resize(int width, int height);
    bool renderFrame(int samplesPerFrame, int maxDepth);
    void resetAccumulation();
    bool isReady() const { return m_ready; }
    const unsigned int *hostPixels() const { return m_hostPixels; }
    int width() const { return m_width; }
    int height() const { return m_height; }
    int frameIndex() const { return m_frameIndex; }
    std::string lastError() const { return m_lastError; }
    void release();

private:
    int m_width = 0;
    int m_height = 0;
    int m_frameIndex = 0;
    bool m_ready = false;
    bool m_sized = false;
    const unsigned int *m_hostPixels = nullptr;
    std::string m_lastError;
};
