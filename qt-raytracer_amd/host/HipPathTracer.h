// HipPathTracer.h — C++ host object over libhippt.so's C ABI (include/hippt.h).
//
// Same public interface and frame-index bookkeeping as the reference's CudaPathTracer
// (src/backends/CudaPathTracer.h:6-23, CudaPathTracer.cpp:14-57): initialize(w, h) re-inits and
// restarts the frame count, renderFrame(maxDepth) renders one sample per pixel for the current
// frame index and advances it, hostPixels() is the library-owned ARGB frame (row 0 = bottom),
// lastError() the last message.  Qt-free (std::string instead of QString) so it builds and runs
// without Qt; RayTracerFboItem's "hip" backend string constructs it exactly like
// m_cudaTracer.  Extensions: scenes, batched frames, non-blocking hand-off.
#pragma once

#include <string>
#include <vector>

#include "hippt.h"

class HipPathTracer {
public:
    HipPathTracer() = default;
    ~HipPathTracer();
    HipPathTracer(const HipPathTracer &) = delete;
    HipPathTracer &operator=(const HipPathTracer &) = delete;

    // --- CudaPathTracer interface -------------------------------------------------------------
    bool initialize(int width, int height);
    bool renderFrame(int maxDepth);
    const unsigned int *hostPixels() const { return m_hostPixels; }
    int frameIndex() const { return m_frameIndex; }
    std::string lastError() const { return m_lastError; }

    // --- extensions ----------------------------------------------------------------------------
    // Triangle mesh from an OBJ/PLY file, one Lambertian material per group (albedo: 3 floats per
    // group; empty = white 0.73), camera as RayTracer.h Camera parameters.
    bool loadMeshFile(const std::string &path, const std::vector<float> &albedo, const double lookfrom[3],
                      const double lookat[3], const double vup[3], double vfovDeg, double aperture, double focus);
    bool uploadScene(const std::vector<float> &verts, const std::vector<int> &triMaterial,
                     const std::vector<float> &spheres, const std::vector<int> &sphereMaterial,
                     const std::vector<hipptMaterial> &materials, const double lookfrom[3], const double lookat[3],
                     const double vup[3], double vfovDeg, double aperture, double focus);
    bool useBuiltinScene();  // the reference kernel's 4 spheres (the default)
    // samplesPerFrame frames in one call (GpuPathTracer::renderFrame(spp, depth) shape).
    bool renderFrames(int samplesPerFrame, int maxDepth);
    // Enqueue frames + copy to a hand-off frame; latestFrame() never blocks.
    bool presentFrames(int samplesPerFrame, int maxDepth);
    const unsigned int *latestFrame(int *frames);
    bool setOption(int key, long long value);

private:
    bool fail(const char *err, const char *fallback);

    int m_width = 0;
    int m_height = 0;
    int m_frameIndex = 0;
    const unsigned int *m_hostPixels = nullptr;
    std::string m_lastError;
};
