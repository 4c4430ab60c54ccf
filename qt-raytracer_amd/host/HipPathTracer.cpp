// HipPathTracer.cpp — see HipPathTracer.h.
#include "HipPathTracer.h"

HipPathTracer::~HipPathTracer() { cudaPathTracerShutdown(); }

bool HipPathTracer::fail(const char *err, const char *fallback) {
    m_lastError = err ? err : fallback;
    return false;
}

bool HipPathTracer::initialize(int width, int height) {
    m_width = width;
    m_height = height;
    m_frameIndex = 0;
    m_hostPixels = nullptr;
    const char *err = nullptr;
    if (!cudaPathTracerInit(width, height, &err)) return fail(err, "HIP initialization failed");
    return true;
}

bool HipPathTracer::renderFrame(int maxDepth) {
    const char *err = nullptr;
    const unsigned int *pixels = nullptr;
    if (!cudaPathTracerRender(m_frameIndex, maxDepth, &pixels, &err)) return fail(err, "HIP render failed");
    m_hostPixels = pixels;
    ++m_frameIndex;
    return true;
}

bool HipPathTracer::loadMeshFile(const std::string &path, const std::vector<float> &albedo,
                                 const double lookfrom[3], const double lookat[3], const double vup[3],
                                 double vfovDeg, double aperture, double focus) {
    hipptMesh mesh;
    const char *err = nullptr;
    if (!hipptReadMesh(path.c_str(), &mesh, &err)) return fail(err, "mesh read failed");
    std::vector<float> alb(albedo);
    if (alb.empty())
        for (int g = 0; g < mesh.numGroups; ++g) alb.insert(alb.end(), {0.73f, 0.73f, 0.73f});
    bool ok = int(alb.size()) == 3 * mesh.numGroups;
    if (!ok) {
        m_lastError = "albedo needs 3 floats per mesh group";
    } else {
        ok = hipptUploadMesh(mesh.verts, mesh.triGroup, mesh.numTris, alb.data(), mesh.numGroups, lookfrom, lookat, vup,
                             vfovDeg, aperture, focus, &err);
        if (!ok) fail(err, "mesh upload failed");
    }
    hipptFreeMesh(&mesh);
    return ok;
}

bool HipPathTracer::uploadScene(const std::vector<float> &verts, const std::vector<int> &triMaterial,
                                const std::vector<float> &spheres, const std::vector<int> &sphereMaterial,
                                const std::vector<hipptMaterial> &materials, const double lookfrom[3],
                                const double lookat[3], const double vup[3], double vfovDeg, double aperture,
                                double focus) {
    const char *err = nullptr;
    if (!hipptUploadScene(verts.data(), triMaterial.data(), int(triMaterial.size()), spheres.data(),
                          sphereMaterial.data(), int(sphereMaterial.size()), materials.data(), int(materials.size()),
                          lookfrom, lookat, vup, vfovDeg, aperture, focus, &err))
        return fail(err, "scene upload failed");
    return true;
}

bool HipPathTracer::useBuiltinScene() {
    const char *err = nullptr;
    if (!hipptUseBuiltinScene(HIPPT_SCENE_SPHERE4, &err)) return fail(err, "scene selection failed");
    return true;
}

bool HipPathTracer::renderFrames(int samplesPerFrame, int maxDepth) {
    const char *err = nullptr;
    const unsigned int *pixels = nullptr;
    if (!hipptRenderFrames(m_frameIndex, samplesPerFrame, maxDepth, &pixels, &err)) return fail(err, "HIP render failed");
    m_hostPixels = pixels;
    m_frameIndex += samplesPerFrame;
    return true;
}

bool HipPathTracer::presentFrames(int samplesPerFrame, int maxDepth) {
    const char *err = nullptr;
    if (!hipptRenderFramesPresent(m_frameIndex, samplesPerFrame, maxDepth, &err)) return fail(err, "HIP render failed");
    m_frameIndex += samplesPerFrame;
    return true;
}

const unsigned int *HipPathTracer::latestFrame(int *frames) {
    const char *err = nullptr;
    const unsigned int *pixels = nullptr;
    if (!hipptLatestFrame(&pixels, frames, &err)) {
        fail(err, "latest frame failed");
        return nullptr;
    }
    return pixels;
}

bool HipPathTracer::setOption(int key, long long value) {
    if (!hipptSetOption(key, value)) {
        m_lastError = "invalid option";
        return false;
    }
    return true;
}
