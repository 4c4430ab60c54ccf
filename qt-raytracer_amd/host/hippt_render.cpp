// hippt_render.cpp — Qt-free C++ caller of libhippt.so through HipPathTracer: the render loop of
// RayTracerFboItem (updatePaintNode → m_cudaTracer->renderFrame(maxDepth) once per frame,
// RayTracerFboItem.cpp:516-575) without the scene graph.
//
//   hippt_render [--backend cuda|vulkan|gl] [--mesh FILE.obj|.ply] [--albedo r,g,b[;r,g,b...]]
//                [--width W] [--height H] [--spp N] [--depth D] [--per-frame] [--present]
//                [--out FILE] [--ppm FILE.ppm]
//
// --backend cuda (default): HipPathTracer, the CudaPathTracer interface.  Without --mesh: the
// reference kernel's built-in 4-sphere scene, one renderFrame per frame (the CUDA backend's
// loop).  With --mesh: the file's triangles (hipptReadMesh) under the Cornell camera, all N
// frames in one renderFrames call, or one call per frame with --per-frame, or through the
// non-blocking hand-off with --present.
// --backend vulkan: HipVulkanPathTracer, one renderFrame(depth) per frame (the app's "vulkan"
// branch, RayTracerFboItem.cpp:576-600).  --backend gl: HipGpuPathTracer, initialize + resize,
// then renderFrame(N, depth) once (or per frame with --per-frame), as the GL branch calls it.
// --out writes the frame words (cuda: ARGB; vulkan / gl: RGBA8; row 0 = bottom, little endian),
// --ppm an image (top row first).  Prints one JSON line.
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <sstream>
#include <string>
#include <vector>

#include "HipComputeTracers.h"
#include "HipPathTracer.h"

namespace {

int usage() {
    std::fprintf(stderr,
                 "usage: hippt_render [--backend cuda|vulkan|gl] [--mesh FILE] [--albedo r,g,b[;...]] [--width W]\n"
                 "                    [--height H] [--spp N] [--depth D] [--per-frame] [--present] [--out FILE]\n"
                 "                    [--ppm FILE.ppm]\n");
    return 2;
}

std::vector<float> parse_floats(const std::string &s) {
    std::vector<float> v;
    std::string tok;
    for (char ch : s + ",") {
        if (ch == ',' || ch == ';') {
            if (!tok.empty()) v.push_back(std::strtof(tok.c_str(), nullptr));
            tok.clear();
        } else {
            tok += ch;
        }
    }
    return v;
}

}  // namespace

int main(int argc, char **argv) {
    std::string mesh, out, ppm, albedoArg, backend = "cuda";
    int width = 320, height = 180, spp = 16, depth = 8;
    bool perFrame = false, present = false;
    for (int i = 1; i < argc; ++i) {
        const std::string a = argv[i];
        auto next = [&]() -> const char * { return i + 1 < argc ? argv[++i] : nullptr; };
        const char *v = nullptr;
        if (a == "--per-frame") perFrame = true;
        else if (a == "--present") present = true;
        else if ((v = next()) == nullptr) return usage();
        else if (a == "--backend") backend = v;
        else if (a == "--mesh") mesh = v;
        else if (a == "--albedo") albedoArg = v;
        else if (a == "--width") width = std::atoi(v);
        else if (a == "--height") height = std::atoi(v);
        else if (a == "--spp") spp = std::atoi(v);
        else if (a == "--depth") depth = std::atoi(v);
        else if (a == "--out") out = v;
        else if (a == "--ppm") ppm = v;
        else return usage();
    }
    if (backend != "cuda" && backend != "vulkan" && backend != "gl") return usage();
    HipPathTracer tracer;
    if (!mesh.empty()) {
        // the scene is the library's (shared by every interface)
        const double from[3] = {278, 278, -800}, at[3] = {278, 278, 0}, up[3] = {0, 1, 0};
        if (!tracer.loadMeshFile(mesh, parse_floats(albedoArg), from, at, up, 40.0, 0.0, 10.0)) {
            std::fprintf(stderr, "hippt_render: %s\n", tracer.lastError().c_str());
            return 1;
        }
    }
    const bool rgba = backend != "cuda";
    const size_t n = size_t(std::max(0, width)) * size_t(std::max(0, height));
    std::vector<unsigned int> frame;
    int frames = 0;
    const auto t0 = std::chrono::steady_clock::now();
    std::string error;
    bool ok = true;
    hipptStats st{};  // read before the tracer object (and with it the library state) goes
    if (backend == "vulkan") {
        HipVulkanPathTracer vk;
        ok = vk.initialize(width, height);
        for (int f = 0; f < spp && ok; ++f) ok = vk.renderFrame(depth);
        if (ok) frame.assign(vk.hostPixels(), vk.hostPixels() + n);
        hipptGetStats(&st);
        frames = vk.frameIndex();
        error = vk.lastError();
    } else if (backend == "gl") {
        HipGpuPathTracer gl;
        ok = gl.initialize() && gl.resize(width, height);
        if (perFrame)
            for (int f = 0; f < spp && ok; ++f) ok = gl.renderFrame(1, depth);
        else
            ok = ok && gl.renderFrame(spp, depth);
        if (ok) frame.assign(gl.hostPixels(), gl.hostPixels() + n);
        hipptGetStats(&st);
        frames = gl.frameIndex();
        error = gl.lastError();
    }
    if (rgba) {
        const double secs = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        if (!ok) {
            std::fprintf(stderr, "hippt_render: %s\n", error.empty() ? "render failed" : error.c_str());
            return 1;
        }
        if (!out.empty()) {
            FILE *f = std::fopen(out.c_str(), "wb");
            if (!f || std::fwrite(frame.data(), sizeof(unsigned int), n, f) != n) return 1;
            std::fclose(f);
        }
        if (!ppm.empty()) {
            FILE *f = std::fopen(ppm.c_str(), "wb");
            if (!f) return 1;
            std::fprintf(f, "P6\n%d %d\n255\n", width, height);
            for (int y = height - 1; y >= 0; --y)
                for (int x = 0; x < width; ++x) {
                    const unsigned p = frame[size_t(y) * width + x];  // bytes R, G, B, A
                    const unsigned char rgb[3] = {(unsigned char)p, (unsigned char)(p >> 8), (unsigned char)(p >> 16)};
                    std::fwrite(rgb, 1, 3, f);
                }
            std::fclose(f);
        }
        // the process-wide word format is back to its default after the RGBA8 interfaces' renders
        std::printf("{\"backend\": \"%s\", \"frames\": %d, \"seconds\": %.6f, \"segments\": %llu, "
                    "\"pixel_samples\": %llu, \"pixel_format_after\": %lld}\n",
                    backend.c_str(), frames, secs, (unsigned long long)st.segments,
                    (unsigned long long)st.pixelSamples, hipptGetOption(HIPPT_OPT_PIXEL_FORMAT));
        return 0;
    }
    if (!tracer.initialize(width, height)) {
        std::fprintf(stderr, "hippt_render: %s\n", tracer.lastError().c_str());
        return 1;
    }
    const unsigned int *pixels = nullptr;
    if (mesh.empty() || perFrame) {
        for (int f = 0; f < spp && ok; ++f) ok = tracer.renderFrame(depth);  // the app's per-paint call
        pixels = tracer.hostPixels();
    } else if (present) {
        int shown = 0, frames = 0;
        for (int f = 0; f < spp && ok; f += 4) {
            ok = tracer.presentFrames(std::min(4, spp - f), depth);
            if (ok && tracer.latestFrame(&frames)) ++shown;  // a UI would draw this image now
        }
        const char *err = nullptr;
        ok = ok && hipptSynchronize(&err);
        pixels = ok ? tracer.latestFrame(&frames) : nullptr;
        ok = ok && pixels && frames == spp;
        if (ok) std::fprintf(stderr, "hippt_render: %d intermediate images were ready without waiting\n", shown);
    } else {
        ok = tracer.renderFrames(spp, depth);
        pixels = tracer.hostPixels();
    }
    const double secs = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    if (!ok || !pixels) {
        std::fprintf(stderr, "hippt_render: %s\n", tracer.lastError().c_str());
        return 1;
    }
    if (!out.empty()) {
        FILE *f = std::fopen(out.c_str(), "wb");
        if (!f || std::fwrite(pixels, sizeof(unsigned int), n, f) != n) return 1;
        std::fclose(f);
    }
    if (!ppm.empty()) {
        FILE *f = std::fopen(ppm.c_str(), "wb");
        if (!f) return 1;
        std::fprintf(f, "P6\n%d %d\n255\n", width, height);
        for (int y = height - 1; y >= 0; --y)
            for (int x = 0; x < width; ++x) {
                const unsigned p = pixels[size_t(y) * width + x];
                const unsigned char rgb[3] = {(unsigned char)(p >> 16), (unsigned char)(p >> 8), (unsigned char)p};
                std::fwrite(rgb, 1, 3, f);
            }
        std::fclose(f);
    }
    hipptGetStats(&st);
    std::printf("{\"backend\": \"cuda\", \"frames\": %d, \"seconds\": %.6f, \"segments\": %llu, "
                "\"pixel_samples\": %llu}\n",
                tracer.frameIndex(), secs, (unsigned long long)st.segments, (unsigned long long)st.pixelSamples);
    return 0;
}
