// hippt_render.cpp — Qt-free C++ caller of libhippt.so through HipPathTracer: the render loop of
// RayTracerFboItem (updatePaintNode → m_cudaTracer->renderFrame(maxDepth) once per frame,
// RayTracerFboItem.cpp:516-575) without the scene graph.
//
//   hippt_render [--mesh FILE.obj|.ply] [--albedo r,g,b[;r,g,b...]] [--width W] [--height H]
//                [--spp N] [--depth D] [--per-frame] [--present] [--out FILE.argb] [--ppm FILE.ppm]
//
// Without --mesh: the reference kernel's built-in 4-sphere scene, one renderFrame per frame (the
// CUDA backend's loop).  With --mesh: the file's triangles (hipptReadMesh) under the Cornell
// camera, all N frames in one renderFrames call, or one call per frame with --per-frame, or
// through the non-blocking hand-off with --present.  --out writes the ARGB words (row 0 =
// bottom, little endian), --ppm an image (top row first).  Prints one JSON line.
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <sstream>
#include <string>
#include <vector>

#include "HipPathTracer.h"

namespace {

int usage() {
    std::fprintf(stderr,
                 "usage: hippt_render [--mesh FILE] [--albedo r,g,b[;...]] [--width W] [--height H] [--spp N]\n"
                 "                    [--depth D] [--per-frame] [--present] [--out FILE.argb] [--ppm FILE.ppm]\n");
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
    std::string mesh, out, ppm, albedoArg;
    int width = 320, height = 180, spp = 16, depth = 8;
    bool perFrame = false, present = false;
    for (int i = 1; i < argc; ++i) {
        const std::string a = argv[i];
        auto next = [&]() -> const char * { return i + 1 < argc ? argv[++i] : nullptr; };
        const char *v = nullptr;
        if (a == "--per-frame") perFrame = true;
        else if (a == "--present") present = true;
        else if ((v = next()) == nullptr) return usage();
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
    HipPathTracer tracer;
    if (!mesh.empty()) {
        const double from[3] = {278, 278, -800}, at[3] = {278, 278, 0}, up[3] = {0, 1, 0};
        if (!tracer.loadMeshFile(mesh, parse_floats(albedoArg), from, at, up, 40.0, 0.0, 10.0)) {
            std::fprintf(stderr, "hippt_render: %s\n", tracer.lastError().c_str());
            return 1;
        }
    }
    if (!tracer.initialize(width, height)) {
        std::fprintf(stderr, "hippt_render: %s\n", tracer.lastError().c_str());
        return 1;
    }
    const auto t0 = std::chrono::steady_clock::now();
    bool ok = true;
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
    const size_t n = size_t(width) * size_t(height);
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
    hipptStats st;
    hipptGetStats(&st);
    std::printf("{\"frames\": %d, \"seconds\": %.6f, \"segments\": %llu, \"pixel_samples\": %llu}\n",
                tracer.frameIndex(), secs, (unsigned long long)st.segments, (unsigned long long)st.pixelSamples);
    return 0;
}
