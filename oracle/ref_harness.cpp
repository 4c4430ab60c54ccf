// ref_harness.cpp — TEST INFRASTRUCTURE ONLY.
//
// Qt-free harness around the UNMODIFIED reference CPU path tracer
// (/root/reference/include/raytracer/RayTracer.h, included from where it lies;
// never copied).  Built by oracle/Makefile into oracle/_ref/ref_harness.  Used for:
//
//   golden   — FP64 known-answer vectors of reference functions (Sphere::hit,
//              AABB::hit, surrounding_box, Camera::get_ray @ aperture 0, BVHNode
//              closest hit over triangles) -> tests/golden/*.json
//   converge — converged radiance image via the reference ray_color (:579-596)
//              for statistical agreement with the FP32 restatement
//   random_scene — the reference's random_scene() (spheres, Lambertian/Metal/Dielectric)
//              dumped as a scene file -> tests/golden/ref_random_scene.scene
//   bench    — RenderWorker::render (RayTracerFboItem.cpp:46-144) restated without
//              Qt: hardware_concurrency threads over an atomic tile queue with the
//              chooseTileSize rule (:793-820); the cpu_baseline of bench.py
//
// The reference has no triangle primitive; `Triangle` below is the harness's
// Möller–Trumbore Hitable (FP64), plugged in through the Hitable interface
// (RayTracer.h:267-272).  The reference AABB::hit (:229-244) rejects zero-thickness
// boxes (t_max <= t_min), so triangle boxes are padded by 1e-4.
#include "raytracer/RayTracer.h"

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <string>

namespace {

class Triangle : public Hitable {
public:
    Triangle(const Point3 &a, const Point3 &b, const Point3 &c, std::shared_ptr<Material> m)
        : v0(a), e1(b - a), e2(c - a), mat(std::move(m)) {
        Vec3 cr = cross(e1, e2);
        double len = cr.length();
        n = len > 0 ? cr / len : Vec3(0, 0, 0);
        Point3 lo(std::fmin(a.x(), std::fmin(b.x(), c.x())), std::fmin(a.y(), std::fmin(b.y(), c.y())),
                  std::fmin(a.z(), std::fmin(b.z(), c.z())));
        Point3 hi(std::fmax(a.x(), std::fmax(b.x(), c.x())), std::fmax(a.y(), std::fmax(b.y(), c.y())),
                  std::fmax(a.z(), std::fmax(b.z(), c.z())));
        const Vec3 pad(1e-4, 1e-4, 1e-4);
        box = AABB(lo - pad, hi + pad);
    }

    bool hit(const Ray &r, double t_min, double t_max, HitRecord &rec) const override {
        Vec3 pv = cross(r.direction(), e2);
        double det = dot(e1, pv);
        if (det == 0.0) return false;
        double inv = 1.0 / det;
        Vec3 tv = r.origin() - v0;
        double u = dot(tv, pv) * inv;
        if (u < 0.0 || u > 1.0) return false;
        Vec3 qv = cross(tv, e1);
        double v = dot(r.direction(), qv) * inv;
        if (v < 0.0 || u + v > 1.0) return false;
        double t = dot(e2, qv) * inv;
        if (t < t_min || t > t_max) return false;
        rec.t = t;
        rec.p = r.at(t);
        rec.set_face_normal(r, n);
        rec.mat_ptr = mat;
        return true;
    }

    bool bounding_box(AABB &out) const override {
        out = box;
        return true;
    }

private:
    Point3 v0;
    Vec3 e1, e2, n;
    std::shared_ptr<Material> mat;
    AABB box;
};

// Counts top-level closest-hit queries (= ray segments).
thread_local unsigned long long tl_segments = 0;
class Counting : public Hitable {
public:
    explicit Counting(const Hitable &w) : world(w) {}
    bool hit(const Ray &r, double tmin, double tmax, HitRecord &rec) const override {
        ++tl_segments;
        return world.hit(r, tmin, tmax, rec);
    }
    bool bounding_box(AABB &out) const override { return world.bounding_box(out); }
    const Hitable &world;
};

struct MatDesc {
    int kind;  // 0 Lambertian, 1 Metal, 2 Dielectric
    float albedo[3], fuzz, ir;
};

struct Scene {
    std::vector<float> verts;
    std::vector<int> mat;
    std::vector<float> spheres;  // cx, cy, cz, r
    std::vector<int> sphMat;
    std::vector<MatDesc> mats;
    double lookfrom[3], lookat[3], vup[3], vfov, aperture, focus;
};

// Scene files written by qt-raytracer_amd/hippt/scenes.py (write_scene_file): v1 'HTPS'
// (Lambertian triangles), v2 'HTP2' (triangles, spheres, material kinds).
bool load_scene(const char *path, Scene &s) {
    std::ifstream f(path, std::ios::binary);
    if (!f) return false;
    int magic = 0;
    f.read(reinterpret_cast<char *>(&magic), 4);
    int nt = 0, ns = 0, nm = 0;
    if (magic == 0x53505448) {
        int hdr[2];
        f.read(reinterpret_cast<char *>(hdr), sizeof(hdr));
        nt = hdr[0];
        nm = hdr[1];
    } else if (magic == 0x32505448) {
        int hdr[3];
        f.read(reinterpret_cast<char *>(hdr), sizeof(hdr));
        nt = hdr[0];
        ns = hdr[1];
        nm = hdr[2];
    } else {
        return false;
    }
    s.verts.resize(size_t(nt) * 9);
    s.mat.resize(nt);
    f.read(reinterpret_cast<char *>(s.verts.data()), s.verts.size() * 4);
    f.read(reinterpret_cast<char *>(s.mat.data()), s.mat.size() * 4);
    s.mats.resize(nm);
    if (magic == 0x53505448) {
        std::vector<float> albedo(size_t(nm) * 3);
        f.read(reinterpret_cast<char *>(albedo.data()), albedo.size() * 4);
        for (int m = 0; m < nm; ++m) s.mats[m] = MatDesc{0, {albedo[3 * m], albedo[3 * m + 1], albedo[3 * m + 2]}, 0, 1};
    } else {
        s.spheres.resize(size_t(ns) * 4);
        s.sphMat.resize(ns);
        f.read(reinterpret_cast<char *>(s.spheres.data()), s.spheres.size() * 4);
        f.read(reinterpret_cast<char *>(s.sphMat.data()), s.sphMat.size() * 4);
        for (int m = 0; m < nm; ++m) {
            int kind;
            float w[5];
            f.read(reinterpret_cast<char *>(&kind), 4);
            f.read(reinterpret_cast<char *>(w), sizeof(w));
            s.mats[m] = MatDesc{kind, {w[0], w[1], w[2]}, w[3], w[4]};
        }
    }
    double cam[12];
    f.read(reinterpret_cast<char *>(cam), sizeof(cam));
    for (int i = 0; i < 3; ++i) {
        s.lookfrom[i] = cam[i];
        s.lookat[i] = cam[3 + i];
        s.vup[i] = cam[6 + i];
    }
    s.vfov = cam[9];
    s.aperture = cam[10];
    s.focus = cam[11];
    return bool(f);
}

std::vector<std::shared_ptr<Hitable>> make_objects(const Scene &s) {
    std::vector<std::shared_ptr<Material>> mats;
    for (const MatDesc &m : s.mats) {
        const Color a(m.albedo[0], m.albedo[1], m.albedo[2]);
        if (m.kind == 1) mats.push_back(std::make_shared<Metal>(a, m.fuzz));
        else if (m.kind == 2) mats.push_back(std::make_shared<Dielectric>(m.ir));
        else mats.push_back(std::make_shared<Lambertian>(a));
    }
    std::vector<std::shared_ptr<Hitable>> objs;
    for (size_t t = 0; t < s.mat.size(); ++t) {
        const float *v = &s.verts[9 * t];
        objs.push_back(std::make_shared<Triangle>(Point3(v[0], v[1], v[2]), Point3(v[3], v[4], v[5]),
                                                  Point3(v[6], v[7], v[8]), mats[s.mat[t]]));
    }
    for (size_t k = 0; k < s.sphMat.size(); ++k) {
        const float *q = &s.spheres[4 * k];
        objs.push_back(std::make_shared<Sphere>(Point3(q[0], q[1], q[2]), q[3], mats[s.sphMat[k]]));
    }
    return objs;
}

// The reference's own random_scene() (RayTracer.h:599-643, nondeterministic RNG) dumped as a
// v2 scene file with RenderWorker::render's camera (RayTracerFboItem.cpp:50-56); coordinates
// and material parameters are rounded to float, which the file and the GPU path use.
int cmd_random_scene(const char *out_path) {
    HitableList world = random_scene();
    std::vector<float> spheres;
    std::vector<int> sphMat;
    std::vector<MatDesc> mats;
    for (const auto &obj : world.objects) {
        auto sp = std::dynamic_pointer_cast<Sphere>(obj);
        if (!sp) return 4;
        MatDesc m{0, {0, 0, 0}, 0, 1};
        if (auto l = std::dynamic_pointer_cast<Lambertian>(sp->mat_ptr)) {
            m = MatDesc{0, {float(l->albedo.x()), float(l->albedo.y()), float(l->albedo.z())}, 0, 1};
        } else if (auto me = std::dynamic_pointer_cast<Metal>(sp->mat_ptr)) {
            m = MatDesc{1, {float(me->albedo.x()), float(me->albedo.y()), float(me->albedo.z())}, float(me->fuzz), 1};
        } else if (auto d = std::dynamic_pointer_cast<Dielectric>(sp->mat_ptr)) {
            m = MatDesc{2, {1, 1, 1}, 0, float(d->ir)};
        } else {
            return 5;
        }
        spheres.insert(spheres.end(), {float(sp->center.x()), float(sp->center.y()), float(sp->center.z()),
                                       float(sp->radius)});
        sphMat.push_back(int(mats.size()));
        mats.push_back(m);
    }
    FILE *f = std::fopen(out_path, "wb");
    if (!f) return 2;
    const int hdr[4] = {0x32505448, 0, int(sphMat.size()), int(mats.size())};
    std::fwrite(hdr, 4, 4, f);
    std::fwrite(spheres.data(), 4, spheres.size(), f);
    std::fwrite(sphMat.data(), 4, sphMat.size(), f);
    for (const MatDesc &m : mats) {
        const float w[5] = {m.albedo[0], m.albedo[1], m.albedo[2], m.fuzz, m.ir};
        std::fwrite(&m.kind, 4, 1, f);
        std::fwrite(w, 4, 5, f);
    }
    const double cam[12] = {13, 2, 3, 0, 0, 0, 0, 1, 0, 20, 0.1, 10};
    std::fwrite(cam, 8, 12, f);
    std::fclose(f);
    return 0;
}

// Deterministic input generator for golden vectors (not the render RNG).
struct Lcg {
    uint64_t s;
    explicit Lcg(uint64_t seed) : s(seed) {}
    double next() {
        s = s * 6364136223846793005ULL + 1442695040888963407ULL;
        return double(s >> 11) * (1.0 / 9007199254740992.0);
    }
    double range(double a, double b) { return a + (b - a) * next(); }
};

void jvec(FILE *f, const Vec3 &v) { std::fprintf(f, "[%.17g,%.17g,%.17g]", v.x(), v.y(), v.z()); }

int cmd_golden(const char *out_path, const char *scene_path) {
    FILE *f = std::fopen(out_path, "w");
    if (!f) return 2;
    Lcg g(12345);
    std::fprintf(f, "{\n");
    // Sphere::hit (RayTracer.h:289-314) with set_face_normal (:215-218)
    std::fprintf(f, "\"sphere_hit\": [\n");
    auto mat = std::make_shared<Lambertian>(Color(0.5, 0.5, 0.5));
    for (int i = 0; i < 500; ++i) {
        Point3 c(g.range(-2, 2), g.range(-2, 2), g.range(-4, -1));
        double r = g.range(0.1, 1.5);
        Point3 o(g.range(-1, 1), g.range(-1, 1), g.range(-0.5, 0.5));
        Vec3 tgt = c + Vec3(g.range(-1.5, 1.5), g.range(-1.5, 1.5), g.range(-1.5, 1.5)) * r;
        Vec3 d = (tgt - o) * g.range(0.5, 2.0);
        Sphere sp(c, r, mat);
        HitRecord rec;
        bool h = sp.hit(Ray(o, d), 0.001, infinity, rec);
        std::fprintf(f, "{\"c\":"); jvec(f, c);
        std::fprintf(f, ",\"r\":%.17g,\"o\":", r); jvec(f, o);
        std::fprintf(f, ",\"d\":"); jvec(f, d);
        std::fprintf(f, ",\"hit\":%d", h ? 1 : 0);
        if (h) {
            std::fprintf(f, ",\"t\":%.17g,\"front\":%d,\"n\":", rec.t, rec.front_face ? 1 : 0);
            jvec(f, rec.normal);
        }
        std::fprintf(f, "}%s\n", i + 1 < 500 ? "," : "");
    }
    std::fprintf(f, "],\n");
    // AABB::hit (:229-244) and surrounding_box (:251-265)
    std::fprintf(f, "\"aabb_hit\": [\n");
    for (int i = 0; i < 500; ++i) {
        Point3 a(g.range(-2, 2), g.range(-2, 2), g.range(-5, -1));
        Point3 b = a + Vec3(g.range(0.05, 2), g.range(0.05, 2), g.range(0.05, 2));
        Point3 o(g.range(-1, 1), g.range(-1, 1), g.range(-0.5, 0.5));
        Vec3 d(g.range(-1, 1), g.range(-1, 1), g.range(-1.5, -0.2));
        AABB box(a, b);
        bool h = box.hit(Ray(o, d), 0.001, infinity);
        std::fprintf(f, "{\"lo\":"); jvec(f, a);
        std::fprintf(f, ",\"hi\":"); jvec(f, b);
        std::fprintf(f, ",\"o\":"); jvec(f, o);
        std::fprintf(f, ",\"d\":"); jvec(f, d);
        std::fprintf(f, ",\"hit\":%d}%s\n", h ? 1 : 0, i + 1 < 500 ? "," : "");
    }
    std::fprintf(f, "],\n\"surrounding_box\": [\n");
    for (int i = 0; i < 200; ++i) {
        Point3 a0(g.range(-3, 3), g.range(-3, 3), g.range(-3, 3));
        Point3 b0 = a0 + Vec3(g.next(), g.next(), g.next());
        Point3 a1(g.range(-3, 3), g.range(-3, 3), g.range(-3, 3));
        Point3 b1 = a1 + Vec3(g.next(), g.next(), g.next());
        AABB m = surrounding_box(AABB(a0, b0), AABB(a1, b1));
        std::fprintf(f, "{\"a\":[");
        jvec(f, a0); std::fprintf(f, ","); jvec(f, b0); std::fprintf(f, "],\"b\":[");
        jvec(f, a1); std::fprintf(f, ","); jvec(f, b1); std::fprintf(f, "],\"m\":[");
        jvec(f, m.min()); std::fprintf(f, ","); jvec(f, m.max());
        std::fprintf(f, "]}%s\n", i + 1 < 200 ? "," : "");
    }
    // Camera::get_ray with aperture 0 (:545-567): the disk draw is scaled by 0, so deterministic.
    std::fprintf(f, "],\n\"camera\": [\n");
    for (int i = 0; i < 100; ++i) {
        Point3 from(g.range(-10, 10), g.range(-10, 10), g.range(-10, 10));
        Point3 at(g.range(-2, 2), g.range(-2, 2), g.range(-2, 2));
        Vec3 vup(0, 1, 0);
        double vfov = g.range(20, 90), aspect = g.range(0.5, 2.5), focus = g.range(0.5, 20);
        Camera cam(from, at, vup, vfov, aspect, 0.0, focus);
        double s = g.next(), t = g.next();
        Ray r = cam.get_ray(s, t);
        std::fprintf(f, "{\"from\":"); jvec(f, from);
        std::fprintf(f, ",\"at\":"); jvec(f, at);
        std::fprintf(f, ",\"vfov\":%.17g,\"aspect\":%.17g,\"focus\":%.17g,\"s\":%.17g,\"t\":%.17g,\"o\":", vfov,
                     aspect, focus, s, t);
        jvec(f, r.origin());
        std::fprintf(f, ",\"d\":");
        jvec(f, r.direction());
        std::fprintf(f, "}%s\n", i + 1 < 100 ? "," : "");
    }
    std::fprintf(f, "],\n\"reflect\": [\n");
    for (int i = 0; i < 100; ++i) {
        Vec3 v(g.range(-1, 1), g.range(-1, 1), g.range(-1, 1));
        Vec3 n = unit_vector(Vec3(g.range(-1, 1), g.range(-1, 1), g.range(-1, 1)));
        double eta = g.range(0.5, 1.5);
        Vec3 uv = unit_vector(v);
        std::fprintf(f, "{\"v\":"); jvec(f, v);
        std::fprintf(f, ",\"n\":"); jvec(f, n);
        std::fprintf(f, ",\"eta\":%.17g,\"reflect\":", eta); jvec(f, reflect(v, n));
        std::fprintf(f, ",\"refract\":"); jvec(f, refract(uv, n, eta));
        std::fprintf(f, "}%s\n", i + 1 < 100 ? "," : "");
    }
    std::fprintf(f, "],\n\"degrees_to_radians\": [");
    for (int i = 0; i < 16; ++i) {
        double a = g.range(-720, 720);
        std::fprintf(f, "[%.17g,%.17g]%s", a, degrees_to_radians(a), i + 1 < 16 ? "," : "");
    }
    std::fprintf(f, "]");
    // BVHNode (:374-465) closest hit over the harness Triangle, scene from file.
    if (scene_path) {
        Scene s;
        if (!load_scene(scene_path, s)) { std::fclose(f); return 3; }
        auto objs = make_objects(s);
        BVHNode world(objs, 0, objs.size());
        float lo[3] = {1e30f, 1e30f, 1e30f}, hi[3] = {-1e30f, -1e30f, -1e30f};
        for (size_t i = 0; i < s.verts.size(); ++i) {
            lo[i % 3] = std::min(lo[i % 3], s.verts[i]);
            hi[i % 3] = std::max(hi[i % 3], s.verts[i]);
        }
        std::fprintf(f, ",\n\"bvh_closest\": [\n");
        const int nrays = 1000;
        for (int i = 0; i < nrays; ++i) {
            // origins inside the scene bounds or at the camera; float-representable inputs
            Point3 o;
            if (i % 4 == 0) o = Point3(s.lookfrom[0], s.lookfrom[1], s.lookfrom[2]);
            else o = Point3(float(g.range(lo[0], hi[0])), float(g.range(lo[1], hi[1])), float(g.range(lo[2], hi[2])));
            Point3 tg(g.range(lo[0], hi[0]), g.range(lo[1], hi[1]), g.range(lo[2], hi[2]));
            Vec3 dd = tg - o;
            Vec3 d(float(dd.x()), float(dd.y()), float(dd.z()));
            HitRecord rec;
            bool h = world.hit(Ray(o, d), 0.001, infinity, rec);
            std::fprintf(f, "{\"o\":"); jvec(f, o);
            std::fprintf(f, ",\"d\":"); jvec(f, d);
            std::fprintf(f, ",\"hit\":%d", h ? 1 : 0);
            if (h) {
                std::fprintf(f, ",\"t\":%.17g,\"n\":", rec.t);
                jvec(f, rec.normal);
            }
            std::fprintf(f, "}%s\n", i + 1 < nrays ? "," : "");
        }
        std::fprintf(f, "]");
    }
    std::fprintf(f, "\n}\n");
    std::fclose(f);
    return 0;
}

// Converged radiance: per-pixel mean and variance of ray_color over spp samples.
int cmd_converge(const char *scene_path, int W, int H, int spp, int depth, const char *out_path, int threads) {
    Scene s;
    if (!load_scene(scene_path, s)) return 3;
    auto objs = make_objects(s);
    BVHNode world(objs, 0, objs.size());
    Camera cam(Point3(s.lookfrom[0], s.lookfrom[1], s.lookfrom[2]), Point3(s.lookat[0], s.lookat[1], s.lookat[2]),
               Vec3(s.vup[0], s.vup[1], s.vup[2]), s.vfov, double(W) / double(H), s.aperture, s.focus);
    std::vector<float> out(size_t(W) * H * 6);
    std::atomic<int> next_row(0);
    auto work = [&]() {
        for (;;) {
            int y = next_row.fetch_add(1);
            if (y >= H) break;
            for (int x = 0; x < W; ++x) {
                double sum[3] = {0, 0, 0}, sq[3] = {0, 0, 0};
                for (int k = 0; k < spp; ++k) {
                    double u = (x + random_double()) / std::max(1, W - 1);
                    double v = (y + random_double()) / std::max(1, H - 1);
                    Color c = ray_color(cam.get_ray(u, v), world, depth);
                    for (int a = 0; a < 3; ++a) { sum[a] += c[a]; sq[a] += c[a] * c[a]; }
                }
                float *o = &out[(size_t(y) * W + x) * 6];
                for (int a = 0; a < 3; ++a) {
                    double m = sum[a] / spp;
                    o[a] = float(m);
                    o[3 + a] = float(std::max(0.0, sq[a] / spp - m * m));
                }
            }
        }
    };
    std::vector<std::thread> ts;
    for (int i = 0; i < std::max(1, threads); ++i) ts.emplace_back(work);
    for (auto &t : ts) t.join();
    FILE *f = std::fopen(out_path, "wb");
    if (!f) return 2;
    std::fwrite(out.data(), 4, out.size(), f);
    std::fclose(f);
    return 0;
}

// RayTracerFboItem::chooseTileSize (:793-820) for the OpenGL scene graph.
int choose_tile(int w, int h) {
    int px = w * h, t = 16;
    if (px >= 1920 * 1080) t = 24;
    if (px >= 2560 * 1440) t = 32;
    return std::clamp(t, 8, 48);
}

// RenderWorker::render (RayTracerFboItem.cpp:46-144) without Qt; timing only.
// Renders every `stride`-th line of a W x H image (a bounded, representative sample of
// the workload: lines 0, stride, 2*stride, ...), tiled over the compacted lines.  With
// `parts` > 1 only the sample's lines k with k % parts == part (one of `parts` processes
// splitting the same sample).
int cmd_bench(const char *scene_path, int W, int H, int stride, int spp, int depth, int threads, int part = 0,
              int parts = 1) {
    if (stride < 1) stride = 1;
    if (parts < 1 || part < 0 || part >= parts) parts = 1, part = 0;
    const int sampleRows = (H + stride - 1) / stride;
    const int rows = sampleRows > part ? (sampleRows - part + parts - 1) / parts : 0;
    Scene s;
    if (!load_scene(scene_path, s)) return 3;
    auto t_setup = std::chrono::steady_clock::now();
    auto objs = make_objects(s);
    BVHNode bvh(objs, 0, objs.size());
    Counting world(bvh);
    Camera cam(Point3(s.lookfrom[0], s.lookfrom[1], s.lookfrom[2]), Point3(s.lookat[0], s.lookat[1], s.lookat[2]),
               Vec3(s.vup[0], s.vup[1], s.vup[2]), s.vfov, double(W) / double(H), s.aperture, s.focus);
    const double invW = 1.0 / double(std::max(1, W - 1)), invH = 1.0 / double(std::max(1, H - 1));
    const double scale = 1.0 / double(spp);
    const int tile = choose_tile(W, H);
    const int tilesX = (W + tile - 1) / tile, tilesY = (rows + tile - 1) / tile;
    const int total = tilesX * tilesY;
    if (threads <= 0) threads = int(std::thread::hardware_concurrency());
    if (threads <= 0) threads = 1;
    std::vector<unsigned> image(size_t(W) * rows);
    std::atomic<int> next(0);
    std::atomic<unsigned long long> segs(0);
    auto t0 = std::chrono::steady_clock::now();
    std::vector<std::thread> ws;
    for (int ti = 0; ti < threads; ++ti) {
        ws.emplace_back([&]() {
            tl_segments = 0;
            for (;;) {
                int idx = next.fetch_add(1, std::memory_order_relaxed);
                if (idx >= total) break;
                int x0 = (idx % tilesX) * tile, y0 = (idx / tilesX) * tile;
                int x1 = std::min(x0 + tile, W), y1 = std::min(y0 + tile, rows);
                for (int line = y0; line < y1; ++line) {
                    const int j = H - 1 - (part + line * parts) * stride;
                    for (int i = x0; i < x1; ++i) {
                        Color pc(0, 0, 0);
                        for (int k = 0; k < spp; ++k) {
                            const double u = (double(i) + random_double()) * invW;
                            const double v = (double(j) + random_double()) * invH;
                            pc += ray_color(cam.get_ray(u, v), world, depth);
                        }
                        const int ir = int(256 * clamp(std::sqrt(scale * pc.x()), 0.0, 0.999));
                        const int ig = int(256 * clamp(std::sqrt(scale * pc.y()), 0.0, 0.999));
                        const int ib = int(256 * clamp(std::sqrt(scale * pc.z()), 0.0, 0.999));
                        image[size_t(line) * W + i] = (255u << 24) | (unsigned(ir) << 16) | (unsigned(ig) << 8) | unsigned(ib);
                    }
                }
            }
            segs.fetch_add(tl_segments);
        });
    }
    for (auto &w : ws) w.join();
    auto t1 = std::chrono::steady_clock::now();
    double secs = std::chrono::duration<double>(t1 - t0).count();
    double setup = std::chrono::duration<double>(t0 - t_setup).count();
    unsigned long long ps = (unsigned long long)W * rows * spp;
    unsigned long long chk = 0;
    for (unsigned p : image) chk = chk * 1315423911ULL + p;
    std::printf("{\"seconds\": %.6f, \"setup_seconds\": %.6f, \"threads\": %d, \"tile\": %d, \"width\": %d, "
                "\"height\": %d, \"rows\": %d, \"stride\": %d, \"spp\": %d, \"depth\": %d, \"pixel_samples\": %llu, "
                "\"segments\": %llu, \"msamples_per_s\": %.6f, \"mpixel_samples_per_s\": %.6f, \"checksum\": %llu}\n",
                secs, setup, threads, tile, W, H, rows, stride, spp, depth, ps, (unsigned long long)segs.load(),
                double(segs.load()) / secs / 1e6, double(ps) / secs / 1e6, chk);
    return 0;
}

}  // namespace

int main(int argc, char **argv) {
    if (argc >= 3 && std::strcmp(argv[1], "golden") == 0)
        return cmd_golden(argv[2], argc >= 4 ? argv[3] : nullptr);
    if (argc >= 8 && std::strcmp(argv[1], "converge") == 0)
        return cmd_converge(argv[2], std::atoi(argv[3]), std::atoi(argv[4]), std::atoi(argv[5]), std::atoi(argv[6]),
                            argv[7], argc >= 9 ? std::atoi(argv[8]) : 1);
    if (argc >= 3 && std::strcmp(argv[1], "random_scene") == 0) return cmd_random_scene(argv[2]);
    if (argc >= 8 && std::strcmp(argv[1], "bench") == 0)
        return cmd_bench(argv[2], std::atoi(argv[3]), std::atoi(argv[4]), std::atoi(argv[5]), std::atoi(argv[6]),
                         std::atoi(argv[7]), argc >= 9 ? std::atoi(argv[8]) : 0, argc >= 10 ? std::atoi(argv[9]) : 0,
                         argc >= 11 ? std::atoi(argv[10]) : 1);
    std::fprintf(stderr,
                 "usage: ref_harness golden OUT.json [SCENE]\n"
                 "       ref_harness converge SCENE W H SPP DEPTH OUT.f32 [THREADS]\n"
                 "       ref_harness bench SCENE W H STRIDE SPP DEPTH [THREADS [PART PARTS]]\n"
                 "       ref_harness random_scene OUT.scene\n");
    return 1;
}
