/*
 * pt_oracle.c — TEST INFRASTRUCTURE ONLY (see pt_oracle.h).
 *
 * CPU restatement of the reference path tracer's hot path.  Compiled with
 * -ffp-contract=off so that every rounding is the one written here; fused
 * multiply-adds appear only as explicit fmaf() calls, which the HIP kernels
 * (qt-raytracer_amd/csrc/hippt_kernels.hip) issue at exactly the same places.
 * Never linked into the product library.
 */
#include "pt_oracle.h"

#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------------- */
/* RNG — CudaPathTracerKernel.cu:23-35 (hash32, rand01)                        */
/* ------------------------------------------------------------------------- */
uint32_t po_hash32(uint32_t x) {
    x ^= x >> 16;
    x *= 0x7feb352du;
    x ^= x >> 15;
    x *= 0x846ca68bu;
    x ^= x >> 16;
    return x;
}

float po_rand01(uint32_t *state) {
    *state = po_hash32(*state);
    return (float)(*state) / 4294967295.0f;
}

/* CudaPathTracerKernel.cu:144 — computed in int there (overflows at 1080p);
 * restated as uint32 wrap-around, which is what the two's-complement int
 * arithmetic produces on every target. */
uint32_t po_pixel_seed(int x, int y, int width, int frame) {
    uint32_t p = (uint32_t)x + (uint32_t)y * (uint32_t)width;
    return p * 9781u + ((uint32_t)frame + 1u) * 6271u;
}

/* ------------------------------------------------------------------------- */
/* Vector helpers.  The mesh path's arithmetic contract:          */
/*   dot(a,b)   = fma(ax,bx, fma(ay,by, az*bz))                               */
/*   cross(a,b) = (fma(ay,bz,-(az*by)), fma(az,bx,-(ax*bz)), fma(ax,by,-(ay*bx)))*/
/* ------------------------------------------------------------------------- */
static inline po_v3 v3(float x, float y, float z) { po_v3 r = {x, y, z}; return r; }
static inline po_v3 vadd(po_v3 a, po_v3 b) { return v3(a.x + b.x, a.y + b.y, a.z + b.z); }
static inline po_v3 vsub(po_v3 a, po_v3 b) { return v3(a.x - b.x, a.y - b.y, a.z - b.z); }
static inline po_v3 vscale(po_v3 a, float s) { return v3(a.x * s, a.y * s, a.z * s); }
static inline po_v3 vmul(po_v3 a, po_v3 b) { return v3(a.x * b.x, a.y * b.y, a.z * b.z); }
static inline float fdot(po_v3 a, po_v3 b) { return fmaf(a.x, b.x, fmaf(a.y, b.y, a.z * b.z)); }
static inline po_v3 fcross(po_v3 a, po_v3 b) {
    return v3(fmaf(a.y, b.z, -(a.z * b.y)), fmaf(a.z, b.x, -(a.x * b.z)), fmaf(a.x, b.y, -(a.y * b.x)));
}
static inline po_v3 ld3(const float *p) { return v3(p[0], p[1], p[2]); }
static inline void st3(float *p, po_v3 v) { p[0] = v.x; p[1] = v.y; p[2] = v.z; }

/* ------------------------------------------------------------------------- */
/* Camera — RayTracer.h:545-561 (FP64 construction, stored FP32)               */
/* ------------------------------------------------------------------------- */
static void d_unit(const double a[3], double out[3]) {
    double len = sqrt(a[0] * a[0] + a[1] * a[1] + a[2] * a[2]);
    double inv = 1.0 / len; /* operator/(v,t) = (1/t)*v, RayTracer.h:137-139 */
    out[0] = inv * a[0]; out[1] = inv * a[1]; out[2] = inv * a[2];
}
static void d_cross(const double a[3], const double b[3], double out[3]) {
    out[0] = a[1] * b[2] - a[2] * b[1];
    out[1] = a[2] * b[0] - a[0] * b[2];
    out[2] = a[0] * b[1] - a[1] * b[0];
}

void po_camera_build(const double lookfrom[3], const double lookat[3], const double vup[3],
                     double vfov_deg, double aspect, double aperture, double focus_dist, po_camera *out) {
    const double pi = 3.1415926535897932385;
    double theta = vfov_deg * pi / 180.0;
    double h = tan(theta / 2);
    double vh = 2.0 * h;
    double vw = aspect * vh;
    double wv[3] = {lookfrom[0] - lookat[0], lookfrom[1] - lookat[1], lookfrom[2] - lookat[2]};
    double w[3], u[3], v[3], c[3];
    d_unit(wv, w);
    d_cross(vup, w, c);
    d_unit(c, u);
    d_cross(w, u, v);
    double hor[3], ver[3], llc[3];
    for (int i = 0; i < 3; ++i) {
        hor[i] = (focus_dist * vw) * u[i];
        ver[i] = (focus_dist * vh) * v[i];
    }
    for (int i = 0; i < 3; ++i) {
        /* origin - horizontal/2 - vertical/2 - focus_dist*w, left to right;
         * horizontal/2 = (1/2)*horizontal per RayTracer.h:137-139 */
        llc[i] = ((lookfrom[i] - 0.5 * hor[i]) - 0.5 * ver[i]) - focus_dist * w[i];
    }
    out->origin = v3((float)lookfrom[0], (float)lookfrom[1], (float)lookfrom[2]);
    out->llc = v3((float)llc[0], (float)llc[1], (float)llc[2]);
    out->horizontal = v3((float)hor[0], (float)hor[1], (float)hor[2]);
    out->vertical = v3((float)ver[0], (float)ver[1], (float)ver[2]);
    out->u = v3((float)u[0], (float)u[1], (float)u[2]);
    out->v = v3((float)v[0], (float)v[1], (float)v[2]);
    out->lens_radius = (float)(aperture / 2);
    out->pad_ = 0.0f;
}

/* Rejection-loop escape.  hash32 is a bijection with short cycles (fixed points 0 and
 * 3496737362, the 2-cycle {160893342, 357741884}, a 5-cycle, ...); a seed on one of them on
 * which every candidate is rejected makes the reference's `while (true)` loops
 * (CudaPathTracerKernel.cu:61-68, RayTracer.h:155-169) spin forever — e.g. pixel
 * (1750, 1610), frame 17 of a 3840x2160 image seeds the 2-cycle.  Contract: after every 64
 * consecutive rejections the state is xored with PO_ESCAPE (a legitimate sequence is
 * rejected 64 times with probability < 0.48^64 ~ 4e-21, so the first 64 attempts are
 * exactly the reference's). */
#define PO_ESCAPE 0x9E3779B9u
#define PO_ESCAPE_EVERY 64

/* random_in_unit_disk — RayTracer.h:163-169; random_double(-1,1) = -1 + 2r (:53-55). */
void po_random_in_unit_disk(uint32_t *state, float p[3]) {
    for (unsigned tries = 1;; ++tries) {
        float x = fmaf(2.0f, po_rand01(state), -1.0f);
        float y = fmaf(2.0f, po_rand01(state), -1.0f);
        if (fmaf(x, x, y * y) >= 1.0f) {
            if (tries % PO_ESCAPE_EVERY == 0) *state ^= PO_ESCAPE;
            continue;
        }
        p[0] = x; p[1] = y; p[2] = 0.0f;
        return;
    }
}

/* random_in_unit_sphere — RayTracer.h:155-161 (x, y, z drawn in that order, as
 * CudaPathTracerKernel.cu:63). */
void po_random_in_unit_sphere(uint32_t *state, float p[3]) {
    for (unsigned tries = 1;; ++tries) {
        float x = fmaf(2.0f, po_rand01(state), -1.0f);
        float y = fmaf(2.0f, po_rand01(state), -1.0f);
        float z = fmaf(2.0f, po_rand01(state), -1.0f);
        if (fmaf(x, x, fmaf(y, y, z * z)) >= 1.0f) {
            if (tries % PO_ESCAPE_EVERY == 0) *state ^= PO_ESCAPE;
            continue;
        }
        p[0] = x; p[1] = y; p[2] = z;
        return;
    }
}

/* Camera::get_ray — RayTracer.h:563-567. */
void po_camera_get_ray(const po_camera *cam, float s, float t, uint32_t *state, float o[3], float d[3]) {
    float disk[3];
    po_random_in_unit_disk(state, disk);
    float rx = cam->lens_radius * disk[0];
    float ry = cam->lens_radius * disk[1];
    po_v3 off = v3(fmaf(cam->v.x, ry, cam->u.x * rx), fmaf(cam->v.y, ry, cam->u.y * rx),
                   fmaf(cam->v.z, ry, cam->u.z * rx));
    po_v3 org = vadd(cam->origin, off);
    po_v3 dir = v3(fmaf(t, cam->vertical.x, fmaf(s, cam->horizontal.x, cam->llc.x)),
                   fmaf(t, cam->vertical.y, fmaf(s, cam->horizontal.y, cam->llc.y)),
                   fmaf(t, cam->vertical.z, fmaf(s, cam->horizontal.z, cam->llc.z)));
    dir = vsub(vsub(dir, cam->origin), off);
    st3(o, org);
    st3(d, dir);
}

/* ------------------------------------------------------------------------- */
/* Triangles (new capability; plugs in as a Hitable, RayTracer.h:267-272)      */
/* ------------------------------------------------------------------------- */
void po_tri_setup(const float v[9], po_tri *out) {
    po_v3 a = ld3(v), b = ld3(v + 3), c = ld3(v + 6);
    po_v3 e1 = vsub(b, a), e2 = vsub(c, a);
    po_v3 cr = fcross(e1, e2);
    float len = sqrtf(fdot(cr, cr));
    out->v0 = a;
    if (!(len > 0.0f)) { /* degenerate: det == 0 for every ray, never hit */
        out->e1 = v3(0.0f, 0.0f, 0.0f);
        out->e2 = v3(0.0f, 0.0f, 0.0f);
        out->n = v3(0.0f, 0.0f, 0.0f);
        return;
    }
    out->e1 = e1;
    out->e2 = e2;
    out->n = vscale(cr, 1.0f / len);
}

int po_tri_hit(const po_tri *tri, const float o[3], const float d[3], float tmin, float *t) {
    po_v3 D = ld3(d), O = ld3(o);
    po_v3 pv = fcross(D, tri->e2);
    float det = fdot(tri->e1, pv);
    if (det == 0.0f) return 0;
    po_v3 tv = vsub(O, tri->v0);
    float un = fdot(tv, pv);
    po_v3 qv = fcross(tv, tri->e1);
    float vn = fdot(D, qv);
    if (det > 0.0f) {
        if (!(un >= 0.0f && vn >= 0.0f && un + vn <= det)) return 0;
    } else {
        if (!(un <= 0.0f && vn <= 0.0f && un + vn >= det)) return 0;
    }
    float tt = fdot(tri->e2, qv) / det;
    if (!(tt >= tmin)) return 0;
    *t = tt;
    return 1;
}

int po_closest_hit(const po_tri *tris, const int *orig_ids, int ntris, const float o[3], const float d[3],
                   float tmin, float *t_out) {
    float best = INFINITY;
    int best_i = -1, best_id = 0x7fffffff;
    for (int i = 0; i < ntris; ++i) {
        float t;
        if (!po_tri_hit(&tris[i], o, d, tmin, &t)) continue;
        int id = orig_ids ? orig_ids[i] : i;
        if (t < best || (t == best && id < best_id)) {
            best = t; best_i = i; best_id = id;
        }
    }
    *t_out = best;
    return best_i;
}

/* Sphere::hit — RayTracer.h:289-314 in FP32 (plain ops). */
int po_sphere_hit(const float c[3], float r, const float o[3], const float d[3], float tmin, float tmax,
                  float *t, float n[3], int *front) {
    po_v3 oc = vsub(ld3(o), ld3(c)), D = ld3(d);
    float a = D.x * D.x + D.y * D.y + D.z * D.z;
    float hb = oc.x * D.x + oc.y * D.y + oc.z * D.z;
    float cc = (oc.x * oc.x + oc.y * oc.y + oc.z * oc.z) - r * r;
    float disc = hb * hb - a * cc;
    if (disc < 0.0f) return 0;
    float sq = sqrtf(disc);
    float root = (-hb - sq) / a;
    if (root < tmin || root > tmax) {
        root = (-hb + sq) / a;
        if (root < tmin || root > tmax) return 0;
    }
    *t = root;
    po_v3 p = vadd(ld3(o), vscale(D, root));
    po_v3 on = vscale(vsub(p, ld3(c)), 1.0f / r);
    int ff = (on.x * D.x + on.y * D.y + on.z * D.z) < 0.0f;
    *front = ff;
    if (!ff) on = vscale(on, -1.0f);
    st3(n, on);
    return 1;
}

/* AABB::hit — RayTracer.h:229-244 in FP32. */
int po_aabb_hit(const float lo[3], const float hi[3], const float o[3], const float d[3], float tmin, float tmax) {
    for (int a = 0; a < 3; ++a) {
        float inv = 1.0f / d[a];
        float t0 = (lo[a] - o[a]) * inv;
        float t1 = (hi[a] - o[a]) * inv;
        if (inv < 0.0f) { float tmp = t0; t0 = t1; t1 = tmp; }
        tmin = t0 > tmin ? t0 : tmin;
        tmax = t1 < tmax ? t1 : tmax;
        if (tmax <= tmin) return 0;
    }
    return 1;
}

/* ------------------------------------------------------------------------- */
/* Accumulation + tonemap — CudaPathTracerKernel.cu:157-178                   */
/* ------------------------------------------------------------------------- */
static inline unsigned q8(float c) {
    return (unsigned)(sqrtf(fminf(fmaxf(c, 0.0f), 1.0f)) * 255.0f);
}

/* The GL / Vulkan backends' RGBA8 UNORM texel of the same colour (GpuPathTracer.cpp:284-285,
 * pathtrace_vulkan.comp:113-114): bytes R, G, B, A, channel = sqrt(clamp(c, 0, 1)) * 255
 * rounded to nearest, ties to even (the float-to-UNORM conversion, round to nearest). */
static inline unsigned u8n(float c) {
    return (unsigned)rintf(sqrtf(fminf(fmaxf(c, 0.0f), 1.0f)) * 255.0f);
}

void po_rgba8(const float *acc4, long long n, uint32_t *out) {
    for (long long i = 0; i < n; ++i) {
        const float *a = acc4 + 4 * i;
        out[i] = (255u << 24) | (u8n(a[2]) << 16) | (u8n(a[1]) << 8) | u8n(a[0]);
    }
}

uint32_t po_accumulate(float acc[4], const float s[3], int f) {
    float ff = (float)f, fc = (float)(f + 1);
    acc[0] = fmaf(acc[0], ff, s[0]) / fc;
    acc[1] = fmaf(acc[1], ff, s[1]) / fc;
    acc[2] = fmaf(acc[2], ff, s[2]) / fc;
    acc[3] = 1.0f;
    return (255u << 24) | (q8(acc[0]) << 16) | (q8(acc[1]) << 8) | q8(acc[2]);
}

/* ------------------------------------------------------------------------- */
/* sphere4 — CudaPathTracerKernel.cu:53-179, literal (no contraction)          */
/* ------------------------------------------------------------------------- */
static inline float pdot(po_v3 a, po_v3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }

static po_v3 s4_normalize(po_v3 v) { /* :53-59 */
    float len = sqrtf(pdot(v, v));
    if (len <= 1e-6f) return v3(0.0f, 0.0f, 0.0f);
    return v3(v.x / len, v.y / len, v.z / len);
}

static po_v3 s4_rius(uint32_t *st) { /* :61-68, plus the short-cycle escape (PO_ESCAPE) */
    for (unsigned tries = 1;; ++tries) {
        float x = po_rand01(st) * 2.0f - 1.0f;
        float y = po_rand01(st) * 2.0f - 1.0f;
        float z = po_rand01(st) * 2.0f - 1.0f;
        po_v3 p = v3(x, y, z);
        if (pdot(p, p) < 1.0f) return p;
        if (tries % PO_ESCAPE_EVERY == 0) *st ^= PO_ESCAPE;
    }
}

static int s4_hit(po_v3 c, float r, po_v3 ro, po_v3 rd, float *t, po_v3 *n, po_v3 *alb) { /* :70-98 */
    po_v3 oc = vsub(ro, c);
    float a = pdot(rd, rd);
    float b = pdot(oc, rd);
    float cc = pdot(oc, oc) - r * r;
    float d = b * b - a * cc;
    if (d < 0.0f) return 0;
    float s = sqrtf(d);
    float t0 = (-b - s) / a;
    float t1 = (-b + s) / a;
    *t = t0 > 0.001f ? t0 : t1;
    if (*t <= 0.001f) return 0;
    po_v3 p = vadd(ro, vscale(rd, *t));
    *n = s4_normalize(vsub(p, c));
    if (r > 50.0f) *alb = v3(0.8f, 0.8f, 0.0f);
    else if (c.x < -0.5f) *alb = v3(0.8f, 0.3f, 0.3f);
    else if (c.x > 0.5f) *alb = v3(0.3f, 0.8f, 0.3f);
    else *alb = v3(0.75f, 0.75f, 0.75f);
    return 1;
}

static po_v3 s4_trace(po_v3 ro, po_v3 rd, uint32_t *st, int max_depth) { /* :100-134 */
    static const float C[4][4] = {
        {0.0f, -100.5f, -1.0f, 100.0f}, {0.0f, 0.0f, -1.0f, 0.5f},
        {-1.0f, 0.0f, -1.4f, 0.5f}, {1.0f, 0.0f, -1.2f, 0.5f}};
    po_v3 thr = v3(1.0f, 1.0f, 1.0f), rad = v3(0.0f, 0.0f, 0.0f);
    for (int depth = 0; depth < max_depth; ++depth) {
        float bt = 1e20f;
        po_v3 bn = v3(0, 0, 0), ba = v3(0, 0, 0);
        int hit = 0;
        for (int i = 0; i < 4; ++i) {
            float t; po_v3 n, a;
            if (s4_hit(v3(C[i][0], C[i][1], C[i][2]), C[i][3], ro, rd, &t, &n, &a) && t < bt) {
                bt = t; bn = n; ba = a; hit = 1;
            }
        }
        if (!hit) {
            po_v3 un = s4_normalize(rd);
            float a = 0.5f * (un.y + 1.0f);
            po_v3 sky = vadd(vscale(v3(1.0f, 1.0f, 1.0f), 1.0f - a), vscale(v3(0.5f, 0.7f, 1.0f), a));
            rad = vadd(rad, vmul(thr, sky));
            break;
        }
        po_v3 hp = vadd(ro, vscale(rd, bt));
        po_v3 sd = s4_normalize(vadd(bn, s4_rius(st)));
        ro = vadd(hp, vscale(bn, 0.001f));
        rd = sd;
        thr = vmul(thr, ba);
    }
    return rad;
}

static void s4_pixel(int x, int y, int width, int height, int frame, int max_depth, float acc[4], uint32_t *out) {
    /* :143-178 */
    uint32_t seed = po_pixel_seed(x, y, width, frame);
    float wd = (float)(width - 1 > 1 ? width - 1 : 1);
    float hd = (float)(height - 1 > 1 ? height - 1 : 1);
    float u = ((float)x + po_rand01(&seed)) / wd;
    float v = ((float)y + po_rand01(&seed)) / hd;
    float aspect = (float)width / (float)height;
    po_v3 origin = v3(0.0f, 0.3f, 1.2f);
    po_v3 ll = v3(-aspect, -1.0f, -1.0f);
    po_v3 hor = v3(2.0f * aspect, 0.0f, 0.0f);
    po_v3 ver = v3(0.0f, 2.0f, 0.0f);
    po_v3 rd = s4_normalize(vsub(vadd(vadd(ll, vscale(hor, u)), vscale(ver, v)), origin));
    po_v3 s = s4_trace(origin, rd, &seed, max_depth);
    /* :157-178, literal */
    float fi = (float)frame, fc = (float)(frame + 1);
    acc[0] = (acc[0] * fi + s.x) / fc;
    acc[1] = (acc[1] * fi + s.y) / fc;
    acc[2] = (acc[2] * fi + s.z) / fc;
    acc[3] = 1.0f;
    *out = (255u << 24) | (q8(acc[0]) << 16) | (q8(acc[1]) << 8) | q8(acc[2]);
}

/* ------------------------------------------------------------------------- */
/* Row-parallel driver (pixels are independent; output is thread-count-free)  */
/* ------------------------------------------------------------------------- */
typedef struct {
    int kind; /* 0 sphere4, 1 mesh */
    const po_scene *sc;
    int width, height, y0, y1, first, count, max_depth;
    float *accum;
    uint32_t *out;
    int row_begin, row_end;
    uint64_t segs, samples;
} po_job;

static void mesh_pixel(const po_scene *sc, int x, int y, int width, int height, int first, int count,
                       int max_depth, float acc[4], uint32_t *out, uint64_t *segs);

static void *po_worker(void *arg) {
    po_job *j = (po_job *)arg;
    for (int y = j->row_begin; y < j->row_end; ++y) {
        for (int x = 0; x < j->width; ++x) {
            size_t idx = (size_t)(y - j->y0) * (size_t)j->width + (size_t)x;
            float *acc = j->accum + idx * 4;
            if (j->kind == 0) {
                for (int f = j->first; f < j->first + j->count; ++f)
                    s4_pixel(x, y, j->width, j->height, f, j->max_depth, acc, &j->out[idx]);
            } else {
                mesh_pixel(j->sc, x, y, j->width, j->height, j->first, j->count, j->max_depth, acc,
                           &j->out[idx], &j->segs);
            }
            j->samples += (uint64_t)j->count;
        }
    }
    return NULL;
}

static void run_jobs(int kind, const po_scene *sc, int width, int height, int y0, int y1, int first, int count,
                     int max_depth, float *accum, uint32_t *out, uint64_t *stats, int nthreads) {
    if (nthreads < 1) nthreads = 1;
    int rows = y1 - y0;
    if (nthreads > rows) nthreads = rows > 0 ? rows : 1;
    po_job *jobs = (po_job *)calloc((size_t)nthreads, sizeof(po_job));
    pthread_t *th = (pthread_t *)calloc((size_t)nthreads, sizeof(pthread_t));
    for (int i = 0; i < nthreads; ++i) {
        po_job *j = &jobs[i];
        j->kind = kind; j->sc = sc; j->width = width; j->height = height; j->y0 = y0; j->y1 = y1;
        j->first = first; j->count = count; j->max_depth = max_depth; j->accum = accum; j->out = out;
        j->row_begin = y0 + (int)((long long)rows * i / nthreads);
        j->row_end = y0 + (int)((long long)rows * (i + 1) / nthreads);
    }
    if (nthreads == 1) {
        po_worker(&jobs[0]);
    } else {
        for (int i = 0; i < nthreads; ++i) pthread_create(&th[i], NULL, po_worker, &jobs[i]);
        for (int i = 0; i < nthreads; ++i) pthread_join(th[i], NULL);
    }
    if (stats) {
        for (int i = 0; i < nthreads; ++i) { stats[0] += jobs[i].segs; stats[1] += jobs[i].samples; }
    }
    free(jobs);
    free(th);
}

void po_sphere4_frames(int width, int height, int y0, int y1, int first_frame, int count, int max_depth,
                       float *accum, uint32_t *out, int nthreads) {
    run_jobs(0, NULL, width, height, y0, y1, first_frame, count, max_depth, accum, out, NULL, nthreads);
}

/* ------------------------------------------------------------------------- */
/* Scene: triangles + spheres + materials, and an oracle-private BVH (median   */
/* split; result-identical to brute force because culling is conservative and  */
/* ties break on the primitive id)                                             */
/* ------------------------------------------------------------------------- */
typedef struct {
    float lo[3], hi[3];
    int left, right; /* internal: children; leaf: left = first, right = -count */
} po_node;

typedef struct { po_v3 c; float r, r2; } po_sph;

struct po_scene {
    int ntris, nsph, nprim; /* primitive id: triangles 0..ntris-1, then spheres */
    po_tri *tris;           /* by triangle index */
    po_sph *sph;            /* by sphere index */
    int *prim_mat;          /* material of primitive id */
    int nmat;
    po_material *mats;
    po_camera cam;
    int accel;
    po_node *nodes;
    int nnodes;
    int *ref; /* BVH leaf order -> primitive id */
};

typedef struct { float lo[3], hi[3], c[3]; int id; } po_prim;

static int cmp_axis;
static int prim_cmp(const void *a, const void *b) {
    const po_prim *p = (const po_prim *)a, *q = (const po_prim *)b;
    float x = p->c[cmp_axis], y = q->c[cmp_axis];
    if (x < y) return -1;
    if (x > y) return 1;
    return p->id - q->id;
}

static int build_rec(po_scene *sc, po_prim *prims, int begin, int end, float pad) {
    int ni = sc->nnodes++;
    po_node *nd = &sc->nodes[ni];
    float lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
    float clo[3] = {INFINITY, INFINITY, INFINITY}, chi[3] = {-INFINITY, -INFINITY, -INFINITY};
    for (int i = begin; i < end; ++i)
        for (int a = 0; a < 3; ++a) {
            lo[a] = fminf(lo[a], prims[i].lo[a]); hi[a] = fmaxf(hi[a], prims[i].hi[a]);
            clo[a] = fminf(clo[a], prims[i].c[a]); chi[a] = fmaxf(chi[a], prims[i].c[a]);
        }
    for (int a = 0; a < 3; ++a) { nd->lo[a] = lo[a] - pad; nd->hi[a] = hi[a] + pad; }
    int n = end - begin;
    if (n <= 4) {
        nd->left = begin; nd->right = -n;
        return ni;
    }
    int axis = 0;
    float ext = chi[0] - clo[0];
    for (int a = 1; a < 3; ++a) if (chi[a] - clo[a] > ext) { ext = chi[a] - clo[a]; axis = a; }
    cmp_axis = axis;
    qsort(prims + begin, (size_t)n, sizeof(po_prim), prim_cmp);
    int mid = begin + n / 2;
    int l = build_rec(sc, prims, begin, mid, pad);
    int r = build_rec(sc, prims, mid, end, pad);
    sc->nodes[ni].left = l;
    sc->nodes[ni].right = r;
    return ni;
}

static void *xmalloc(size_t n) { return malloc(n > 0 ? n : 1); }

po_scene *po_scene_create2(const float *verts, const int *tri_mat, int ntris, const float *spheres,
                           const int *sph_mat, int nsph, const po_material *mats, int nmat, const po_camera *cam,
                           int accel) {
    po_scene *sc = (po_scene *)calloc(1, sizeof(po_scene));
    if (ntris < 0) ntris = 0;
    if (nsph < 0) nsph = 0;
    if (nmat < 0) nmat = 0;
    sc->ntris = ntris;
    sc->nsph = nsph;
    sc->nprim = ntris + nsph;
    sc->nmat = nmat;
    sc->cam = *cam;
    sc->accel = accel && sc->nprim > 0;
    sc->mats = (po_material *)xmalloc(sizeof(po_material) * (size_t)nmat);
    for (int m = 0; m < nmat; ++m) {
        sc->mats[m] = mats[m];
        /* Metal(a, f): fuzz(f < 1 ? f : 1), RayTracer.h:494 */
        if (sc->mats[m].kind == PO_METAL && !(sc->mats[m].fuzz < 1.0f)) sc->mats[m].fuzz = 1.0f;
    }
    sc->tris = (po_tri *)xmalloc(sizeof(po_tri) * (size_t)ntris);
    sc->sph = (po_sph *)xmalloc(sizeof(po_sph) * (size_t)nsph);
    sc->prim_mat = (int *)xmalloc(sizeof(int) * (size_t)sc->nprim);
    sc->ref = (int *)xmalloc(sizeof(int) * (size_t)sc->nprim);
    for (int i = 0; i < ntris; ++i) {
        po_tri_setup(verts + 9 * (size_t)i, &sc->tris[i]);
        sc->prim_mat[i] = tri_mat[i];
    }
    for (int j = 0; j < nsph; ++j) {
        const float *q = spheres + 4 * (size_t)j;
        sc->sph[j].c = v3(q[0], q[1], q[2]);
        sc->sph[j].r = q[3];
        sc->sph[j].r2 = q[3] * q[3];
        sc->prim_mat[ntris + j] = sph_mat[j];
    }
    for (int i = 0; i < sc->nprim; ++i) sc->ref[i] = i;
    if (!sc->accel) return sc;
    po_prim *prims = (po_prim *)xmalloc(sizeof(po_prim) * (size_t)sc->nprim);
    float maxabs = fmaxf(fmaxf(fabsf(cam->origin.x), fabsf(cam->origin.y)), fabsf(cam->origin.z));
    for (int i = 0; i < sc->nprim; ++i) {
        float mn[3], mx[3];
        if (i < ntris) {
            const float *v = verts + 9 * (size_t)i;
            for (int a = 0; a < 3; ++a) {
                mn[a] = fminf(fminf(v[a], v[3 + a]), v[6 + a]);
                mx[a] = fmaxf(fmaxf(v[a], v[3 + a]), v[6 + a]);
            }
        } else {
            const po_sph *q = &sc->sph[i - ntris];
            float c[3] = {q->c.x, q->c.y, q->c.z}, r = fabsf(q->r) * (1.0f + 1.0f / 4096.0f);
            for (int a = 0; a < 3; ++a) { mn[a] = c[a] - r; mx[a] = c[a] + r; }
        }
        for (int a = 0; a < 3; ++a) {
            prims[i].lo[a] = mn[a]; prims[i].hi[a] = mx[a];
            prims[i].c[a] = 0.5f * (mn[a] + mx[a]);
            maxabs = fmaxf(maxabs, fmaxf(fabsf(mn[a]), fabsf(mx[a])));
        }
        prims[i].id = i;
    }
    float pad = maxabs * (1.0f / 65536.0f) + 1e-30f;
    sc->nodes = (po_node *)xmalloc(sizeof(po_node) * (size_t)(2 * sc->nprim));
    sc->nnodes = 0;
    build_rec(sc, prims, 0, sc->nprim, pad);
    for (int i = 0; i < sc->nprim; ++i) sc->ref[i] = prims[i].id;
    free(prims);
    return sc;
}

po_scene *po_scene_create(const float *verts, const int *tri_mat, int ntris, const float *albedo, int nmat,
                          const po_camera *cam, int accel) {
    if (nmat < 0) nmat = 0;
    po_material *mats = (po_material *)xmalloc(sizeof(po_material) * (size_t)nmat);
    for (int m = 0; m < nmat; ++m) {
        mats[m].kind = PO_LAMBERTIAN;
        mats[m].albedo[0] = albedo[3 * m];
        mats[m].albedo[1] = albedo[3 * m + 1];
        mats[m].albedo[2] = albedo[3 * m + 2];
        mats[m].fuzz = 0.0f;
        mats[m].ir = 1.0f;
    }
    po_scene *sc = po_scene_create2(verts, tri_mat, ntris, NULL, NULL, 0, mats, nmat, cam, accel);
    free(mats);
    return sc;
}

void po_scene_destroy(po_scene *sc) {
    if (!sc) return;
    free(sc->tris); free(sc->sph); free(sc->prim_mat); free(sc->mats); free(sc->nodes); free(sc->ref);
    free(sc);
}

/* Sphere::hit (RayTracer.h:289-314) in the contract's FP32 form: the smaller root if it is
 * >= tmin, else the larger one (the t_max test of :302-305 is the caller's (t, id) ordering).
 * The roots of the reference's quadratic are computed in the precision-robust form (Haines et
 * al., Ray Tracing Gems ch. 7): disc = a (r^2 - |l|^2) with l the centre-to-line vector, and
 * q = -(hb + sign(hb) sqrt(disc)), roots q/a and c/q.  The reference's literal
 * hb^2 - a c cancels catastrophically in FP32 when the origin is far from the sphere (t off
 * by ~1e-3, hit points inside the sphere, paths trapped by self-intersection); in FP64 it
 * does not, and this form reproduces its roots. */
int po_sphere_t(const float c[3], float r2, const float o[3], const float d[3], float tmin, float *t) {
    po_v3 D = ld3(d), oc = vsub(ld3(o), ld3(c));
    float a = fdot(D, D);
    float hb = fdot(oc, D);
    float k = hb / a;
    po_v3 l = v3(fmaf(-k, D.x, oc.x), fmaf(-k, D.y, oc.y), fmaf(-k, D.z, oc.z));
    float disc = a * (r2 - fdot(l, l));
    if (disc < 0.0f) return 0;
    float sq = sqrtf(disc);
    float q = hb >= 0.0f ? -(hb + sq) : sq - hb;
    float cc = fdot(oc, oc) - r2;
    float t0 = q / a, t1 = cc / q;
    float tn = fminf(t0, t1), tf = fmaxf(t0, t1);
    float root = tn;
    if (!(root >= tmin)) {
        root = tf;
        if (!(root >= tmin)) return 0;
    }
    *t = root;
    return 1;
}

static int prim_hit(const po_scene *sc, int id, const float o[3], const float d[3], float tmin, float *t) {
    if (id < sc->ntris) return po_tri_hit(&sc->tris[id], o, d, tmin, t);
    const po_sph *q = &sc->sph[id - sc->ntris];
    float c[3] = {q->c.x, q->c.y, q->c.z};
    return po_sphere_t(c, q->r2, o, d, tmin, t);
}

/* Conservative slab test against a padded box. */
static inline int box_hit(const po_node *nd, po_v3 o, po_v3 inv, float tmin, float tmax) {
    float t0x = (nd->lo[0] - o.x) * inv.x, t1x = (nd->hi[0] - o.x) * inv.x;
    float t0y = (nd->lo[1] - o.y) * inv.y, t1y = (nd->hi[1] - o.y) * inv.y;
    float t0z = (nd->lo[2] - o.z) * inv.z, t1z = (nd->hi[2] - o.z) * inv.z;
    float tn = fmaxf(fmaxf(fminf(t0x, t1x), fminf(t0y, t1y)), fmaxf(fminf(t0z, t1z), tmin));
    float tf = fminf(fminf(fmaxf(t0x, t1x), fmaxf(t0y, t1y)), fminf(fmaxf(t0z, t1z), tmax));
    return tn <= tf * 1.0000005f;
}

/* Closest hit = lexicographic minimum of (t, primitive id) over all primitives with t >= tmin. */
static int scene_closest(const po_scene *sc, po_v3 o, po_v3 d, float tmin, float *t_out) {
    float oo[3] = {o.x, o.y, o.z}, dd[3] = {d.x, d.y, d.z};
    float best = INFINITY;
    int best_id = -1, best_key = 0x7fffffff; /* the kernels' initial (bestT, bestO) */
    if (!sc->accel) {
        for (int id = 0; id < sc->nprim; ++id) {
            float t;
            if (!prim_hit(sc, id, oo, dd, tmin, &t)) continue;
            if (t < best || (t == best && id < best_key)) { best = t; best_id = best_key = id; }
        }
        *t_out = best;
        return best_id;
    }
    po_v3 inv = v3(1.0f / d.x, 1.0f / d.y, 1.0f / d.z);
    int stack[128];
    int sp = 0;
    stack[sp++] = 0;
    while (sp > 0) {
        const po_node *nd = &sc->nodes[stack[--sp]];
        if (!box_hit(nd, o, inv, tmin, best)) continue;
        if (nd->right < 0) {
            for (int i = nd->left; i < nd->left - nd->right; ++i) {
                int id = sc->ref[i];
                float t;
                if (!prim_hit(sc, id, oo, dd, tmin, &t)) continue;
                if (t < best || (t == best && id < best_key)) { best = t; best_id = best_key = id; }
            }
        } else {
            stack[sp++] = nd->right;
            stack[sp++] = nd->left;
        }
    }
    *t_out = best;
    return best_id;
}

static inline po_v3 vneg(po_v3 a) { return v3(-a.x, -a.y, -a.z); }

/* reflect — RayTracer.h:174-176: v - (2*dot(v,n))*n. */
static inline po_v3 reflect3(po_v3 v, po_v3 n) {
    float k = 2.0f * fdot(v, n);
    return v3(v.x - k * n.x, v.y - k * n.y, v.z - k * n.z);
}

/* refract — RayTracer.h:178-183, cos_theta = min(dot(-uv, n), 1). */
static inline po_v3 refract3(po_v3 uv, po_v3 n, float ratio) {
    float c = fminf(fdot(vneg(uv), n), 1.0f);
    po_v3 perp = v3((uv.x + c * n.x) * ratio, (uv.y + c * n.y) * ratio, (uv.z + c * n.z) * ratio);
    float par = -sqrtf(fabsf(1.0f - fdot(perp, perp)));
    return v3(perp.x + par * n.x, perp.y + par * n.y, perp.z + par * n.z);
}

void po_reflect(const float v[3], const float n[3], float out[3]) { st3(out, reflect3(ld3(v), ld3(n))); }
void po_refract(const float uv[3], const float n[3], float ratio, float out[3]) {
    st3(out, refract3(ld3(uv), ld3(n), ratio));
}

/* Scatter at a hit (ray_color :585-590 with the material's scatter, :473-540).  Updates the
 * ray and the throughput; returns 0 when the material absorbs (Metal below the surface). */
int po_scatter(const po_scene *sc, int prim, float t, float o[3], float d[3], uint32_t *st, float thr[3]) {
    po_v3 O = ld3(o), D = ld3(d);
    po_v3 p = v3(fmaf(t, D.x, O.x), fmaf(t, D.y, O.y), fmaf(t, D.z, O.z)); /* Ray::at */
    po_v3 on;
    if (prim < sc->ntris) {
        on = sc->tris[prim].n;
    } else { /* (p - center) / radius, :308 */
        const po_sph *q = &sc->sph[prim - sc->ntris];
        on = v3((p.x - q->c.x) / q->r, (p.y - q->c.y) / q->r, (p.z - q->c.z) / q->r);
    }
    int front = fdot(D, on) < 0.0f; /* set_face_normal, :215-218 */
    po_v3 n = front ? on : vneg(on);
    const po_material *m = &sc->mats[sc->prim_mat[prim]];
    po_v3 sd;
    if (m->kind == PO_METAL) { /* Metal::scatter, :496-501 */
        po_v3 ud = vscale(D, 1.0f / sqrtf(fdot(D, D)));
        po_v3 refl = reflect3(ud, n);
        float r[3];
        po_random_in_unit_sphere(st, r);
        sd = v3(refl.x + m->fuzz * r[0], refl.y + m->fuzz * r[1], refl.z + m->fuzz * r[2]);
        if (!(fdot(sd, n) > 0.0f)) return 0;
        thr[0] *= m->albedo[0]; thr[1] *= m->albedo[1]; thr[2] *= m->albedo[2];
    } else if (m->kind == PO_DIELECTRIC) { /* Dielectric::scatter, :512-530 */
        float ratio = front ? (1.0f / m->ir) : m->ir;
        po_v3 ud = vscale(D, 1.0f / sqrtf(fdot(D, D)));
        float cos_t = fminf(fdot(vneg(ud), n), 1.0f);
        float sin_t = sqrtf(1.0f - cos_t * cos_t);
        int refl = ratio * sin_t > 1.0f;
        if (!refl) { /* reflectance (Schlick, :533-538) > random_double(), drawn only here (||) */
            float r0 = (1.0f - ratio) / (1.0f + ratio);
            r0 = r0 * r0;
            float x = 1.0f - cos_t, x2 = x * x;
            float sch = r0 + (1.0f - r0) * (x2 * x2 * x);
            refl = sch > po_rand01(st);
        }
        if (refl) {
            sd = reflect3(ud, n);
        } else {
            sd = refract3(ud, n, ratio);
        }
    } else { /* Lambertian::scatter, :477-484 */
        float r[3];
        po_random_in_unit_sphere(st, r);
        po_v3 rv = ld3(r);
        po_v3 ru = vscale(rv, 1.0f / sqrtf(fdot(rv, rv)));
        sd = vadd(n, ru);
        if (fdot(sd, sd) < 1e-8f) sd = n;
        thr[0] *= m->albedo[0]; thr[1] *= m->albedo[1]; thr[2] *= m->albedo[2];
    }
    st3(o, p);
    st3(d, sd);
    return 1;
}

/* One (pixel, frame) sample: RenderWorker::render's u/v (RayTracerFboItem.cpp:109-110),
 * Camera::get_ray, then ray_color (RayTracer.h:579-596) unrolled into a throughput loop. */
void po_mesh_sample(const po_scene *sc, int width, int height, int x, int y, int frame, int max_depth,
                    float rgb[3], int *segs_out) {
    uint32_t st = po_pixel_seed(x, y, width, frame);
    float invw = 1.0f / (float)(width - 1 > 1 ? width - 1 : 1);
    float invh = 1.0f / (float)(height - 1 > 1 ? height - 1 : 1);
    float s = ((float)x + po_rand01(&st)) * invw;
    float t = ((float)y + po_rand01(&st)) * invh;
    float of[3], df[3];
    po_camera_get_ray(&sc->cam, s, t, &st, of, df);
    float thr[3] = {1.0f, 1.0f, 1.0f};
    po_v3 L = v3(0.0f, 0.0f, 0.0f);
    int segs = 0;
    for (int depth = 0; depth < max_depth; ++depth) {
        float th;
        po_v3 o = ld3(of), d = ld3(df);
        int hi = scene_closest(sc, o, d, 0.001f, &th);
        ++segs;
        if (hi < 0) { /* miss: sky gradient, RayTracer.h:593-595 */
            float uy = (1.0f / sqrtf(fdot(d, d))) * d.y;
            float a = 0.5f * (uy + 1.0f);
            float b = 1.0f - a;
            po_v3 sky = v3(fmaf(a, 0.5f, b), fmaf(a, 0.7f, b), fmaf(a, 1.0f, b));
            L = vmul(ld3(thr), sky);
            break;
        }
        if (depth + 1 >= max_depth) break; /* the next ray_color call returns 0 (:582-583) */
        if (!po_scatter(sc, hi, th, of, df, &st, thr)) break; /* absorbed: 0 (:590) */
    }
    st3(rgb, L);
    if (segs_out) *segs_out = segs;
}

static void mesh_pixel(const po_scene *sc, int x, int y, int width, int height, int first, int count,
                       int max_depth, float acc[4], uint32_t *out, uint64_t *segs) {
    for (int f = first; f < first + count; ++f) {
        float L[3];
        int ns = 0;
        po_mesh_sample(sc, width, height, x, y, f, max_depth, L, &ns);
        *segs += (uint64_t)ns;
        *out = po_accumulate(acc, L, f);
    }
}

void po_mesh_frames(const po_scene *sc, int width, int height, int y0, int y1, int first_frame, int count,
                    int max_depth, float *accum, uint32_t *out, uint64_t *stats, int nthreads) {
    run_jobs(1, sc, width, height, y0, y1, first_frame, count, max_depth, accum, out, stats, nthreads);
}
