/*
 * pt_oracle.h — TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement (plain C, FP32, deterministic hash RNG) of the reference path
 * tracer's hot path, used ONLY by tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg as the checker.  The product path (libhippt.so) never links or
 * calls anything in oracle/.
 *
 * Two algorithms are restated:
 *
 *  1. "sphere4" — the reference GPU megakernel, CudaPathTracerKernel.cu:23-179
 *     (hash32/rand01 :23-35, normalize :53-59, randomInUnitSphere :61-68,
 *      hitSphere :70-98, traceRay :100-134, pathTraceKernel :136-179).
 *     This is what the legacy cudaPathTracer* ABI renders.
 *
 *  2. "mesh" — the reference CPU path tracer's shading model
 *     (RayTracer.h: Camera :543-576, ray_color :579-596, Lambertian :473-488,
 *      Metal :490-504, Dielectric :506-540, Sphere::hit :289-314,
 *      random_in_unit_sphere :155-161, random_in_unit_disk :163-169,
 *      set_face_normal :215-218) over triangles and spheres, in FP32, driven by the GPU
 *     kernels' integer-seeded hash RNG (CudaPathTracerKernel.cu:23-35,144) and
 *     accumulated/quantised per CudaPathTracerKernel.cu:157-178.  Triangles are
 *     new capability (the reference has only spheres); the closest hit is
 *     defined BVH-independently as the lexicographic minimum of (t, primitive id)
 *     over all primitives (see DESIGN.md "Semantic contract").
 *
 * Parity pinning: the FP32 helpers are checked against FP64 golden vectors
 * produced by compiling the reference RayTracer.h (oracle/ref_harness.cpp) and
 * against the reference's own gtest known answers (tests/unit/*.cpp); see
 * tests/golden/ and DESIGN.md §Oracle.
 */
#ifndef PT_ORACLE_H
#define PT_ORACLE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct { float x, y, z; } po_v3;

/* Camera in the form the kernels consume (RayTracer.h:545-561 computed in FP64,
 * stored as FP32). */
typedef struct {
    po_v3 origin, llc, horizontal, vertical, u, v;
    float lens_radius;
    float pad_;
} po_camera;

/* Triangle in the intersection form: v0, e1 = v1-v0, e2 = v2-v0, unit normal. */
typedef struct { po_v3 v0, e1, e2, n; } po_tri;

/* ---- RNG (CudaPathTracerKernel.cu:23-35) ---- */
uint32_t po_hash32(uint32_t x);
float po_rand01(uint32_t *state);
uint32_t po_pixel_seed(int x, int y, int width, int frame);

/* ---- helpers exposed for known-answer tests ---- */
void po_camera_build(const double lookfrom[3], const double lookat[3], const double vup[3],
                     double vfov_deg, double aspect, double aperture, double focus_dist,
                     po_camera *out);
void po_tri_setup(const float v[9], po_tri *out);
/* Möller–Trumbore restated with the contract's division-free edge tests;
 * returns 1 and writes *t on a hit with t >= tmin. */
int po_tri_hit(const po_tri *tri, const float o[3], const float d[3], float tmin, float *t);
/* RayTracer.h Sphere::hit (:289-314) in FP32: returns 1 on hit, writes t, normal (face-forwarded), front. */
int po_sphere_hit(const float c[3], float r, const float o[3], const float d[3], float tmin, float tmax,
                  float *t, float n[3], int *front);
/* RayTracer.h AABB::hit (:229-244) in FP32. */
int po_aabb_hit(const float lo[3], const float hi[3], const float o[3], const float d[3], float tmin, float tmax);
/* random_in_unit_sphere / random_in_unit_disk driven by the hash RNG. */
void po_random_in_unit_sphere(uint32_t *state, float p[3]);
void po_random_in_unit_disk(uint32_t *state, float p[3]);
/* Camera::get_ray (RayTracer.h:563-567). */
void po_camera_get_ray(const po_camera *cam, float s, float t, uint32_t *state, float o[3], float d[3]);
/* Closest hit over a triangle list, brute force.  Returns index (into tris) or -1. */
int po_closest_hit(const po_tri *tris, const int *orig_ids, int ntris, const float o[3], const float d[3],
                   float tmin, float *t_out);

/* ---- sphere4: the legacy CUDA kernel (CudaPathTracerKernel.cu:136-179) ---- */
/* Renders one frame for rows [y0, y1) of a width x height image.
 * accum: (y1-y0)*width*4 floats (in/out), out: (y1-y0)*width ARGB words. */
void po_sphere4_frames(int width, int height, int y0, int y1, int first_frame, int count, int max_depth,
                       float *accum, uint32_t *out, int nthreads);

/* ---- mesh path ---- */
typedef struct po_scene po_scene;
/* Materials (RayTracer.h:473-540): kind PO_LAMBERTIAN uses albedo; PO_METAL albedo + fuzz
 * (clamped to <= 1 as Metal's constructor does); PO_DIELECTRIC ir. */
enum { PO_LAMBERTIAN = 0, PO_METAL = 1, PO_DIELECTRIC = 2 };
typedef struct { int kind; float albedo[3]; float fuzz; float ir; } po_material;
/* Triangles (verts ntris*9, tri_mat) and spheres (cx, cy, cz, r per sphere, sph_mat); the
 * primitive id orders ties: triangles 0..ntris-1, then spheres. */
po_scene *po_scene_create2(const float *verts, const int *tri_mat, int ntris, const float *spheres,
                           const int *sph_mat, int nsph, const po_material *mats, int nmat, const po_camera *cam,
                           int accel);
/* Sphere::hit root selection in the contract's FP32 form (no t_max). */
int po_sphere_t(const float c[3], float r2, const float o[3], const float d[3], float tmin, float *t);
/* reflect / refract (RayTracer.h:174-183) in the contract's FP32 form. */
void po_reflect(const float v[3], const float n[3], float out[3]);
void po_refract(const float uv[3], const float n[3], float ratio, float out[3]);
/* Scatter at primitive `prim` hit at t: updates o/d/thr; 0 = absorbed. */
int po_scatter(const po_scene *sc, int prim, float t, float o[3], float d[3], uint32_t *state, float thr[3]);
/* Lambertian-only triangle scene: verts: ntris*9 floats (v0,v1,v2), tri_mat: ntris ints, albedo: nmat*3
 * floats. accel: 0 = brute force, 1 = oracle-private median-split BVH (results identical by
 * construction; tested). */
po_scene *po_scene_create(const float *verts, const int *tri_mat, int ntris, const float *albedo, int nmat,
                          const po_camera *cam, int accel);
void po_scene_destroy(po_scene *sc);
/* Renders `count` frames starting at first_frame for rows [y0, y1), running-average accumulation
 * exactly as repeated single-frame launches.  stats[0] += segments traced (closest-hit queries),
 * stats[1] += pixel-samples. */
void po_mesh_frames(const po_scene *sc, int width, int height, int y0, int y1, int first_frame, int count,
                    int max_depth, float *accum, uint32_t *out, uint64_t *stats, int nthreads);
/* Radiance of a single (pixel, frame) sample; segs (optional) receives the segment count. */
void po_mesh_sample(const po_scene *sc, int width, int height, int x, int y, int frame, int max_depth,
                    float rgb[3], int *segs);

/* Running-average + tonemap step (CudaPathTracerKernel.cu:157-178). */
uint32_t po_accumulate(float acc[4], const float sample[3], int frame_index);
/* RGBA8 UNORM words (GL / Vulkan backends) of n accumulated RGBA float colours. */
void po_rgba8(const float *acc4, long long n, uint32_t *out);

#ifdef __cplusplus
}
#endif
#endif
