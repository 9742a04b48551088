/*
 * oracle/oracle.h -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the reference's two per-pixel hot paths, used as the
 * parity checker for the HIP kernels and as the timed CPU baseline
 * ("cpu_baseline.kind = port" in bench.py).  Only tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg may load this library; the product path
 * (se-195-project-ray-tracer_amd/) never links or calls it.
 *
 *   Whitted : raytracer3.0.06.no_rec.samp/scene.cpp + raytracer.cpp
 *   smallpt : smallptgpu-v1.6/geomfunc.h + smallptCPU.cpp + displayfunc.cpp
 *   queue   : Raytracer3.2.03/raytracer/OpenCL Raytracer/raytracer_non_OpenCL.c
 *             + scene.c (the 3.2.x queue tracer's CPU path)
 *
 * Parity pin: SURVEY.md §8(c) known-answer hashes produced by the reference
 * itself (tests/golden/known_answers.json) plus oracle/_ref builds of the
 * reference sources that compile without stand-ins (see oracle/Makefile).
 *
 * Struct layouts are byte-identical to the reference's:
 *   Primitive 96 B  raytracer.h:23-32 (+ Material :18-21, plane common.h:49-53)
 *   Sphere    44 B  smallptgpu-v1.6/geom.h:43-47
 *   Camera    60 B  smallptgpu-v1.6/camera.h:29-34
 *   Primitive_2 96 B Raytracer3.2.03/.../raytracer_non_OpenCL.c:67-81
 */
#ifndef RT_ORACLE_H
#define RT_ORACLE_H

#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct { float x, y, z; } orv3;

/* raytracer.h:23-32 */
typedef struct {
    int32_t type;          /* PRIMTYPE: SPHERE=1, PLANE=2, BOX=3 (raytracer.h:12-16) */
    int32_t m_Light;
    orv3    m_Centre;
    float   m_SqRadius, m_Radius, m_RRadius;
    orv3    plane_N;       /* plane m_Plane (common.h:49-53) */
    float   plane_D;
    float   plane_cell[4];
    orv3    m_Color;       /* Material (raytracer.h:18-21) */
    float   m_Refl, m_Refr, m_Diff, m_Spec, m_RIndex;
} or_primitive;

/* smallptgpu-v1.6/geom.h:43-47 */
typedef struct {
    float rad;
    orv3  p, e, c;
    int32_t refl;          /* enum Refl: DIFF=0, SPEC=1, REFR=2 */
} or_sphere;

/* smallptgpu-v1.6/camera.h:29-34 */
typedef struct {
    orv3 orig, target;
    orv3 dir, x, y;
} or_camera;

/* ---------------- Whitted (raytracer3.0.06.no_rec.samp) ---------------- */

/* Scene_InitScene (scene.cpp:217-272): writes the 17 primitives, returns count. */
int  orw_scene_init(or_primitive *out, int cap);

/* Engine_InitRender + Engine_Render (raytracer.cpp:278-530) over rows
 * [row_begin,row_end) (reference: [20, H-70)).  Requires row_begin >= 20:
 * the reference's m_SY recurrence starts at row 20.  counters (nullable):
 *   [0] Engine_Raytrace calls (traced rays)   [1] shadow rays
 *   [2] Primitive_Intersect calls             [3] TIR-with-traced-child events
 * nthreads: 1 = the reference's single thread; >1 = OpenMP over rows. */
void orw_render(const or_primitive *prims, int n, uint32_t *dest, int w, int h,
                int row_begin, int row_end, uint64_t *counters, int nthreads);
/* GPU-semantics variant: raytrace_kernel of openCLcode.cl (rows [20, min(530,h))). */
void orw_render_ocl(const or_primitive *prims, int n, uint32_t *dest, int w, int h,
                    uint64_t *counters, int nthreads);

/* Single primitive helpers, exposed for unit tests (scene.cpp:34-53,125-190). */
int  orw_primitive_intersect(const or_primitive *p, const float ray[6], float *dist);
void orw_primitive_normal(const or_primitive *p, const float pos[3], float out[3]);

/* ---------------- smallpt (smallptgpu-v1.6) ---------------- */

/* CornellSpheres (scene.h:29-40), returns count (9). */
int  ors_cornell(or_sphere *out, int cap);
/* UpdateCamera (displayfunc.cpp:182-195): fills dir/x/y from orig/target. */
void ors_update_camera(or_camera *cam, int width, int height);
/* AllocateBuffers seed fill (smallptGPU.cpp:105-110): srand(seed) then
 * seeds[i] = max(rand(), 2) for i < n. */
void ors_seeds_init(uint32_t *seeds, size_t n, unsigned seed);
/* GetRandom (simplernd.h:34-48) */
float ors_get_random(uint32_t *s0, uint32_t *s1);
/* UpdateRenderingCPU (smallptCPU.cpp:77-132) for rows [row_begin,row_end),
 * samples first_sample .. first_sample+nsamples-1.  direct_lighting selects
 * RadianceDirectLighting (geomfunc.h:340-483) instead of RadiancePathTracing.
 * counters (nullable): [0] Intersect calls  [1] IntersectP calls
 *                      [2] sphere tests     [3] samples */
void ors_render(const or_sphere *s, unsigned n, const or_camera *cam,
                float *colors, uint32_t *seeds, uint32_t *pixels, int w, int h,
                int row_begin, int row_end, int first_sample, int nsamples,
                int direct_lighting, uint64_t *counters, int nthreads);

/* scene_build_complex.pl logic (HyperSphere) with the given max depth;
 * writes up to cap spheres in the Perl script's emission order, returns the
 * number it would emit. */
int  ors_hypersphere(or_sphere *out, int cap, double max_depth);

/* ---------------- queue tracer (Raytracer3.2.03) ---------------- */

typedef struct { float x, y, z, w; } orq_f4;       /* float_4, raytracer_non_OpenCL.c:42-44 */

/* Primitive_2, raytracer_non_OpenCL.c:67-81 (bool is_light: one byte) */
typedef struct {
    orq_f4  m_color;
    float   m_refl, m_diff, m_refr, m_refr_index, m_spec, dummy_3;
    int32_t type;          /* prim_type: PLANE=0, SPHERE=1 */
    uint8_t is_light;
    uint8_t pad_[3];
    orq_f4  normal, center;
    float   depth, radius, sq_radius, r_radius;
} orq_primitive;

/* create_scene (scene.c:48-97, CHOOSE_SCENE 0) after raytracer.c:721-746's
 * copy into Primitive_2; returns 17. */
int  orq_scene_init(orq_primitive *out, int cap);
/* raytracer_non_kernel (raytracer_non_OpenCL.c:285-449) over rows
 * [row_begin,row_end) of the w x h frame; pixels: uchar_4 (r,g,b,0) per pixel.
 * counters (nullable): [0] rays traced (raytrace calls)  [1] shadow rays
 *   [2] intersect calls  [3] undefined-behaviour events (see queue_oracle.c). */
void orq_render(const orq_primitive *P, int n, uint8_t *pixels, int w, int h, int row_begin, int row_end,
                uint64_t *counters, int nthreads);

/* FNV-1a-64 over bytes, as used for the SURVEY.md §8(c) known answers. */
uint64_t or_fnv1a64(const void *data, size_t nbytes);

#ifdef __cplusplus
}
#endif
#endif
