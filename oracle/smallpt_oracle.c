/*
 * oracle/smallpt_oracle.c -- TEST INFRASTRUCTURE ONLY (see oracle.h).
 *
 * Plain-C restatement of the smallpt CPU path of smallptgpu-v1.6
 * (SURVEY.md §8(a) rows S1-S9): geomfunc.h radiance estimators driven by the
 * UpdateRenderingCPU pixel body (smallptCPU.cpp:84-123).  Evaluation order
 * follows the reference macros in vec.h; the two GetRandom() arguments of
 * UniformSampleSphere (geomfunc.h:138) are drawn right-to-left, as g++ (the
 * oracle compiler, SURVEY.md §7 "Argument evaluation order") evaluates them.
 * libm calls are the float overloads the C++ reference resolves to
 * (sqrtf, sinf/cosf, fabsf, powf).
 */
#include <math.h>
#include <stdlib.h>
#include <string.h>
#include "oracle.h"

#define EPSILON 0.01f                     /* geom.h:29 */
#define FLOAT_PI 3.14159265358979323846f  /* geom.h:30 */
#define DIFF 0
#define SPEC 1
#define REFR 2

typedef orv3 Vec;
typedef struct { Vec o, d; } Ray;         /* geom.h:32-34 */

/* vec.h:31-44 (macro order of evaluation kept) */
static inline Vec vinit(float a, float b, float c) { Vec v = {a, b, c}; return v; }
static inline Vec vadd(Vec a, Vec b) { return vinit(a.x + b.x, a.y + b.y, a.z + b.z); }
static inline Vec vsub(Vec a, Vec b) { return vinit(a.x - b.x, a.y - b.y, a.z - b.z); }
static inline Vec vmul(Vec a, Vec b) { return vinit(a.x * b.x, a.y * b.y, a.z * b.z); }
static inline Vec vsmul(float k, Vec b) { return vinit(k * b.x, k * b.y, k * b.z); }
static inline float vdot(Vec a, Vec b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
static inline Vec vnorm(Vec v) { float l = 1.f / sqrtf(vdot(v, v)); return vsmul(l, v); }
static inline Vec vxcross(Vec a, Vec b)
{
    return vinit(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
static inline int viszero(Vec v) { return (v.x == 0.f) && (v.x == 0.f) && (v.z == 0.f); } /* vec.h:44 (tests x twice) */
#define OMAX(a, b) (((a) > (b)) ? (a) : (b))                         /* vec.h:52 */
#define OCLAMP(x, a, b) ((x) < (a) ? (a) : ((x) > (b) ? (b) : (x)))  /* vec.h:47 */
#define OSIGN(x) ((x) > 0 ? 1 : -1)                                  /* vec.h:59 */

typedef struct { uint64_t isect, isectp, tests, samples; } scount;

/* GetRandom, simplernd.h:34-48 */
float ors_get_random(uint32_t *seed0, uint32_t *seed1)
{
    *seed0 = 36969u * ((*seed0) & 65535u) + ((*seed0) >> 16);
    *seed1 = 18000u * ((*seed1) & 65535u) + ((*seed1) >> 16);
    uint32_t ires = ((*seed0) << 16) + (*seed1);
    union { float f; uint32_t ui; } res;
    res.ui = (ires & 0x007fffffu) | 0x40000000u;
    return (res.f - 2.f) / 2.f;
}

/* SphereIntersect, geomfunc.h:32-59 */
static float sphere_intersect(const or_sphere *s, const Ray *r)
{
    Vec op = vsub(s->p, r->o);
    float b = vdot(op, r->d);
    float det = b * b - vdot(op, op) + s->rad * s->rad;
    if (det < 0.f) return 0.f;
    det = sqrtf(det);
    float t = b - det;
    if (t > EPSILON) return t;
    t = b + det;
    if (t > EPSILON) return t;
    return 0.f;
}

/* UniformSampleSphere, geomfunc.h:61-69 */
static Vec uniform_sample_sphere(float u1, float u2)
{
    const float zz = 1.f - 2.f * u1;
    const float r = sqrtf(OMAX(0.f, 1.f - zz * zz));
    const float phi = 2.f * FLOAT_PI * u2;
    const float xx = r * cosf(phi);
    const float yy = r * sinf(phi);
    return vinit(xx, yy, zz);
}

/* Intersect, geomfunc.h:71-92: i descending, strict '<' (highest index wins ties) */
static int intersect(const or_sphere *S, unsigned n, const Ray *r, float *t, unsigned *id, scount *c)
{
    float inf = (*t) = 1e20f;
    unsigned i = n;
    c->isect++;
    c->tests += n;
    for (; i--;) {
        const float d = sphere_intersect(&S[i], r);
        if ((d != 0.f) && (d < *t)) { *t = d; *id = i; }
    }
    return (*t < inf);
}

/* IntersectP, geomfunc.h:94-110 */
static int intersect_p(const or_sphere *S, unsigned n, const Ray *r, float maxt, scount *c)
{
    unsigned i = n;
    c->isectp++;
    for (; i--;) {
        c->tests++;
        const float d = sphere_intersect(&S[i], r);
        if ((d != 0.f) && (d < maxt)) return 1;
    }
    return 0;
}

/* SampleLights, geomfunc.h:112-165 */
static Vec sample_lights(const or_sphere *S, unsigned n, uint32_t *s0, uint32_t *s1,
                         Vec hit, Vec normal, scount *c)
{
    Vec result = vinit(0.f, 0.f, 0.f);
    for (unsigned i = 0; i < n; i++) {
        const or_sphere *light = &S[i];
        if (!viszero(light->e)) {
            Ray shadow;
            shadow.o = hit;
            /* UniformSampleSphere(GetRandom(), GetRandom(), ..): g++ draws the
             * second argument first. */
            float u2 = ors_get_random(s0, s1);
            float u1 = ors_get_random(s0, s1);
            Vec unit = uniform_sample_sphere(u1, u2);
            Vec sp = vsmul(light->rad, unit);
            sp = vadd(sp, light->p);
            shadow.d = vsub(sp, hit);
            const float len = sqrtf(vdot(shadow.d, shadow.d));
            shadow.d = vsmul(1.f / len, shadow.d);
            float wo = vdot(shadow.d, unit);
            if (wo > 0.f) continue;
            wo = -wo;
            const float wi = vdot(shadow.d, normal);
            if ((wi > 0.f) && (!intersect_p(S, n, &shadow, len - EPSILON, c))) {
                Vec col = light->e;
                const float s = (4.f * FLOAT_PI * light->rad * light->rad) * wi * wo / (len * len);
                col = vsmul(s, col);
                result = vadd(result, col);
            }
        }
    }
    return result;
}

/* RadiancePathTracing (geomfunc.h:167-338) and, with dl != 0,
 * RadianceDirectLighting (geomfunc.h:340-483). */
static Vec radiance(const or_sphere *S, unsigned n, Ray ray, uint32_t *s0, uint32_t *s1,
                    int dl, scount *c)
{
    Vec rad = vinit(0.f, 0.f, 0.f);
    Vec thr = vinit(1.f, 1.f, 1.f);
    int specular_bounce = 1;
    for (unsigned depth = 0;; ++depth) {
        if (depth > 6) return rad;
        float t;
        unsigned id = 0;
        if (!intersect(S, n, &ray, &t, &id, c)) return rad;
        const or_sphere *obj = &S[id];
        Vec hit = vsmul(t, ray.d);
        hit = vadd(ray.o, hit);
        Vec normal = vsub(hit, obj->p);
        normal = vnorm(normal);
        const float dp = vdot(normal, ray.d);
        const float inv_sign_dp = -1.f * OSIGN(dp);
        Vec nl = vsmul(inv_sign_dp, normal);
        Vec ecol = obj->e;
        if (!viszero(ecol)) {
            if (specular_bounce) {
                ecol = vsmul(fabsf(dp), ecol);
                ecol = vmul(thr, ecol);
                rad = vadd(rad, ecol);
            }
            return rad;
        }
        if (obj->refl == DIFF) {
            specular_bounce = 0;
            thr = vmul(thr, obj->c);
            Vec ld = sample_lights(S, n, s0, s1, hit, nl, c);
            ld = vmul(thr, ld);
            rad = vadd(rad, ld);
            if (dl) return rad;                                /* geomfunc.h:413-414 */
            float r1 = 2.f * FLOAT_PI * ors_get_random(s0, s1);
            float r2 = ors_get_random(s0, s1);
            float r2s = sqrtf(r2);
            Vec w = nl;
            Vec a = (fabsf(w.x) > .1f) ? vinit(0.f, 1.f, 0.f) : vinit(1.f, 0.f, 0.f);
            Vec u = vxcross(a, w);
            u = vnorm(u);
            Vec v = vxcross(w, u);
            u = vsmul(cosf(r1) * r2s, u);
            v = vsmul(sinf(r1) * r2s, v);
            Vec nd = vadd(u, v);
            w = vsmul(sqrtf(1 - r2), w);
            nd = vadd(nd, w);
            ray.o = hit;
            ray.d = nd;
            continue;
        } else if (obj->refl == SPEC) {
            specular_bounce = 1;
            Vec nd = vsmul(2.f * vdot(normal, ray.d), normal);
            nd = vsub(ray.d, nd);
            thr = vmul(thr, obj->c);
            ray.o = hit;
            ray.d = nd;
            continue;
        } else {
            specular_bounce = 1;
            Vec nd = vsmul(2.f * vdot(normal, ray.d), normal);
            nd = vsub(ray.d, nd);
            Ray refl_ray = {hit, nd};
            int into = (vdot(normal, nl) > 0);
            float nc = 1.f, nt = 1.5f;
            float nnt = into ? nc / nt : nt / nc;
            float ddn = vdot(ray.d, nl);
            float cos2t = 1.f - nnt * nnt * (1.f - ddn * ddn);
            if (cos2t < 0.f) {
                thr = vmul(thr, obj->c);
                ray = refl_ray;
                continue;
            }
            float kk = (into ? 1 : -1) * (ddn * nnt + sqrtf(cos2t));
            Vec nkk = vsmul(kk, normal);
            Vec td = vsmul(nnt, ray.d);
            td = vsub(td, nkk);
            td = vnorm(td);
            float a = nt - nc;
            float b = nt + nc;
            float R0 = a * a / (b * b);
            float cc = 1 - (into ? -ddn : vdot(td, normal));
            float Re = R0 + (1 - R0) * cc * cc * cc * cc * cc;
            float Tr = 1.f - Re;
            float P = .25f + .5f * Re;
            float RP = Re / P;
            float TP = Tr / (1.f - P);
            if (ors_get_random(s0, s1) < P) {
                thr = vsmul(RP, thr);
                thr = vmul(thr, obj->c);
                ray = refl_ray;
            } else {
                thr = vsmul(TP, thr);
                thr = vmul(thr, obj->c);
                ray.o = hit;
                ray.d = td;
            }
            continue;
        }
    }
}

/* toInt, vec.h:62 */
static int to_int(float x)
{
    return (int)(powf(OCLAMP(x, 0.f, 1.f), 1.f / 2.2f) * 255.f + .5f);
}

void ors_render(const or_sphere *S, unsigned n, const or_camera *cam, float *colors,
                uint32_t *seeds, uint32_t *pixels, int width, int height, int row_begin,
                int row_end, int first_sample, int nsamples, int dl, uint64_t *counters,
                int nthreads)
{
    const float invWidth = 1.f / width;                         /* smallptCPU.cpp:80-81 */
    const float invHeight = 1.f / height;
    uint64_t t_isect = 0, t_isectp = 0, t_tests = 0, t_samples = 0;
    if (nthreads < 1) nthreads = 1;
    if (row_begin < 0) row_begin = 0;
    if (row_end > height) row_end = height;
#pragma omp parallel for schedule(dynamic, 1) num_threads(nthreads) \
    reduction(+ : t_isect, t_isectp, t_tests, t_samples) if (nthreads > 1)
    for (int y = row_begin; y < row_end; y++) {
        scount c = {0, 0, 0, 0};
        for (int x = 0; x < width; x++) {
            const int i = (height - y - 1) * width + x;         /* :86 flipped slot */
            const int i2 = 2 * i;
            Vec *col = (Vec *)&colors[3 * (size_t)i];
            for (int k = 0; k < nsamples; k++) {
                const int current = first_sample + k;
                const float r1 = ors_get_random(&seeds[i2], &seeds[i2 + 1]) - .5f;
                const float r2 = ors_get_random(&seeds[i2], &seeds[i2 + 1]) - .5f;
                const float kcx = (x + r1) * invWidth - .5f;
                const float kcy = (y + r2) * invHeight - .5f;
                Vec rdir = vinit(cam->x.x * kcx + cam->y.x * kcy + cam->dir.x,
                                 cam->x.y * kcx + cam->y.y * kcy + cam->dir.y,
                                 cam->x.z * kcx + cam->y.z * kcy + cam->dir.z);
                Vec rorig = vsmul(0.1f, rdir);
                rorig = vadd(rorig, cam->orig);
                rdir = vnorm(rdir);
                Ray ray = {rorig, rdir};
                Vec r = radiance(S, n, ray, &seeds[i2], &seeds[i2 + 1], dl, &c);
                if (current == 0) {                             /* :110-118 */
                    *col = r;
                } else {
                    const float k1 = current;
                    const float k2 = 1.f / (k1 + 1.f);
                    col->x = (col->x * k1 + r.x) * k2;
                    col->y = (col->y * k1 + r.y) * k2;
                    col->z = (col->z * k1 + r.z) * k2;
                }
                c.samples++;
            }
            if (nsamples > 0)                                   /* :120-122 */
                pixels[(size_t)y * width + x] = (uint32_t)(to_int(col->x) | (to_int(col->y) << 8) |
                                                           (to_int(col->z) << 16));
        }
        t_isect += c.isect; t_isectp += c.isectp; t_tests += c.tests; t_samples += c.samples;
    }
    if (counters) {
        counters[0] = t_isect; counters[1] = t_isectp;
        counters[2] = t_tests; counters[3] = t_samples;
    }
}

/* CornellSpheres, scene.h:29-40 */
int ors_cornell(or_sphere *out, int cap)
{
    static const float WALL_RAD = 1e4f;
    const or_sphere cs[9] = {
        {WALL_RAD, {WALL_RAD + 1.f, 40.8f, 81.6f}, {0.f, 0.f, 0.f}, {.75f, .25f, .25f}, DIFF},
        {WALL_RAD, {-WALL_RAD + 99.f, 40.8f, 81.6f}, {0.f, 0.f, 0.f}, {.25f, .25f, .75f}, DIFF},
        {WALL_RAD, {50.f, 40.8f, WALL_RAD}, {0.f, 0.f, 0.f}, {.75f, .75f, .75f}, DIFF},
        {WALL_RAD, {50.f, 40.8f, -WALL_RAD + 270.f}, {0.f, 0.f, 0.f}, {0.f, 0.f, 0.f}, DIFF},
        {WALL_RAD, {50.f, WALL_RAD, 81.6f}, {0.f, 0.f, 0.f}, {.75f, .75f, .75f}, DIFF},
        {WALL_RAD, {50.f, -WALL_RAD + 81.6f, 81.6f}, {0.f, 0.f, 0.f}, {.75f, .75f, .75f}, DIFF},
        {16.5f, {27.f, 16.5f, 47.f}, {0.f, 0.f, 0.f}, {.9f, .9f, .9f}, SPEC},
        {16.5f, {73.f, 16.5f, 78.f}, {0.f, 0.f, 0.f}, {.9f, .9f, .9f}, REFR},
        {7.f, {50.f, 81.6f - 15.f, 81.6f}, {12.f, 12.f, 12.f}, {0.f, 0.f, 0.f}, DIFF},
    };
    if (cap < 9) return -1;
    memcpy(out, cs, sizeof(cs));
    return 9;
}

/* UpdateCamera, displayfunc.cpp:182-195 (fov computed in double, narrowed) */
void ors_update_camera(or_camera *cam, int width, int height)
{
    cam->dir = vsub(cam->target, cam->orig);
    cam->dir = vnorm(cam->dir);
    const Vec up = {0.f, 1.f, 0.f};
    const float fov = (float)((3.14159265358979323846 / 180.f) * 45.f);
    cam->x = vxcross(cam->dir, up);
    cam->x = vnorm(cam->x);
    cam->x = vsmul(width * fov / height, cam->x);
    cam->y = vxcross(cam->x, cam->dir);
    cam->y = vnorm(cam->y);
    cam->y = vsmul(fov, cam->y);
}

/* AllocateBuffers seed fill, smallptGPU.cpp:105-110 */
void ors_seeds_init(uint32_t *seeds, size_t n, unsigned seed)
{
    srand(seed);
    for (size_t i = 0; i < n; i++) {
        seeds[i] = (uint32_t)rand();
        if (seeds[i] < 2) seeds[i] = 2;
    }
}

/* scene_build_complex.pl:5-50 (HyperSphere / PrintSphere), computed in
 * double like Perl and narrowed to float like ReadScene's %f. */
typedef struct { or_sphere *out; int cap, count; double max_depth; } hs_ctx;

static void hs_emit(hs_ctx *c, double depth, double x, double y, double z, double rad)
{
    double k = depth / c->max_depth;
    double col1 = 0.75 * k, col2 = 0.75 * (1.0 - k);
    if (c->count < c->cap) {
        or_sphere *s = &c->out[c->count];
        s->rad = (float)rad;
        s->p.x = (float)x; s->p.y = (float)y; s->p.z = (float)z;
        s->e.x = s->e.y = s->e.z = 0.f;
        s->c.x = (float)col2; s->c.y = 0.f; s->c.z = (float)col1;
        s->refl = DIFF;
    }
    c->count++;
}

static void hs_rec(hs_ctx *c, double depth, double x, double y, double z, double rad, int dir)
{
    if (!(depth <= c->max_depth)) return;
    hs_emit(c, depth, x, y, z, rad);
    double nr = rad / 2.0;
    if (dir != 0) hs_rec(c, depth + 1.0, x - rad - nr, y, z, nr, 1);
    if (dir != 1) hs_rec(c, depth + 1.0, x + rad + nr, y, z, nr, 0);
    if (dir != 2) hs_rec(c, depth + 1.0, x, y - rad - nr, z, nr, 3);
    if (dir != 3) hs_rec(c, depth + 1.0, x, y + rad + nr, z, nr, 2);
    if (dir != 4) hs_rec(c, depth + 1.0, x, y, z - rad - nr, nr, 5);
    if (dir != 5) hs_rec(c, depth + 1.0, x, y, z + rad + nr, nr, 4);
}

int ors_hypersphere(or_sphere *out, int cap, double max_depth)
{
    hs_ctx c = {out, cap, 0, max_depth};
    hs_rec(&c, 0.0, 0.0, 0.0, 0.0, 15.0, 2);                   /* :60 */
    return c.count;
}
