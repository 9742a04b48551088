/*
 * oracle/queue_oracle.c -- TEST INFRASTRUCTURE ONLY (see oracle.h).
 *
 * C restatement of the Raytracer3.2.03 queue tracer's CPU path,
 * raytracer_non_OpenCL.c:285-449 (raytracer_non_kernel) and its helpers
 * :95-281, with the arithmetic g++ gives the reference (the project compiles
 * the .c files as C++, OpenCL Raytracer.vcxproj:85-121):
 *   sqrt(float)      -> sqrtf  (std::sqrt(float) overload)
 *   exp(float)       -> expf
 *   pow(float, 20)   -> pow((double)x, 20.0): libstdc++'s promoting template,
 *                       so `spec` is (float)(pow_d * (double)m_spec * (double)shade)
 * Pinned: equal, bit for bit, to the reference's own sources compiled in
 * place (oracle/_ref/libref_queue.so), and that build reproduces the
 * reference's committed 800x600 output test.bmp byte for byte
 * (tests/test_oracle_queue.py).
 *
 * Undefined behaviour in the reference, defined here as "no children" and
 * counted in counters[3]: a ray that hits nothing at depth < 5 reads
 * primitives[-1] (:373), and a ray that hits a light leaves point_intersect
 * uninitialised (:197-200) before its children read it.  Neither happens in
 * the reference scene (the six planes close the room; the lights have
 * refl = refr = 0).
 */
#include <math.h>
#include <string.h>
#include "oracle.h"

#define Q_TRACEDEPTH 5
#define Q_MAXRAYS 64             /* raytracer_non_OpenCL.c:18 */
#define Q_EPS 0.001f             /* :26 */

typedef struct {
    orq_f4 o, d;
    float weight, depth;
    int origin_primitive, type;  /* ORIGIN 0, REFLECTED 1, REFRACTED 2 (:56-60) */
    float r_index;
    orq_f4 transparency;
} qray;

/* dot macro (:50): A.x*B.x + A.y*B.y + A.z*B.z, left to right. */
#define QDOT(A, B) ((A).x * (B).x + (A).y * (B).y + (A).z * (B).z)

/* plane_intersect / sphere_intersect / intersect, :95-160. */
static int q_intersect(const orq_primitive *p, const qray *ray, float *cumu)
{
    if (p->type == 0) {
        const float d = QDOT(p->normal, ray->d);
        if (d != 0) {
            const float td = QDOT(p->normal, ray->o);
            const float dist = -(td + p->depth) / d;
            if (dist > 0 && dist < *cumu) { *cumu = dist; return 1; }
        }
        return 0;
    }
    if (p->type == 1) {
        orq_f4 v;
        v.x = ray->o.x - p->center.x;
        v.y = ray->o.y - p->center.y;
        v.z = ray->o.z - p->center.z;
        float b = QDOT(v, ray->d);
        b = -b;
        const float td = QDOT(v, v);
        float det = (b * b) - td + p->sq_radius;
        int ret = 0;
        if (det > 0) {
            det = sqrtf(det);
            const float i1 = b - det, i2 = b + det;
            if (i2 > 0) {
                if (i1 < 0) {
                    if (i2 < *cumu) { *cumu = i2; ret = -1; }
                } else if (i1 < *cumu) {
                    *cumu = i1; ret = 1;
                }
            }
        }
        return ret;
    }
    return 0;
}

/* get_normal, :162-177. */
static orq_f4 q_normal(const orq_primitive *p, orq_f4 pt)
{
    orq_f4 t;
    if (p->type == 0) return p->normal;
    if (p->type == 1) {
        t.x = (pt.x - p->center.x) * p->r_radius;
        t.y = (pt.y - p->center.y) * p->r_radius;
        t.z = (pt.z - p->center.z) * p->r_radius;
        t.w = 0.f;
        return t;
    }
    t.x = t.y = t.z = t.w = 0.f;
    return t;
}

/* raytrace, :179-281.  cnt: [1] shadow rays, [2] intersect calls. */
static int q_raytrace(const qray *ray, orq_f4 *acc, float *dist, orq_f4 *pi, int *result,
                      const orq_primitive *P, int n, uint64_t *cnt)
{
    *dist = 10000000.0f;
    int prim = -1;
    for (int s = 0; s < n; s++) {
        int res = q_intersect(&P[s], ray, dist);
        if (res) { prim = s; *result = res; }
    }
    cnt[2] += (uint64_t)n;
    if (prim == -1) return -1;
    const orq_primitive *hp = &P[prim];
    if (hp->is_light) {
        *acc = hp->m_color;
        return prim;
    }
    pi->x = ray->o.x + (ray->d.x * (*dist));
    pi->y = ray->o.y + (ray->d.y * (*dist));
    pi->z = ray->o.z + (ray->d.z * (*dist));
    pi->w = 0.f;
    for (int l = 0; l < n; l++) {
        if (!P[l].is_light) continue;
        float shade = 1.0f;
        orq_f4 t;
        t.x = P[l].center.x - pi->x;
        t.y = P[l].center.y - pi->y;
        t.z = P[l].center.z - pi->z;
        float llen = sqrtf(t.x * t.x + t.y * t.y + t.z * t.z);
        orq_f4 L;
        L.x = (1.0f / llen) * t.x;
        L.y = (1.0f / llen) * t.y;
        L.z = (1.0f / llen) * t.z;
        L.w = 0.f;
        if (P[l].type == 1) {
            qray r;
            r.o.x = pi->x + L.x * Q_EPS;
            r.o.y = pi->y + L.y * Q_EPS;
            r.o.z = pi->z + L.z * Q_EPS;
            r.d = L;
            cnt[1]++;
            for (int s = 0; s < n; s++) {
                if (P[s].is_light) continue;
                cnt[2]++;
                if (q_intersect(&P[s], &r, &llen)) { shade = 0; break; }
            }
        }
        const orq_f4 N = q_normal(hp, *pi);
        if (hp->m_diff > 0) {
            const float dp = QDOT(N, L);
            if (dp > 0) {
                const float diff = dp * hp->m_diff * shade;
                acc->x += diff * hp->m_color.x * P[l].m_color.x;
                acc->y += diff * hp->m_color.y * P[l].m_color.y;
                acc->z += diff * hp->m_color.z * P[l].m_color.z;
            }
        }
        if (hp->m_spec > 0) {
            const float td = QDOT(L, N);
            orq_f4 R;
            R.x = L.x - 2.0f * td * N.x;
            R.y = L.y - 2.0f * td * N.y;
            R.z = L.z - 2.0f * td * N.z;
            const float dp = QDOT(ray->d, R);
            if (dp > 0) {
                const float spec = (float)(pow((double)dp, 20.0) * (double)hp->m_spec * (double)shade);
                acc->x += spec * P[l].m_color.x;
                acc->y += spec * P[l].m_color.y;
                acc->z += spec * P[l].m_color.z;
            }
        }
    }
    return prim;
}

/* The pixel body of raytracer_non_kernel, :304-447. */
static void q_pixel(const orq_primitive *P, int n, uint8_t *px, int w, int h, int x, int y, uint64_t *cnt)
{
    const float WX1 = -3.0f, WX2 = 3.0f, WY1 = 2.25f, WY2 = -2.25f;
    const float DX = (WX2 - WX1) / w;
    const float DY = (WY2 - WY1) / h;
    const float SY = WY1 + y * DY;
    const float SX = WX1 + x * DX;
    const orq_f4 cam = {0.f, 0.25f, -7.0f, 0.f};
    qray q[Q_MAXRAYS];
    int nq = 0, front = 0, back = 0;
    orq_f4 acc = {0.f, 0.f, 0.f, 0.f};
    for (int tx = -1; tx < 2; tx++)
        for (int ty = -1; ty < 2; ty++) {
            orq_f4 dir;
            dir.x = SX + DX * (tx / 2.0f) - cam.x;
            dir.y = SY + DY * (ty / 2.0f) - cam.y;
            dir.z = 0 - cam.z;
            dir.w = 0 - cam.w;
            const float len = 1.0f / sqrtf(dir.x * dir.x + dir.y * dir.y + dir.z * dir.z);
            dir.x *= len; dir.y *= len; dir.z *= len;
            qray r;
            r.o = cam; r.d = dir;
            r.weight = 1.0f; r.depth = 0;
            r.origin_primitive = -1; r.type = 0; r.r_index = 1.0f;
            r.transparency.x = r.transparency.y = r.transparency.z = 1; r.transparency.w = 0;
            if (back >= Q_MAXRAYS) back = 0;                       /* PUSH_RAY, :30-34 */
            q[back++] = r; nq++;
            while (nq > 0) {
                if (front >= Q_MAXRAYS) front = 0;                 /* POP_RAY, :36-40 */
                const qray cur = q[front++]; nq--;
                orq_f4 rc = {0.f, 0.f, 0.f, 0.f}, pi = {0.f, 0.f, 0.f, 0.f};
                float dist;
                int result = 0;
                cnt[0]++;
                const int prim = q_raytrace(&cur, &rc, &dist, &pi, &result, P, n, cnt);
                if (cur.type == 0) {
                    acc.x += rc.x * cur.weight;
                    acc.y += rc.y * cur.weight;
                    acc.z += rc.z * cur.weight;
                } else if (cur.type == 1) {
                    const orq_f4 oc = P[cur.origin_primitive].m_color;
                    acc.x += rc.x * cur.weight * oc.x * cur.transparency.x;
                    acc.y += rc.y * cur.weight * oc.y * cur.transparency.y;
                    acc.z += rc.z * cur.weight * oc.z * cur.transparency.z;
                } else {
                    acc.x += rc.x * cur.weight * cur.transparency.x;
                    acc.y += rc.y * cur.weight * cur.transparency.y;
                    acc.z += rc.z * cur.weight * cur.transparency.z;
                }
                if (cur.depth < Q_TRACEDEPTH) {
                    if (prim < 0 || P[prim].is_light) {
                        /* undefined in the reference (see the header) */
                        if (prim < 0 || P[prim].m_refl > 0.0f || P[prim].m_refr > 0.0f) cnt[3]++;
                        continue;
                    }
                    const orq_primitive *hp = &P[prim];
                    const float refl = hp->m_refl;
                    if (refl > 0.0f) {
                        const orq_f4 N = q_normal(hp, pi);
                        const float td = QDOT(cur.d, N);
                        orq_f4 R;
                        R.x = cur.d.x - 2.0f * td * N.x;
                        R.y = cur.d.y - 2.0f * td * N.y;
                        R.z = cur.d.z - 2.0f * td * N.z;
                        R.w = 0.f;
                        qray nr;
                        nr.o.x = pi.x + R.x * Q_EPS;
                        nr.o.y = pi.y + R.y * Q_EPS;
                        nr.o.z = pi.z + R.z * Q_EPS;
                        nr.o.w = 0.f;
                        nr.d = R;
                        nr.depth = cur.depth + 1;
                        nr.weight = refl * cur.weight;
                        nr.type = 1;
                        nr.origin_primitive = prim;
                        nr.r_index = cur.r_index;
                        nr.transparency = cur.transparency;
                        if (back >= Q_MAXRAYS) back = 0;
                        q[back++] = nr; nq++;
                    }
                    const float refr = hp->m_refr;
                    if (refr > 0.0f) {
                        const float mri = hp->m_refr_index;
                        const float nn = cur.r_index / mri;
                        const orq_f4 t = q_normal(hp, pi);
                        orq_f4 N;
                        N.x = t.x * (float)result;
                        N.y = t.y * (float)result;
                        N.z = t.z * (float)result;
                        const float td = QDOT(N, cur.d);
                        const float cosI = -td;
                        const float cosT2 = 1.0f - nn * nn * (1.0f - cosI * cosI);
                        if (cosT2 > 0.0f) {
                            const float k = nn * cosI - sqrtf(cosT2);
                            orq_f4 T;
                            T.x = (nn * cur.d.x) + k * N.x;
                            T.y = (nn * cur.d.y) + k * N.y;
                            T.z = (nn * cur.d.z) + k * N.z;
                            T.w = 0.f;
                            qray nr;
                            nr.o.x = pi.x + T.x * Q_EPS;
                            nr.o.y = pi.y + T.y * Q_EPS;
                            nr.o.z = pi.z + T.z * Q_EPS;
                            nr.o.w = 0.f;
                            nr.d = T;
                            nr.depth = cur.depth + 1;
                            nr.weight = cur.weight;
                            nr.type = 2;
                            nr.origin_primitive = prim;
                            nr.r_index = mri;
                            nr.transparency.x = cur.transparency.x * expf(hp->m_color.x * 0.15f * (-dist));
                            nr.transparency.y = cur.transparency.y * expf(hp->m_color.y * 0.15f * (-dist));
                            nr.transparency.z = cur.transparency.z * expf(hp->m_color.z * 0.15f * (-dist));
                            nr.transparency.w = 0.f;
                            if (back >= Q_MAXRAYS) back = 0;
                            q[back++] = nr; nq++;
                        }
                    }
                }
            }
        }
    int red = (int)(acc.x * (256 / 9));
    int green = (int)(acc.y * (256 / 9));
    int blue = (int)(acc.z * (256 / 9));
    if (red > 255) red = 255;
    if (green > 255) green = 255;
    if (blue > 255) blue = 255;
    uint8_t *o = px + 4 * ((size_t)y * w + x);
    o[0] = (uint8_t)red; o[1] = (uint8_t)green; o[2] = (uint8_t)blue; o[3] = 0;
}

void orq_render(const orq_primitive *P, int n, uint8_t *pixels, int w, int h, int row_begin, int row_end,
                uint64_t *counters, int nthreads)
{
    uint64_t c0 = 0, c1 = 0, c2 = 0, c3 = 0;
#pragma omp parallel for schedule(dynamic, 1) num_threads(nthreads > 0 ? nthreads : 1) reduction(+ : c0, c1, c2, c3)
    for (int y = row_begin; y < row_end; y++) {
        uint64_t c[4] = {0, 0, 0, 0};
        for (int x = 0; x < w; x++) q_pixel(P, n, pixels, w, h, x, y, c);
        c0 += c[0]; c1 += c[1]; c2 += c[2]; c3 += c[3];
    }
    if (counters) {
        counters[0] = c0; counters[1] = c1; counters[2] = c2; counters[3] = c3;
    }
}

/* scene.c:53-97 (CHOOSE_SCENE 0) converted as raytracer.c:721-746 does. */
static orq_primitive q_material(float r, float g, float b, float refl, float refr, float ri, float diff,
                                float spec)
{
    orq_primitive p;
    memset(&p, 0, sizeof p);
    p.m_color.x = r; p.m_color.y = g; p.m_color.z = b;
    p.m_refl = refl; p.m_diff = diff; p.m_refr = refr; p.m_refr_index = ri; p.m_spec = spec;
    return p;
}

static orq_primitive q_plane(orq_primitive m, int light, float nx, float ny, float nz, float depth)
{
    m.type = 0; m.is_light = (uint8_t)(light != 0);
    m.normal.x = nx; m.normal.y = ny; m.normal.z = nz;
    m.depth = depth;
    return m;
}

static orq_primitive q_sphere(orq_primitive m, int light, float cx, float cy, float cz, float radius)
{
    m.type = 1; m.is_light = (uint8_t)(light != 0);
    m.center.x = cx; m.center.y = cy; m.center.z = cz;
    m.radius = radius;
    m.sq_radius = radius * radius;
    m.r_radius = 1.0f / radius;
    return m;
}

int orq_scene_init(orq_primitive *out, int cap)
{
    if (cap < 17) return -1;
    const float light = 0.85f;
    int k = 0;
    out[k++] = q_plane(q_material(0.6f, 0.6f, 0.6f, 0.0f, 0.0f, 0.0f, 0.4f, 1.8f), 0, 0.0f, 0.75f, 0.0f, 4.4f);
    out[k++] = q_sphere(q_material(0.08f, 0.08f, 0.08f, 0.2f, 1.0f, 1.4f, 0.0f, 0.0f), 0, 3.4f, -3.4f, 23.0f, 2.5f);
    out[k++] = q_sphere(q_material(0.07f, 0.17f, 0.07f, 0.1f, 1.0f, 1.2f, 0.0f, 0.0f), 0, -0.7f, -4.90f, 27.0f, 1.0f);
    out[k++] = q_sphere(q_material(1.0f, 1.0f, 1.0f, 0.8f, 0.0f, 0.0f, 0.0f, 0.0f), 0, -3.4f, -3.4f, 29.0f, 2.5f);
    out[k++] = q_sphere(q_material(1.5f, 0.7f, 0.7f, 0.1f, 0.0f, 0.0f, 0.2f, 0.2f), 0, 0.5f, -4.1f, 29.0f, 1.5f);
    out[k++] = q_sphere(q_material(0.7f, 0.7f, 1.7f, 0.2f, 0.0f, 0.0f, 0.2f, 0.2f), 0, -6.0f, -4.1f, 32.0f, 1.5f);
    out[k++] = q_sphere(q_material(0.07f, 0.17f, 0.07f, 0.3f, 1.0f, 1.2f, 0.2f, 0.8f), 0, -6.7f, -4.90f, 29.0f, 1.0f);
    out[k++] = q_sphere(q_material(0.08f, 0.08f, 0.08f, 0.7f, 1.0f, 1.3f, 0.8f, 0.0f), 0, 6.4f, -4.9f, 18.0f, 1.0f);
    out[k++] = q_plane(q_material(1.0f, 0.6f, 0.6f, 0.0f, 0.0f, 0.0f, 0.8f, 1.5f), 0, 0.7f, 0.0f, 0.0f, 5.4f);
    out[k++] = q_plane(q_material(0.7f, 0.6f, 1.0f, 0.0f, 0.0f, 0.0f, 0.8f, 0.8f), 0, -0.7f, 0.0f, 0.0f, 5.4f);
    out[k++] = q_plane(q_material(1.0f, 1.0f, 1.0f, 0.0f, 0.0f, 0.0f, 1.2f, 0.8f), 0, 0.0f, -0.8f, 0.0f, 5.4f);
    out[k++] = q_plane(q_material(1.5f, 1.5f, 1.5f, 0.0f, 0.0f, 0.0f, 1.2f, 0.8f), 0, 0.0f, 0.0f, -0.14f, 5.4f);
    out[k++] = q_plane(q_material(0.1f, 0.1f, 0.1f, 0.0f, 0.0f, 0.0f, 1.0f, 1.0f), 0, 0.0f, 0.0f, 0.72f, 5.4f);
    out[k++] = q_sphere(q_material(light, light, light, 0.0f, 0.0f, 0.0f, 0.0f, 1.8f), 1, 0.0f, 6.5f, 22.0f, 0.35f);
    out[k++] = q_sphere(q_material(light, light, light, 0.0f, 0.0f, 0.0f, 0.0f, 1.8f), 1, -3.0f, 6.5f, 22.0f, 0.35f);
    out[k++] = q_sphere(q_material(light, light, light, 0.0f, 0.0f, 0.0f, 0.0f, 1.8f), 1, 3.0f, 6.5f, 22.0f, 0.35f);
    /* n_primitives = 17 (:55) with 16 created: the last is memset's zero
     * primitive -- a PLANE of normal 0 that nothing ever hits, tested by every
     * shadow ray. */
    memset(&out[k++], 0, sizeof out[0]);
    return k;
}
