/*
 * oracle/whitted_oracle.c -- TEST INFRASTRUCTURE ONLY (see oracle.h).
 *
 * Plain-C restatement of the Whitted CPU path of
 * raytracer3.0.06.no_rec.samp (the bit-exact parity oracle, SURVEY.md §8(a)
 * rows W1-W8).  Every floating-point expression keeps the reference's
 * evaluation order; compile with -ffp-contract=off and without FMA ISA flags
 * (glibc sqrtf/powf/expf are the reference's libm calls: raytracer.asm:608,965).
 */
#include <math.h>
#include <string.h>
#include "oracle.h"

#define SPHERE 1
#define PLANE 2
#define HIT 1       /* scene.h:7-9 */
#define MISS 0
#define INPRIM -1
#define EPSILON 0.001f  /* common.h:24 */
#define TRACEDEPTH 4    /* common.h:25 */
#define NODECOUNT 63    /* raytracer.cpp:336 */

typedef orv3 vec3;
typedef struct { vec3 o, d; } ray_t;   /* raytracer.h:39-42 */

/* Primitive_Create, scene.cpp:55-83 */
static void prim_create(or_primitive *p, int type, float cx, float cy, float cz,
                        float radius_depth, float r, float g, float b,
                        float refl, float refr, float rindex, float diff,
                        float spec, int light)
{
    memset(p, 0, sizeof(*p));
    p->type = type;
    p->m_Light = light ? 1 : 0;
    p->m_Color.x = r; p->m_Color.y = g; p->m_Color.z = b;
    p->m_Refl = refl; p->m_Refr = refr; p->m_RIndex = rindex;
    p->m_Diff = diff; p->m_Spec = spec;
    int is_sphere = (type == SPHERE);
    p->m_Centre.x = is_sphere ? cx : 0;
    p->m_Centre.y = is_sphere ? cy : 0;
    p->m_Centre.z = is_sphere ? cz : 0;
    p->m_Radius = is_sphere ? radius_depth : 0;
    p->m_SqRadius = is_sphere ? radius_depth * radius_depth : 0;
    p->m_RRadius = is_sphere ? ((radius_depth > 0) ? 1.0f / radius_depth : 0) : 0;
    p->plane_D = is_sphere ? 0 : radius_depth;
    p->plane_N.x = is_sphere ? 0 : cx;
    p->plane_N.y = is_sphere ? 0 : cy;
    p->plane_N.z = is_sphere ? 0 : cz;
}

/* Scene_InitScene, scene.cpp:217-272 (the maxx*maxy grid loop is dead: :222) */
int orw_scene_init(or_primitive *P, int cap)
{
    if (cap < 17) return -1;
    int pc = 0;
    prim_create(&P[pc++], PLANE, 0.0f, 0.75f, 0.0f, 4.4f, 0.6f, 0.6f, 0.6f, 0.0f, 0.0f, 0.0f, 0.4f, 1.8f, 0);   /* :228 floor */
    prim_create(&P[pc++], SPHERE, 0.0f, 6.5f, 22.0f, 0.35f, 0.85f, 0.85f, 0.85f, 0.0f, 0.0f, 0.0f, 1.0f, 1.0f, 1); /* :230 light */
    prim_create(&P[pc++], SPHERE, 3.4f, -3.40f, 23.0f, 2.5f, 0.08f, 0.08f, 0.08f, 1.9f, 1.0f, 2.3f, 0.0f, 0.0f, 0); /* :232 */
    prim_create(&P[pc++], SPHERE, -0.7f, -4.90f, 27.0f, 1.0f, 0.07f, 0.17f, 0.07f, 0.1f, 1.5f, 2.3f, 0.2f, 0.8f, 0); /* :235 */
    prim_create(&P[pc++], SPHERE, -3.4f, -3.40f, 29.0f, 2.5f, 1.0f, 1.0f, 1.0f, 0.8f, 0.0f, 0.0f, 0.0f, 0.0f, 0);   /* :237 */
    prim_create(&P[pc++], SPHERE, 0.5f, -4.10f, 29.0f, 1.5f, 1.5f, 0.7f, 0.7f, 0.1f, 0.0f, 0.0f, 0.2f, 0.2f, 0);    /* :239 */
    prim_create(&P[pc++], SPHERE, -6.0f, -4.10f, 32.0f, 1.5f, 0.7f, 0.7f, 1.7f, 0.2f, 0.0f, 0.0f, 0.2f, 0.2f, 0);   /* :241 */
    prim_create(&P[pc++], SPHERE, -6.7f, -4.90f, 29.0f, 1.0f, 0.07f, 0.17f, 0.07f, 0.1f, 1.5f, 2.3f, 0.2f, 0.8f, 0); /* :243 */
    prim_create(&P[pc++], SPHERE, 6.4f, -4.90f, 18.0f, 1.0f, 0.18f, 0.18f, 0.18f, 1.7f, 1.0f, 2.6f, 1.8f, 0.0f, 0);  /* :245 */
    prim_create(&P[pc++], PLANE, 0.7f, 0.0f, 0.0f, 5.4f, 1.0f, 0.6f, 0.6f, 0.0f, 0.0f, 0.0f, 0.8f, 1.5f, 0);        /* :247 */
    prim_create(&P[pc++], PLANE, -0.7f, 0.0f, 0.0f, 5.4f, 0.7f, 0.6f, 1.0f, 0.0f, 0.0f, 0.0f, 0.8f, 0.8f, 0);       /* :249 */
    prim_create(&P[pc++], PLANE, 0.0f, -0.8f, 0.0f, 5.4f, 1.0f, 1.0f, 1.0f, 0.0f, 0.0f, 0.0f, 1.2f, 0.8f, 0);       /* :251 */
    prim_create(&P[pc++], PLANE, 0.0f, 0.0f, -0.14f, 5.4f, 2.5f, 2.5f, 2.5f, 0.0f, 0.0f, 0.0f, 1.2f, 0.8f, 0);      /* :253 */
    prim_create(&P[pc++], PLANE, 0.0f, 0.0f, 0.72f, 5.4f, 0.1f, 0.1f, 0.1f, 0.0f, 0.0f, 0.0f, 1.0f, 1.0f, 0);       /* :255 */
    prim_create(&P[pc++], SPHERE, -3.0f, 6.5f, 22.0f, 0.35f, 0.85f, 0.85f, 0.85f, 0.0f, 0.0f, 0.0f, 0.0f, 1.8f, 1);  /* :257 */
    prim_create(&P[pc++], SPHERE, 3.0f, 6.5f, 22.0f, 0.35f, 0.85f, 0.85f, 0.85f, 0.0f, 0.0f, 0.0f, 0.0f, 1.8f, 1);   /* :259 */
    prim_create(&P[pc++], SPHERE, -5.8f, -5.55f, 31.0f, 0.35f, 1.15f, 0.35f, 0.35f, 1.0f, 1.0f, 2.3f, 0.0f, 1.8f, 1); /* :261 */
    return pc;
}

/* Primitive_Intersect, scene.cpp:125-190 */
static int prim_intersect(const or_primitive *p, const ray_t *r, float *a_dist)
{
    if (p->type == SPHERE) {
        vec3 v;
        v.x = r->o.x; v.y = r->o.y; v.z = r->o.z;
        v.x -= p->m_Centre.x; v.y -= p->m_Centre.y; v.z -= p->m_Centre.z;
        float b = v.x * r->d.x + v.y * r->d.y + v.z * r->d.z;
        b = -b;
        float det = (b * b) - (v.x * v.x + v.y * v.y + v.z * v.z) + p->m_SqRadius;
        int retval = MISS;
        if (det > 0) {
            det = sqrtf(det);
            float i1 = b - det;
            float i2 = b + det;
            if (i2 > 0) {
                if (i1 < 0) {
                    if (i2 < *a_dist) { *a_dist = i2; retval = INPRIM; }
                } else {
                    if (i1 < *a_dist) { *a_dist = i1; retval = HIT; }
                }
            }
        }
        return retval;
    } else if (p->type == PLANE) {
        float d = p->plane_N.x * r->d.x + p->plane_N.y * r->d.y + p->plane_N.z * r->d.z;
        if (d != 0) {
            float dist = -((p->plane_N.x * r->o.x + p->plane_N.y * r->o.y + p->plane_N.z * r->o.z) + p->plane_D) / d;
            if (dist > 0) {
                if (dist < *a_dist) { *a_dist = dist; return HIT; }
            }
        }
        return MISS;
    }
    return MISS;
}

/* Primitive_GetNormal, scene.cpp:34-53 */
static vec3 prim_normal(const or_primitive *p, vec3 pos)
{
    vec3 n;
    if (p->type == SPHERE) {
        n.x = pos.x - p->m_Centre.x;
        n.y = pos.y - p->m_Centre.y;
        n.z = pos.z - p->m_Centre.z;
        n.x *= p->m_RRadius; n.y *= p->m_RRadius; n.z *= p->m_RRadius;
    } else if (p->type == PLANE) {
        n = p->plane_N;
    } else {
        n.x = n.y = n.z = 0;
    }
    return n;
}

int orw_primitive_intersect(const or_primitive *p, const float ray[6], float *dist)
{
    ray_t r = {{ray[0], ray[1], ray[2]}, {ray[3], ray[4], ray[5]}};
    return prim_intersect(p, &r, dist);
}

void orw_primitive_normal(const or_primitive *p, const float pos[3], float out[3])
{
    vec3 q = {pos[0], pos[1], pos[2]};
    vec3 n = prim_normal(p, q);
    out[0] = n.x; out[1] = n.y; out[2] = n.z;
}

typedef struct { uint64_t traced, shadow, tests, tir; } wcount;

/* Engine_Raytrace, raytracer.cpp:30-271 */
/* ocl != 0: the device twin in openCLcode.h:150-390, identical except that a
 * light hit adds the light's colour (openCLcode.h:176-182) instead of 1. */
static int engine_raytrace(const or_primitive *P, int n, const ray_t *a_ray, vec3 *acc,
                           int depth, float *a_rindex, float *a_dist, float *a_refl,
                           int *a_refl_index, ray_t *a_refl_ray, float *a_refr,
                           int *a_refr_index, ray_t *a_refr_ray, wcount *cnt, int ocl)
{
    if (depth > TRACEDEPTH) return -1;
    cnt->traced++;
    *a_dist = 1000000.0f;
    int prim_index = 0, result = 0, hit_once = 0;
    for (int s = 0; s < n; s++) {                                   /* :39-49 */
        int res;
        cnt->tests++;
        if ((res = prim_intersect(&P[s], a_ray, a_dist))) { hit_once = 1; prim_index = s; result = res; }
    }
    if (hit_once == 0) return -1;                                   /* :51 */
    const or_primitive *pr = &P[prim_index];
    if (pr->m_Light > 0) {                                          /* :53-57 */
        if (ocl) { acc->x += pr->m_Color.x; acc->y += pr->m_Color.y; acc->z += pr->m_Color.z; }
        else { acc->x += 1; acc->y += 1; acc->z += 1; }
        return prim_index;
    }
    vec3 pi;                                                        /* :61-65 */
    pi = a_ray->d;
    pi.x *= *a_dist; pi.y *= *a_dist; pi.z *= *a_dist;
    pi.x += a_ray->o.x; pi.y += a_ray->o.y; pi.z += a_ray->o.z;

    for (int p_index = 0; p_index < n; p_index++) {                 /* :68-176 */
        const or_primitive *light = &P[p_index];
        if (!(light->m_Light > 0)) continue;
        float shade = 1.0f;
        if (light->type == SPHERE) {                                /* :76-110 */
            vec3 L;
            L.x = light->m_Centre.x - pi.x; L.y = light->m_Centre.y - pi.y; L.z = light->m_Centre.z - pi.z;
            float tdist = sqrtf(L.x * L.x + L.y * L.y + L.z * L.z);
            L.x *= (1.0f / tdist); L.y *= (1.0f / tdist); L.z *= (1.0f / tdist);
            ray_t r;
            r.o.x = pi.x + L.x * EPSILON; r.o.y = pi.y + L.y * EPSILON; r.o.z = pi.z + L.z * EPSILON;
            r.d = L;
            cnt->shadow++;
            for (int s = 0; s < n; s++) {
                if (P[s].m_Light == 0) {
                    cnt->tests++;
                    if (prim_intersect(&P[s], &r, &tdist)) { shade = 0; break; }
                }
            }
        }
        if (shade > 0) {                                            /* :112-174 */
            vec3 L = light->m_Centre;
            L.x -= pi.x; L.y -= pi.y; L.z -= pi.z;
            float L_len = sqrtf(L.x * L.x + L.y * L.y + L.z * L.z);
            if (L_len > 0.0f) { L.x *= (1.0f / L_len); L.y *= (1.0f / L_len); L.z *= (1.0f / L_len); }
            else { L.x = L.y = L.z = 0; }
            vec3 N = prim_normal(pr, pi);
            if (pr->m_Diff > 0) {
                float dot = L.x * N.x + L.y * N.y + L.z * N.z;
                if (dot > 0) {
                    float diff = dot * pr->m_Diff * shade;
                    vec3 dv = pr->m_Color;
                    dv.x *= light->m_Color.x; dv.y *= light->m_Color.y; dv.z *= light->m_Color.z;
                    dv.x *= diff; dv.y *= diff; dv.z *= diff;
                    acc->x += dv.x; acc->y += dv.y; acc->z += dv.z;
                }
            }
            if (pr->m_Spec > 0) {
                vec3 V = a_ray->d;
                vec3 R;
                float tempDot = (L.x * N.x + L.y * N.y + L.z * N.z);
                R.x = L.x - 2.0f * tempDot * N.x;
                R.y = L.y - 2.0f * tempDot * N.y;
                R.z = L.z - 2.0f * tempDot * N.z;
                float dot = (V.x * R.x + V.y * R.y + V.z * R.z);
                if (dot > 0) {
                    float spec = powf(dot, 20) * pr->m_Spec * shade;
                    acc->x += spec * light->m_Color.x;
                    acc->y += spec * light->m_Color.y;
                    acc->z += spec * light->m_Color.z;
                }
            }
        }
    }

    *a_refr = pr->m_Refr;                                           /* :181-236 */
    if ((*a_refr > 0) && (depth < TRACEDEPTH)) {
        float rindex = pr->m_RIndex;
        float nn = *a_rindex / rindex;
        *a_rindex = rindex;
        vec3 N = prim_normal(pr, pi);
        N.x *= (float)result; N.y *= (float)result; N.z *= (float)result;
        float cosI = N.x * a_ray->d.x + N.y * a_ray->d.y + N.z * a_ray->d.z;
        cosI = -cosI;
        float cosT2 = 1.0f - nn * nn * (1.0f - cosI * cosI);
        if (cosT2 > 0.0f) {
            vec3 D = a_ray->d, T;
            T.x = (nn * D.x) + (nn * cosI - sqrtf(cosT2)) * N.x;
            T.y = (nn * D.y) + (nn * cosI - sqrtf(cosT2)) * N.y;
            T.z = (nn * D.z) + (nn * cosI - sqrtf(cosT2)) * N.z;
            a_refr_ray->o.x = pi.x + T.x * EPSILON;
            a_refr_ray->o.y = pi.y + T.y * EPSILON;
            a_refr_ray->o.z = pi.z + T.z * EPSILON;
            a_refr_ray->d = T;
            *a_refr_index = prim_index;
        } else {
            *a_refr_index = -1;   /* TIR: *a_refr stays > 0, a_refr_ray stays stale (:231-233) */
        }
    } else {
        *a_refr_index = -1;
    }

    *a_refl = pr->m_Refl;                                           /* :241-267 */
    if (*a_refl > 0.0f) {
        vec3 N = prim_normal(pr, pi);
        vec3 D = a_ray->d, R;
        float dotForR = (D.x * N.x + D.y * N.y + D.z * N.z);
        R.x = D.x - 2.0f * dotForR * N.x;
        R.y = D.y - 2.0f * dotForR * N.y;
        R.z = D.z - 2.0f * dotForR * N.z;
        a_refl_ray->o.x = pi.x + R.x * EPSILON;
        a_refl_ray->o.y = pi.y + R.y * EPSILON;
        a_refl_ray->o.z = pi.z + R.z * EPSILON;
        a_refl_ray->d = R;
        *a_refl_index = prim_index;
    } else {
        *a_refl_index = -1;
    }
    return prim_index;
}

/* One pixel of Engine_Render (raytracer.cpp:311-525): 3x3 sub-samples, the
 * 63-node breadth-first ray tree, back-accumulation and XRGB pack. */
/* ocl != 0: raytrace_kernel of openCLcode.cl:5-247 -- 2x2 sub-samples
 * (tx, ty in {-1, 0}, :66), refl child folded before refr child (:199-233),
 * x(256/4) scale (:238-240); SX/SY come from the caller. */
static uint32_t render_pixel(const or_primitive *P, int n, float SX, float SY,
                             float DX, float DY, wcount *cnt, int ocl)
{
    vec3 camera = {0.0f, 0.25f, -7.0f};                             /* :315 */
    vec3 total = {0, 0, 0};
    ray_t o_ray, refl_ray, refr_ray;
    ray_t tr_refl_ray[NODECOUNT], tr_refr_ray[NODECOUNT];
    float cx[NODECOUNT], cy[NODECOUNT], cz[NODECOUNT];
    float tr_refl[NODECOUNT], tr_refr[NODECOUNT], tr_rindex[NODECOUNT], tr_dist[NODECOUNT];
    int tr_refl_index[NODECOUNT], tr_refr_index[NODECOUNT];

    const int tend = ocl ? 1 : 2;
    for (int tx = -1; tx < tend; tx++) for (int ty = -1; ty < tend; ty++) { /* :351 */
        for (int i = 0; i < NODECOUNT; i++) {
            cx[i] = cy[i] = cz[i] = 0;
            tr_refl[i] = 0; tr_refl_index[i] = -1; tr_rindex[i] = 1.0f;
            tr_refr[i] = 0; tr_refr_index[i] = -1; tr_dist[i] = 0;
        }
        vec3 dir;                                                   /* :364-367 */
        dir.x = (SX + DX * (float)tx / 2.0f) - camera.x;
        dir.y = (SY + DY * (float)ty / 2.0f) - camera.y;
        dir.z = (0) - camera.z;
        {
            float l = 1 / sqrtf(dir.x * dir.x + dir.y * dir.y + dir.z * dir.z);
            dir.x *= l; dir.y *= l; dir.z *= l;
        }
        o_ray.d = dir; o_ray.o = camera;
        refl_ray = o_ray;
        tr_refl_ray[0] = o_ray;
        refr_ray = o_ray;

        float dist = 0, refl = 0, refr = 0, rin = 1.0f;
        int refl_index = -1, refr_index = -1;
        vec3 acc = {0, 0, 0};
        engine_raytrace(P, n, &o_ray, &acc, 1, &rin, &dist, &refl, &refl_index, &refl_ray,
                        &refr, &refr_index, &refr_ray, cnt, ocl);   /* :383 */
        cx[0] = acc.x; cy[0] = acc.y; cz[0] = acc.z;
        tr_refl_ray[0] = refl_ray; tr_refl[0] = refl; tr_refl_index[0] = refl_index;
        tr_refr_ray[0] = refr_ray; tr_rindex[0] = rin; tr_refr[0] = refr;
        tr_refr_index[0] = refr_index; tr_dist[0] = dist;
        if (refr > 0 && refr_index == -1) cnt->tir++;

        for (int i = 1; i < NODECOUNT; i += 2) {                    /* :398-472 */
            int p = (i - 1) / 2;
            for (int side = 0; side < 2; side++) {
                int c = i + side;
                float flag = side == 0 ? tr_refl[p] : tr_refr[p];
                if (flag > 0) {
                    o_ray = side == 0 ? tr_refl_ray[p] : tr_refr_ray[p];
                    acc.x = cx[c]; acc.y = cy[c]; acc.z = cz[c];
                    dist = 0; refl = 0; refr = 0; refl_index = -1; refr_index = -1;
                    rin = tr_rindex[p];
                    engine_raytrace(P, n, &o_ray, &acc, 1, &rin, &dist, &refl, &refl_index,
                                    &refl_ray, &refr, &refr_index, &refr_ray, cnt, ocl);
                    cx[c] = acc.x; cy[c] = acc.y; cz[c] = acc.z;
                    tr_refl_ray[c] = refl_ray; tr_refl[c] = refl; tr_refl_index[c] = refl_index;
                    tr_refr_ray[c] = refr_ray; tr_refr[c] = refr; tr_refr_index[c] = refr_index;
                    tr_rindex[c] = rin; tr_dist[c] = dist;
                    if (c < NODECOUNT / 2 && refr > 0 && refr_index == -1) cnt->tir++;
                } else {
                    cx[c] = cy[c] = cz[c] = 0;
                    tr_refl[c] = 0; tr_refl_index[c] = -1;
                    tr_refr[c] = 0; tr_refr_index[c] = -1;
                }
            }
        }

        for (int i = NODECOUNT - 1; i >= 2; i -= 2) {               /* :476-511 */
            int p = (i - 1) / 2;
            for (int k = 0; k < 2; k++) {
                /* CPU: refraction child (i) then reflection child (i-1);
                 * openCLcode.cl:199-233: reflection child first. */
                const int refr_side = ocl ? (k == 1) : (k == 0);
                if (refr_side) {
                    acc.x = cx[i]; acc.y = cy[i]; acc.z = cz[i];
                    if ((tr_refr_index[p] > -1) && (tr_refr[p] > 0)) {
                        const or_primitive *q = &P[tr_refr_index[p]];
                        vec3 ab;
                        ab.x = q->m_Color.x * 0.15f * -tr_dist[p];
                        ab.y = q->m_Color.y * 0.15f * -tr_dist[p];
                        ab.z = q->m_Color.z * 0.15f * -tr_dist[p];
                        acc.x = cx[i] * expf(ab.x);
                        acc.y = cy[i] * expf(ab.y);
                        acc.z = cz[i] * expf(ab.z);
                    }
                } else {
                    acc.x = cx[i - 1]; acc.y = cy[i - 1]; acc.z = cz[i - 1];
                    if ((tr_refl_index[p] > -1) && (tr_refl[p] > 0)) {
                        const or_primitive *q = &P[tr_refl_index[p]];
                        acc.x = cx[i - 1] * q->m_Color.x * tr_refl[p];
                        acc.y = cy[i - 1] * q->m_Color.y * tr_refl[p];
                        acc.z = cz[i - 1] * q->m_Color.z * tr_refl[p];
                    }
                }
                cx[p] += acc.x; cy[p] += acc.y; cz[p] += acc.z;
            }
        }
        total.x += cx[0]; total.y += cy[0]; total.z += cz[0];        /* :513-515 */
    }
    const int scale = ocl ? (256 / 4) : (256 / 9);                  /* openCLcode.cl:238-240 */
    int red = (int)(total.x * scale);                               /* :517-523 */
    int green = (int)(total.y * scale);
    int blue = (int)(total.z * scale);
    if (red > 255) red = 255;
    if (green > 255) green = 255;
    if (blue > 255) blue = 255;
    return (uint32_t)((red << 16) + (green << 8) + blue);
}

void orw_render(const or_primitive *P, int n, uint32_t *dest, int w, int h,
                int row_begin, int row_end, uint64_t *counters, int nthreads)
{
    /* Engine_InitRender, raytracer.cpp:278-294 */
    float WX1 = -3, WX2 = 3, WY1 = 2.25f, WY2 = -2.25f;
    float DX = (WX2 - WX1) / w;
    float DY = (WY2 - WY1) / h;
    float SY = WY1;
    SY += 20 * DY;
    if (row_begin < 20 || row_end > h || row_begin >= row_end) return;
    /* m_SY accumulates sequentially from row 20 (raytracer.cpp:526) and m_SX
     * from WX1 per row (:309, :524): tabulate both so rows can run in any order. */
    float SYrow[row_end > 0 ? row_end : 1];
    for (int y = 20; y < row_end; y++) { SYrow[y] = SY; SY += DY; }
    float SXcol[w > 0 ? w : 1];
    { float sx = WX1; for (int x = 0; x < w; x++) { SXcol[x] = sx; sx += DX; } }

    uint64_t t_traced = 0, t_shadow = 0, t_tests = 0, t_tir = 0;
    if (nthreads < 1) nthreads = 1;
#pragma omp parallel for schedule(dynamic, 1) num_threads(nthreads) \
    reduction(+ : t_traced, t_shadow, t_tests, t_tir) if (nthreads > 1)
    for (int y = row_begin; y < row_end; y++) {
        wcount c = {0, 0, 0, 0};
        for (int x = 0; x < w; x++)
            dest[(size_t)y * w + x] = render_pixel(P, n, SXcol[x], SYrow[y], DX, DY, &c, 0);
        t_traced += c.traced; t_shadow += c.shadow; t_tests += c.tests; t_tir += c.tir;
    }
    if (counters) {
        counters[0] = t_traced; counters[1] = t_shadow;
        counters[2] = t_tests; counters[3] = t_tir;
    }
}

/* raytrace_kernel of openCLcode.cl:5-247 on the CPU: rows [20, min(530, h))
 * (:66-67), SX = WX1 + x*DX and SY = WY1 + y*DY per pixel (:22-23), 2x2
 * sub-samples, light colour on light hits, refl-before-refr folding, x64.
 * The OpenCL built-ins (sqrt, '/', exp, pow) are taken as the correctly
 * rounded / glibc functions of the CPU path. */
void orw_render_ocl(const or_primitive *P, int n, uint32_t *dest, int w, int h,
                    uint64_t *counters, int nthreads)
{
    const float WX1 = -3.0f, WX2 = 3.0f, WY1 = 2.25f, WY2 = -2.25f;
    const float DX = (WX2 - WX1) / w;
    const float DY = (WY2 - WY1) / h;
    const int row_end = h < 530 ? h : 530;
    uint64_t t_traced = 0, t_shadow = 0, t_tests = 0, t_tir = 0;
    if (nthreads < 1) nthreads = 1;
#pragma omp parallel for schedule(dynamic, 1) num_threads(nthreads) \
    reduction(+ : t_traced, t_shadow, t_tests, t_tir) if (nthreads > 1)
    for (int y = 20; y < row_end; y++) {
        wcount c = {0, 0, 0, 0};
        const float SY = WY1 + y * DY;
        for (int x = 0; x < w; x++) {
            const float SX = WX1 + x * DX;
            dest[(size_t)y * w + x] = render_pixel(P, n, SX, SY, DX, DY, &c, 1);
        }
        t_traced += c.traced; t_shadow += c.shadow; t_tests += c.tests; t_tir += c.tir;
    }
    if (counters) {
        counters[0] = t_traced; counters[1] = t_shadow;
        counters[2] = t_tests; counters[3] = t_tir;
    }
}

uint64_t or_fnv1a64(const void *data, size_t nbytes)
{
    const unsigned char *p = (const unsigned char *)data;
    uint64_t hsh = 0xcbf29ce484222325ULL;
    for (size_t i = 0; i < nbytes; i++) { hsh ^= p[i]; hsh *= 0x100000001b3ULL; }
    return hsh;
}
