// spt_bvh_check.cpp -- test-only CPU checks of smallpt's hierarchy builders
// (csrc/spt_bvh.h): the 8-wide tree's structure, and a scalar restatement of
// the device walk (smallpt.hip's wide_visit / bvh_walk_wide, minus the wave
// scheduling) compared with the reference's full scan (geomfunc.h:71-110:
// every sphere, i descending, update iff d != 0 && d < t) ray by ray.
// Built with -ffp-contract=off: the sphere test is the reference's float
// formula; the box tests use fmaf as the device does (culling only).
#include <math.h>
#include <stdint.h>
#include <string.h>
#include <algorithm>
#include <vector>
#include "spt_bvh.h"

namespace {

constexpr float EPS = 0.01f;     // geom.h:29
constexpr float MISS = INFINITY;

float sphere_hit(const rt_sphere &s, const float *o, const float *d)
{
    // SphereIntersect, geomfunc.h:32-59 (a miss as +inf)
    const float opx = s.p.x - o[0], opy = s.p.y - o[1], opz = s.p.z - o[2];
    const float b = opx * d[0] + opy * d[1] + opz * d[2];
    float det = b * b - (opx * opx + opy * opy + opz * opz) + s.rad * s.rad;
    if (det < 0.f) return MISS;
    det = sqrtf(det);
    float t = b - det;
    if (t > EPS) return t;
    t = b + det;
    return t > EPS ? t : MISS;
}

struct Prepared {
    const rt_sphere *sp;
    int n;
    std::vector<int> always;
    sptbvh::BvhBuild b2;
    sptbvh::WideBuild wide;
};

int g_leaf_max = sptbvh::LEAF;

void prepare(Prepared &P, const rt_sphere *sp, int n)
{
    P.sp = sp;
    P.n = n;
    sptbvh::partition_and_build(sp, n, P.always, P.b2);
    P.wide.leaf_max = g_leaf_max;
    P.wide.build(P.b2);
}

float f32(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }

float g_K = 2.f;
int g_mode = 0;          // tools: 1 = re-test a popped child against the current t, 2 = visit order by entry distance
float g_tn[8];
int g_first = -1;

// Visit-order hit mask of wide node `nd` (bit p: the child in slot p ^ oct).
unsigned visit(const Prepared &P, int nd, const float *o, const float *inv, int oct, float alpha, float lim,
               int idmin = -1)
{
    const uint32_t *w = &P.wide.words[(size_t)nd * sptbvh::WIDE_WORDS];
    const uint32_t *hid = &P.wide.maxid[(size_t)nd * sptbvh::WIDE];   // the counted any-hit's pruning
    const float p[3] = {f32(w[0]), f32(w[1]), f32(w[2])};
    const float D0 = f32(w[4]), K = f32(w[5]);
    const float cx = p[0] - o[0], cy = p[1] - o[1], cz = p[2] - o[2];
    const float dist = sqrtf(fmaf(cx, cx, fmaf(cy, cy, cz * cz)));
    const float m = fmaf(alpha, dist + D0, K);
    const float c[3] = {cx, cy, cz};
    float a[3], bn[3], bf[3];
    for (int k = 0; k < 3; k++) {
        const float sc = f32(((w[3] >> (8 * k)) & 255u) << 23);
        a[k] = sc * inv[k];
        const float b = c[k] * inv[k], mk = m * fabsf(inv[k]);
        bn[k] = b - mk;
        bf[k] = b + mk;
    }
    unsigned hm = 0;
    for (int s = 0; s < 8; s++) {
        if (!((w[3] >> (24 + s)) & 1u)) continue;
        if (idmin >= 0 && (int)hid[s] <= idmin) continue;
        float tn = 0.f, tf = lim;
        for (int k = 0; k < 3; k++) {
            const bool neg = (oct >> k) & 1;
            const uint32_t lo = (w[16 + 6 * (s >> 2) + k] >> (8 * (s & 3))) & 255u;
            const uint32_t hi = (w[16 + 6 * (s >> 2) + 3 + k] >> (8 * (s & 3))) & 255u;
            const float qn = (float)(neg ? hi : lo), qf = (float)(neg ? lo : hi);
            tn = std::max(tn, fmaf(qn, a[k], bn[k]));
            tf = std::min(tf, fmaf(qf, a[k], bf[k]));
        }
        g_tn[s] = tn;
        if (tn <= tf) hm |= 1u << (s ^ oct);
    }
    return hm;
}

// The device walk's result for one ray: nearest (t, id) or, shadow, an
// occluder (the highest index: the counted kernel's IntersectP position).
long long g_leaves = 0, g_tests = 0;

void walk(const Prepared &P, const float *o, const float *d, bool shadow, float maxt, float &t_out, int &id_out,
          long long &visits)
{
    float t = shadow ? maxt : 1e20f;
    int id = -1;
    for (int i : P.always) {
        const float dd = sphere_hit(P.sp[i], o, d);
        if (shadow) {
            if (dd < maxt && i > id) id = i;
        } else if (dd < t || (dd == t && i > id)) {
            t = dd;
            id = i;
        }
    }
    float dv[3];
    for (int k = 0; k < 3; k++) dv[k] = fabsf(d[k]) < 1e-30f ? copysignf(1e-30f, d[k]) : d[k];
    const float inv[3] = {1.f / dv[0], 1.f / dv[1], 1.f / dv[2]};
    const float e = fabsf(d[0] * d[0] + d[1] * d[1] + d[2] * d[2] - 1.f);
    const float alpha = e < 0x1p-16f ? g_K * (1.04e-3f + sqrtf(e + 0x1p-22f)) : 1e30f;
    const int oct = (dv[0] < 0.f ? 1 : 0) | (dv[1] < 0.f ? 2 : 0) | (dv[2] < 0.f ? 4 : 0);
    if (P.wide.nnodes > 0) {
        std::vector<uint32_t> stack;
        int cur = 0;
        unsigned m = visit(P, 0, o, inv, oct, alpha, shadow ? maxt : t, shadow ? id : -1);
        visits++;
        while (true) {
            while (m == 0 && !stack.empty()) {
                cur = (int)(stack.back() >> 8);
                m = stack.back() & 255u;
                stack.pop_back();
            }
            if (m == 0) break;
            int pbit = __builtin_ctz(m);
            if ((g_mode & 4) && g_first >= 0 && ((m >> g_first) & 1u)) pbit = g_first;
            g_first = -1;
            if (g_mode & 2) {                      // nearest entry first (re-tested against the current t)
                float best = INFINITY;
                for (unsigned mm = m; mm; mm &= mm - 1) {
                    const int q = __builtin_ctz(mm);
                    visit(P, cur, o, inv, oct, alpha, shadow ? maxt : t);
                    if (g_tn[q ^ oct] < best) { best = g_tn[q ^ oct]; pbit = q; }
                }
            }
            m &= ~(1u << pbit);
            const int s = pbit ^ oct;
            if (g_mode & 1) {                      // re-test the popped child with the current t
                const unsigned hm2 = visit(P, cur, o, inv, oct, alpha, shadow ? maxt : t);
                if (!((hm2 >> pbit) & 1u)) continue;
            }
            const int32_t cw = (int32_t)P.wide.words[(size_t)cur * sptbvh::WIDE_WORDS + 8 + s];
            if (cw < 0) {
                const int f = (~cw) & 0xffffff, c = (~cw) >> 24;
                g_leaves++;
                g_tests += c;
                for (int q = 0; q < c; q++) {
                    const int i = P.b2.idx[f + q];
                    const float dd = sphere_hit(P.sp[i], o, d);
                    if (shadow) {
                        if (dd < maxt && i > id) id = i;
                    } else if (dd < t || (dd == t && i > id)) {
                        t = dd;
                        id = i;
                    }
                }
            } else {
                const unsigned hm = visit(P, cw, o, inv, oct, alpha, shadow ? maxt : t, shadow ? id : -1);
                visits++;
                if (hm) {
                    if (m) stack.push_back(((uint32_t)cur << 8) | m);
                    if (g_mode & 4) {                  // descend into the nearest hit child first
                        float best = INFINITY;
                        int bp = -1;
                        for (unsigned mm = hm; mm; mm &= mm - 1) {
                            const int q = __builtin_ctz(mm);
                            if (g_tn[q ^ oct] < best) { best = g_tn[q ^ oct]; bp = q; }
                        }
                        g_first = bp;
                    }
                    if ((int)stack.size() > P.wide.depth - 1) { t_out = NAN; id_out = -2; return; }   // stack bound violated
                    cur = cw;
                    m = hm;
                }
            }
        }
    }
    t_out = t;
    id_out = id;
}

}  // namespace

extern "C" {

void spt_bvh_set_leaf_max(int k) { g_leaf_max = k; }
void spt_bvh_set_mode(int m) { g_mode = m; }
void spt_bvh_set_k(float k) { g_K = k; }

// Per-ray statistics of the last spt_bvh_wide_check: leaves and spheres tested.
void spt_bvh_walk_stats(long long *out)
{
    out[0] = g_leaves;
    out[1] = g_tests;
    g_leaves = g_tests = 0;
}

// out: binary nodes, wide nodes, wide depth, always spheres, wide bytes
int spt_bvh_wide_stats(const rt_sphere *sp, int n, long long *out)
{
    Prepared P;
    prepare(P, sp, n);
    out[0] = (long long)P.b2.nodes.size();
    out[1] = P.wide.nnodes;
    out[2] = P.wide.depth;
    out[3] = (long long)P.always.size();
    out[4] = (long long)P.wide.words.size() * 4;
    return 0;
}

// Rays (o.xyz, d.xyz) x nrays; shadow rays use maxt[r] (NULL: nearest hit).
// Writes the walk's and the full scan's (t, id) and returns the mismatches.
long long spt_bvh_wide_check(const rt_sphere *sp, int n, const float *rays, const float *maxt, long long nrays,
                             float *t_walk, int *id_walk, float *t_scan, int *id_scan, long long *visits)
{
    Prepared P;
    prepare(P, sp, n);
    long long bad = 0, v = 0;
    for (long long r = 0; r < nrays; r++) {
        const float *o = rays + 6 * r, *d = o + 3;
        const bool shadow = maxt != nullptr;
        float tw;
        int iw;
        walk(P, o, d, shadow, shadow ? maxt[r] : 0.f, tw, iw, v);
        // the reference: Intersect (nearest, ties to the highest index) or
        // IntersectP (any d < maxt; the highest such index, as counted)
        float t = shadow ? maxt[r] : 1e20f;
        int id = -1;
        for (int i = n - 1; i >= 0; i--) {
            const float dd = sphere_hit(sp[i], o, d);
            if (shadow) {
                if (dd < maxt[r] && id < 0) id = i;
            } else if (dd < t) {
                t = dd;
                id = i;
            }
        }
        if (shadow) t = maxt[r];
        t_walk[r] = tw;
        id_walk[r] = iw;
        t_scan[r] = t;
        id_scan[r] = id;
        uint32_t a, b;
        memcpy(&a, &tw, 4);
        memcpy(&b, &t, 4);
        if (iw != id || (!shadow && a != b)) bad++;
    }
    if (visits) *visits = v;
    return bad;
}

}  // extern "C"
