// queue.hip -- gfx950 kernels for the Raytracer3.2.03 queue tracer.
//
// Computes, bit for bit, what raytracer_non_kernel
// (Raytracer3.2.03/raytracer/OpenCL Raytracer/raytracer_non_OpenCL.c:285-449,
// the CPU twin raytracer.c:756 calls instead of its OpenCL kernel) writes:
// per pixel 3x3 primary sub-samples (:317-318), each expanded by a FIFO ray
// queue (:30-40) into a breadth-first tree of reflected and refracted rays to
// depth 5 (:370-432), every ray's colour added to the pixel's accumulator AS
// IT IS POPPED (:351-368) -- weighted by its own weight, transparency and
// (reflected rays) the colour of the primitive it left -- and the sum packed
// as uchar4 (r, g, b, 0) with the x(256/9) scale and 255 clamp (:436-447).
//
// Differences from raytracer3.0.06 (whitted.hip) that shape the kernels: no
// back-accumulation up the tree (a node's term is final when it is traced),
// no stale refraction ray (total internal reflection just queues nothing),
// and the pixel's sum is one sequential float chain over all its nodes in
// queue order: tree 0's nodes in BFS order, then tree 1's, ...  The BFS order
// of a tree is heap order (node i's children are 2i+1 reflected, 2i+2
// refracted, pushed in that order, :371-431).
//
// Mapping (MI355X-first):
//   * level-synchronous trees (rt_levelq.h queues): root_kernel traces the 9
//     primary rays of every pixel (one coherent launch, a lane = a pixel),
//     level_kernel L = 1..5 traces one level of every tree from a compacted
//     queue; each node's term (3 floats) and child slots are recorded;
//   * final_kernel folds each pixel's chain in the reference's order: the
//     leading trees without children were already summed by root_kernel, the
//     rest are walked breadth-first through their child links (a 32-slot
//     per-lane ring in LDS holds pool slots, not rays);
//   * glibc's double pow (the specular term) is replaced by x^20 in five
//     double multiplies plus a rounding certificate (spec20); a tree with a
//     term it cannot certify (~1 evaluation in 2^24), or with a node that did
//     not fit the pool, is flagged, and fix_kernel re-evaluates its pixel:
//     node by node in heap order, each node's ray re-derived from the root
//     (registers only, no per-lane ray queue), traced with rtm::pow_d;
//   * the <= 64 primitives are staged per block into LDS as per-type SoA;
//   * the reference's libm: sqrt -> correctly rounded sqrtf, exp(float) ->
//     glibc expf, pow(float, 20) -> glibc's double pow (g++'s promoting
//     std::pow), all restated bit-exactly in rt_glibc_math.h.
#include "rt_common.h"
#include "rt_glibc_math.h"
#include "rt_levelq.h"

namespace rt {
namespace queue {

constexpr int MAXP = 64;        // raytracer.c:720 allocates 50 Primitive_2
constexpr int LEVELS = 6;       // depths 0..5 (TRACEDEPTH 5, :4)
constexpr int NSUB = 9;         // 3 x 3 sub-samples (:317-318)
constexpr float EPS = 0.001f;   // :26
constexpr int PLANE = 0, SPHERE = 1;
constexpr int RING = 32;        // BFS ring per lane in final_kernel (a level-4 node
                                // leaves at most 32 level-5 slots queued)

struct Scene {
    // Dense per-type geometry for the nearest-hit loop (ties resolved to the
    // lowest primitive index, as the reference's strict '<' over ascending s).
    float4 sph[MAXP];     // centre.xyz, sq_radius
    float4 pln[MAXP];     // normal.xyz, depth
    int sph_id[MAXP], pln_id[MAXP];
    // Non-light primitives (the shadow loop's occluders, :232-240) and their
    // position in the reference's loop (for the test counter).
    float4 osph[MAXP], opln[MAXP];
    int osph_pos[MAXP], opln_pos[MAXP];
    // Per primitive, for per-lane lookups of the hit primitive.
    float4 col[MAXP];     // m_color.xyz, m_refl
    float4 mat[MAXP];     // m_refr, m_refr_index, m_diff, m_spec
    float4 geo[MAXP];     // sphere: centre.xyz, r_radius   plane: normal.xyz
    float4 cen[MAXP];     // center.xyz (the light position of :215-217)
    int type[MAXP];
    int light[MAXP];
    int lights[MAXP];     // is_light primitives, in index order
    int n, ns, np, nos, nop, nlights, nnonlight, pad_;
};

// One queued ray (Ray, :83-92): what its trace and its term need.
struct Node {
    ray3 r;
    float w;              // weight
    v3 tr;                // transparency
    int origin;           // origin_primitive (REFLECTED: its colour scales the term)
    int type;             // ORIGIN 0, REFLECTED 1, REFRACTED 2
    int rcode;            // r_index: 0 = 1.0f, k > 0 = m_refr_index of primitive k-1
};

struct Hit {
    v3 col;               // ray_col
    v3 pi;                // point_intersect
    int prim;             // -1: no hit
    int result;           // HIT 1 / INPRIM -1
    float dist;
    unsigned cnt;         // tests | shadow rays << 16 (work counters)
    bool amb;             // a specular term needs the exact pow (spec20)
};

// The specular factor (float)(pow((double)dp, 20.0) * (double)pspec) of
// :270 -- g++'s promoting std::pow, i.e. glibc's double pow -- without the
// table-driven pow.  x^20 by repeated squaring in double is within 2^-50 of
// x^20 (a float x squares exactly; four more roundings), and glibc's pow is
// within 0.52 ulp of it, so the double product glibc's value gives lies
// within 2^-49 of d = p * pspec.  If d * (1 - 2^-48) and d * (1 + 2^-48)
// round to the same float, so does that product (rounding is monotonic):
// that float is the reference's.  Otherwise (a float rounding boundary within
// 2^-48 of d, about one evaluation in 2^24) `amb` is set and the caller
// re-evaluates the node with rtm::pow_d (EXACT).  UNCERT (test hook,
// RT_QUEUE_EXACT_ALL=1): no term is certified, every one takes that path.
template <bool EXACT, bool UNCERT = false>
__device__ __forceinline__ float spec20(float dp, float pspec, bool &amb)
{
    if (EXACT) return (float)(rtm::pow_d((double)dp, 20.0) * (double)pspec);
    const double x = (double)dp, x2 = x * x, x4 = x2 * x2, x8 = x4 * x4, x16 = x8 * x8;
    const double d = (x16 * x4) * (double)pspec;
    const float lo = (float)(d * (1.0 - 0x1p-48)), hi = (float)(d * (1.0 + 0x1p-48));
    amb |= lo != hi || UNCERT;
    return lo;
}

// Sphere half of intersect (:111-148): the candidate distance (INPRIM: i2,
// HIT: i1) or +inf with res = 0.
__device__ __forceinline__ float sphere_cand(float4 g, const ray3 &r, int &res)
{
    const float vx = r.o.x - g.x, vy = r.o.y - g.y, vz = r.o.z - g.z;
    float b = vx * r.d.x + vy * r.d.y + vz * r.d.z;
    b = -b;
    const float det = (b * b) - (vx * vx + vy * vy + vz * vz) + g.w;
    res = 0;
    float cand = __builtin_inff();
    if (det > 0) {
        const float sq = sqrt_exact(det);
        const float i1 = b - sq, i2 = b + sq;
        if (i2 > 0) {
            cand = i1 < 0 ? i2 : i1;
            res = i1 < 0 ? -1 : 1;
        }
    }
    return cand;
}

// plane_intersect (:95-109) without branches: the division for every lane,
// its result kept only where the reference divides (d != 0) and t > 0.  (The
// per-lane-branch forms of this and of the sphere loops cost more exec-mask
// instructions than VALU, and an all-occluded exit per occluder sphere or
// per plane did not pay: profiles/r04.)
__device__ __forceinline__ float plane_cand_lean(float4 g, const ray3 &r)
{
    const float d = g.x * r.d.x + g.y * r.d.y + g.z * r.d.z;
    const float t = -((g.x * r.o.x + g.y * r.o.y + g.z * r.o.z) + g.w) / d;
    return (d != 0 && t > 0) ? t : __builtin_inff();
}

// get_normal, :162-177.
__device__ __forceinline__ v3 normal_at(const Scene &S, int p, v3 pt)
{
    const float4 g = S.geo[p];
    const int t = S.type[p];
    if (t == SPHERE) return mk((pt.x - g.x) * g.w, (pt.y - g.y) * g.w, (pt.z - g.z) * g.w);
    if (t == PLANE) return mk(g.x, g.y, g.z);
    return mk(0.f, 0.f, 0.f);
}

// raytrace's nearest hit (:181-193: below 1e7, lowest index on ties) for R
// rays per lane in lock-step: each sphere and plane record read once for all
// of them, their dependency chains interleaved (R = 2 in the latency-bound
// root kernel).  sphere_cand as one wave-uniform branch over a straight-line
// body (sqrt_nr for every lane, its range checked once per loop).  det <= 0
// or NaN needs no test of its own: sqrt_nr returns NaN there (v_rsq of a
// negative, 0 x inf at zero), so i2 > 0 fails.
template <int R>
__device__ __forceinline__ void nearest_n(const Scene &S, const ray3 (&ray)[R], float (&dist)[R], int (&prim)[R],
                                          int (&result)[R])
{
    bool bad[R];
#pragma unroll
    for (int q = 0; q < R; q++) {
        dist[q] = 10000000.0f;
        prim[q] = -1;
        result[q] = 1;
        bad[q] = false;
    }
    for (int k = 0; k < S.ns; k++) {
        const float4 g = S.sph[k];
        float b[R], det[R];
        bool anyp = false;
#pragma unroll
        for (int q = 0; q < R; q++) {
            const float vx = ray[q].o.x - g.x, vy = ray[q].o.y - g.y, vz = ray[q].o.z - g.z;
            b[q] = vx * ray[q].d.x + vy * ray[q].d.y + vz * ray[q].d.z;
            b[q] = -b[q];
            det[q] = (b[q] * b[q]) - (vx * vx + vy * vy + vz * vz) + g.w;
            anyp = anyp || det[q] > 0;
        }
        if (wave_any(anyp)) {
            const int id = S.sph_id[k];
#pragma unroll
            for (int q = 0; q < R; q++) {
                const float sq = sqrt_nr(det[q]);
                bad[q] = bad[q] || (det[q] > 0 && !sqrt_nr_ok(det[q]));
                const float i1 = b[q] - sq, i2 = b[q] + sq;
                const float c = i1 < 0 ? i2 : i1;
                const bool take = i2 > 0 && (c < dist[q] || (c == dist[q] && prim[q] >= 0 && id < prim[q]));
                dist[q] = take ? c : dist[q];
                prim[q] = take ? id : prim[q];
                result[q] = take ? (i1 < 0 ? -1 : 1) : result[q];
            }
        }
    }
#pragma unroll
    for (int q = 0; q < R; q++) {
        if (wave_any(bad[q])) {                             // (rare: det outside sqrt_nr's range)
            dist[q] = 10000000.0f;
            prim[q] = -1;
            result[q] = 1;
            for (int k = 0; k < S.ns; k++) {
                int res;
                const float c = sphere_cand(S.sph[k], ray[q], res);
                const int id = S.sph_id[k];
                if (res && (c < dist[q] || (c == dist[q] && prim[q] >= 0 && id < prim[q]))) {
                    dist[q] = c; prim[q] = id; result[q] = res;
                }
            }
        }
    }
#pragma unroll 4
    for (int k = 0; k < S.np; k++) {
        const float4 g = S.pln[k];
        const int id = S.pln_id[k];
#pragma unroll
        for (int q = 0; q < R; q++) {
            const float c = plane_cand_lean(g, ray[q]);
            const bool take = c < dist[q] || (c == dist[q] && prim[q] >= 0 && id < prim[q]);
            dist[q] = take ? c : dist[q];
            prim[q] = take ? id : prim[q];
            result[q] = take ? 1 : result[q];
        }
    }
}

// The rest of raytrace (:195-281) from the nearest hit.  EXACT: the specular
// factor by rtm::pow_d (else spec20's certified shortcut, h.amb when it
// cannot certify).
template <bool COUNT, bool EXACT = false, bool UNCERT = false>
__device__ Hit shade_hit(const Scene &S, const ray3 &ray, float dist, int prim, int result)
{
    Hit h;
    h.amb = false;
    h.col = mk(0.f, 0.f, 0.f);
    h.pi = mk(0.f, 0.f, 0.f);
    h.prim = prim;
    h.result = result;
    h.dist = dist;
    unsigned tests = (unsigned)S.n, shadows = 0;
    if (prim >= 0 && S.light[prim]) {                        // :197-200
        const float4 c = S.col[prim];
        h.col = mk(c.x, c.y, c.z);
    } else if (prim >= 0) {
        v3 pi;                                                // :203-205
        pi.x = ray.o.x + (ray.d.x * dist);
        pi.y = ray.o.y + (ray.d.y * dist);
        pi.z = ray.o.z + (ray.d.z * dist);
        h.pi = pi;
        const float4 hc = S.col[prim];
        const float4 hm = S.mat[prim];
        const float pdiff = hm.z, pspec = hm.w;
        const v3 N = normal_at(S, prim, pi);
        for (int li = 0; li < S.nlights; li++) {              // :207-277, lights in index order
            const int l = S.lights[li];
            const float4 lc = S.cen[l];
            const float4 lm = S.col[l];
            float shade = 1.0f;
            const v3 t = mk(lc.x - pi.x, lc.y - pi.y, lc.z - pi.z);
            const float d2 = t.x * t.x + t.y * t.y + t.z * t.z;
            float len, inv;
            if (!wave_any(!sqrt_nr_ok(d2))) {                 // :218-223 L_LEN and 1.0f / L_LEN
                len = sqrt_nr(d2);
                inv = rcp_nr(len);
            } else {
                len = sqrt_rn(d2);
                inv = 1.0f / len;
            }
            const v3 L = mk(inv * t.x, inv * t.y, inv * t.z);
            if (S.type[l] == SPHERE) {                        // :224-241
                ray3 r;
                r.o = mk(pi.x + L.x * EPS, pi.y + L.y * EPS, pi.z + L.z * EPS);
                r.d = L;
                shadows++;
                // Any non-light primitive nearer than the light centre shades
                // the point; the reference stops at the first, so only its
                // position matters (test counter).
                int first = 0x7fffffff;
                bool sbad = false;
                for (int k = 0; k < S.nos; k++) {
                    const float4 g = S.osph[k];
                    const float vx = r.o.x - g.x, vy = r.o.y - g.y, vz = r.o.z - g.z;
                    float b = vx * r.d.x + vy * r.d.y + vz * r.d.z;
                    b = -b;
                    const float det = (b * b) - (vx * vx + vy * vy + vz * vz) + g.w;
                    if (wave_any(det > 0)) {
                        const float sq = sqrt_nr(det);
                        sbad = sbad || (det > 0 && !sqrt_nr_ok(det));
                        const float i1 = b - sq, i2 = b + sq;
                        const float c = i1 < 0 ? i2 : i1;
                        const bool occ = i2 > 0 && c < len;
                        first = occ ? min(first, S.osph_pos[k]) : first;
                    }
                }
                if (wave_any(sbad)) {
                    first = 0x7fffffff;
                    for (int k = 0; k < S.nos; k++) {
                        int res;
                        const float c = sphere_cand(S.osph[k], r, res);
                        if (res && c < len) first = min(first, S.osph_pos[k]);
                        if (!COUNT && !wave_any(first == 0x7fffffff)) break;
                    }
                }
                const bool pl_any = COUNT || wave_any(first == 0x7fffffff);   // (all occluded by a sphere: no plane test)
#pragma unroll 4
                for (int k = 0; pl_any && k < S.nop; k++) {
                    const float c = plane_cand_lean(S.opln[k], r);
                    first = c < len ? min(first, S.opln_pos[k]) : first;
                }
                if (first != 0x7fffffff) shade = 0.0f;
                tests += first != 0x7fffffff ? (unsigned)first + 1u : (unsigned)S.nnonlight;
            }
            if (pdiff > 0) {                                  // :244-254
                const float dp = N.x * L.x + N.y * L.y + N.z * L.z;
                if (dp > 0) {
                    const float diff = dp * pdiff * shade;
                    h.col.x += diff * hc.x * lm.x;
                    h.col.y += diff * hc.y * lm.y;
                    h.col.z += diff * hc.z * lm.z;
                }
            }
            // :256-275.  An occluded light adds (float)(pow * m_spec * 0.0) =
            // +0 (pow of a dot <= ~1 is finite): only lit points evaluate pow.
            if (pspec > 0 && shade > 0) {
                const float td = L.x * N.x + L.y * N.y + L.z * N.z;
                const v3 R = mk(L.x - 2.0f * td * N.x, L.y - 2.0f * td * N.y, L.z - 2.0f * td * N.z);
                const float dp = ray.d.x * R.x + ray.d.y * R.y + ray.d.z * R.z;
                if (dp > 0) {
                    // shade = 1 here: the reference's * (double)shade is exact
                    const float spec = spec20<EXACT, UNCERT>(dp, pspec, h.amb);
                    h.col.x += spec * lm.x;
                    h.col.y += spec * lm.y;
                    h.col.z += spec * lm.z;
                }
            }
        }
    }
    h.cnt = COUNT ? (tests | (shadows << 16)) : 0u;
    return h;
}

// raytrace, :179-281.
template <bool COUNT, bool EXACT = false, bool UNCERT = false>
__device__ Hit trace(const Scene &S, const ray3 &ray)
{
    const ray3 rr[1] = {ray};
    float dist[1];
    int prim[1], result[1];
    nearest_n<1>(S, rr, dist, prim, result);
    return shade_hit<COUNT, EXACT, UNCERT>(S, ray, dist[0], prim[0], result[0]);
}

// The term the pixel's accumulator receives when `n` is popped (:351-368).
__device__ __forceinline__ v3 term(const Scene &S, const Node &n, const Hit &h)
{
    v3 c;
    c.x = h.col.x * n.w;
    c.y = h.col.y * n.w;
    c.z = h.col.z * n.w;
    if (n.type == 1) {
        const float4 oc = S.col[n.origin];
        c.x = c.x * oc.x * n.tr.x;
        c.y = c.y * oc.y * n.tr.y;
        c.z = c.z * oc.z * n.tr.z;
    } else if (n.type == 2) {
        c.x = c.x * n.tr.x;
        c.y = c.y * n.tr.y;
        c.z = c.z * n.tr.z;
    }
    return c;
}

// Children of `n` at depth < 5 (:370-432): bit 0 reflected child, bit 1
// refracted child (none after total internal reflection).  A ray that hit
// nothing or hit a light has undefined children in the reference
// (primitives[-1], uninitialised point_intersect): none here, flagged by
// bit 2 when the reference would have read them.  Only the flags: the
// children themselves are built by make_child once their queue slots are
// known, so neither is held across the allocation.
__device__ __forceinline__ float refr_cos_t2(const Scene &S, const Node &n, const Hit &h, float &nn, v3 &N)
{
    const int p = h.prim;
    const float rin = n.rcode ? S.mat[n.rcode - 1].y : 1.0f;
    nn = rin / S.mat[p].y;
    const v3 t = normal_at(S, p, h.pi);
    const float fr = (float)h.result;
    N = mk(t.x * fr, t.y * fr, t.z * fr);
    const float td = N.x * n.r.d.x + N.y * n.r.d.y + N.z * n.r.d.z;
    const float cosI = -td;
    return 1.0f - nn * nn * (1.0f - cosI * cosI);
}

__device__ __forceinline__ int child_flags(const Scene &S, const Node &n, const Hit &h)
{
    if (h.prim < 0) return 4;
    const int p = h.prim;
    const float refl = S.col[p].w, refr = S.mat[p].x;
    if (S.light[p]) return (refl > 0.0f || refr > 0.0f) ? 4 : 0;
    int f = refl > 0.0f ? 1 : 0;                              // :373-376
    if (refr > 0.0f) {                                        // :396-409
        float nn;
        v3 N;
        if (refr_cos_t2(S, n, h, nn, N) > 0.0f) f |= 2;
    }
    return f;
}

// The reflected (refr = false, :377-393) or refracted (:410-430) child.
__device__ __forceinline__ Node make_child(const Scene &S, const Node &n, const Hit &h, bool refr)
{
    const int p = h.prim;
    Node c;
    c.origin = p;
    if (!refr) {
        const v3 N = normal_at(S, p, h.pi);
        const float td = n.r.d.x * N.x + n.r.d.y * N.y + n.r.d.z * N.z;
        const v3 R = mk(n.r.d.x - 2.0f * td * N.x, n.r.d.y - 2.0f * td * N.y, n.r.d.z - 2.0f * td * N.z);
        c.r.o = mk(h.pi.x + R.x * EPS, h.pi.y + R.y * EPS, h.pi.z + R.z * EPS);
        c.r.d = R;
        c.w = S.col[p].w * n.w;
        c.tr = n.tr;
        c.type = 1;
        c.rcode = n.rcode;
        return c;
    }
    float nn;
    v3 N;
    const float cosT2 = refr_cos_t2(S, n, h, nn, N);
    const float cosI = -(N.x * n.r.d.x + N.y * n.r.d.y + N.z * n.r.d.z);
    const float k = nn * cosI - sqrt_exact(cosT2);
    const v3 T = mk((nn * n.r.d.x) + k * N.x, (nn * n.r.d.y) + k * N.y, (nn * n.r.d.z) + k * N.z);
    c.r.o = mk(h.pi.x + T.x * EPS, h.pi.y + T.y * EPS, h.pi.z + T.z * EPS);
    c.r.d = T;
    c.w = n.w;
    const float4 pc = S.col[p];
    const float nd = -h.dist;
    c.tr.x = n.tr.x * rtm::expf(pc.x * 0.15f * nd);
    c.tr.y = n.tr.y * rtm::expf(pc.y * 0.15f * nd);
    c.tr.z = n.tr.z * rtm::expf(pc.z * 0.15f * nd);
    c.type = 2;
    c.rcode = p + 1;
    return c;
}

__device__ __forceinline__ int expand(const Scene &S, const Node &n, const Hit &h, Node &cl, Node &cr)
{
    const int f = child_flags(S, n, h);
    if (f & 1) cl = make_child(S, n, h, false);
    if (f & 2) cr = make_child(S, n, h, true);
    return f;
}

// Primary ray of sub-sample `sub` (tx outer, ty inner, :317-339) of the pixel
// with SX = WX1 + x*DX, SY = WY1 + y*DY (:304-305).
__device__ __forceinline__ Node primary(int sub, int x, int y, float DX, float DY)
{
    const float SX = -3.0f + x * DX, SY = 2.25f + y * DY;
    const float tx = (float)(sub / 3 - 1), ty = (float)(sub % 3 - 1);
    v3 d;
    d.x = SX + DX * (tx / 2.0f) - 0.0f;
    d.y = SY + DY * (ty / 2.0f) - 0.25f;
    d.z = 0.0f - (-7.0f);
    const float l = inv_len(d.x * d.x + d.y * d.y + d.z * d.z);
    d.x *= l; d.y *= l; d.z *= l;
    Node n;
    n.r.o = mk(0.0f, 0.25f, -7.0f);
    n.r.d = d;
    n.w = 1.0f;
    n.tr = mk(1.f, 1.f, 1.f);
    n.origin = -1;
    n.type = 0;
    n.rcode = 0;
    return n;
}

// Scene image from the reference's 96-byte Primitive_2 array: one wave, a
// lane per primitive (MAXP = 64); each list position is the count of the
// earlier primitives of its kind (ballot prefix), the reference's order.
__device__ __forceinline__ void build_scene(const rtq_primitive *__restrict__ prims, int nprims, Scene &S)
{
    static_assert(MAXP <= 64, "one lane per primitive");
    const int p = __lane_id();
    const bool v = p < nprims;
    rtq_primitive q{};
    if (v) q = prims[p];
    const bool light = v && q.is_light, occluder = v && !q.is_light;
    const bool sph = v && q.type == SPHERE, pln = v && q.type == PLANE;
    const unsigned long long below = (1ull << p) - 1ull;       // lanes before this one
    const auto rank = [&](bool b) { return __popcll(__builtin_amdgcn_ballot_w64(b) & below); };
    const int il = rank(light), in = rank(occluder), is = rank(sph), ip = rank(pln);
    const int ios = rank(sph && occluder), iop = rank(pln && occluder);
    if (v) {
        S.col[p] = make_float4(q.m_color.x, q.m_color.y, q.m_color.z, q.m_refl);
        S.mat[p] = make_float4(q.m_refr, q.m_refr_index, q.m_diff, q.m_spec);
        S.geo[p] = q.type == SPHERE ? make_float4(q.center.x, q.center.y, q.center.z, q.r_radius)
                                    : make_float4(q.normal.x, q.normal.y, q.normal.z, 0.f);
        S.cen[p] = make_float4(q.center.x, q.center.y, q.center.z, 0.f);
        S.type[p] = q.type;
        S.light[p] = light ? 1 : 0;
    }
    if (light) S.lights[il] = p;
    if (sph) {
        const float4 g = make_float4(q.center.x, q.center.y, q.center.z, q.sq_radius);
        S.sph[is] = g;
        S.sph_id[is] = p;
        if (occluder) { S.osph[ios] = g; S.osph_pos[ios] = in; }
    } else if (pln) {
        const float4 g = make_float4(q.normal.x, q.normal.y, q.normal.z, q.depth);
        S.pln[ip] = g;
        S.pln_id[ip] = p;
        if (occluder) { S.opln[iop] = g; S.opln_pos[iop] = in; }
    }
    const int nl = __popcll(__builtin_amdgcn_ballot_w64(light)), nn = __popcll(__builtin_amdgcn_ballot_w64(occluder));
    const int ns = __popcll(__builtin_amdgcn_ballot_w64(sph)), np = __popcll(__builtin_amdgcn_ballot_w64(pln));
    const int nos = __popcll(__builtin_amdgcn_ballot_w64(sph && occluder));
    const int nop = __popcll(__builtin_amdgcn_ballot_w64(pln && occluder));
    if (p == 0) {
        S.n = nprims; S.nlights = nl; S.nnonlight = nn;
        S.ns = ns; S.np = np; S.nos = nos; S.nop = nop;
    }
}

// A slab's preparation in one launch: the per-slab counters and flag words
// zeroed (grid-stride, 16-B stores) and, when `prims` is given, the arena's
// scene image built by the first wave (it replaces a one-lane scene pass and
// three fills: ~23 -> ~5 us per 800x600 frame).
__global__ void __launch_bounds__(256) prep_kernel(const rtq_primitive *__restrict__ prims, int nprims,
                                                   Scene *__restrict__ scene, uint4 *__restrict__ z0, int n0,
                                                   uint4 *__restrict__ z1, int n1, uint4 *__restrict__ z2, int n2)
{
    if (prims && blockIdx.x == 0 && threadIdx.x < 64) build_scene(prims, nprims, *scene);
    const uint4 zero = make_uint4(0u, 0u, 0u, 0u);
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n0 + n1 + n2; i += gridDim.x * blockDim.x) {
        if (i < n0) z0[i] = zero;
        else if (i < n0 + n1) z1[i - n0] = zero;
        else z2[i - n0 - n1] = zero;
    }
}

__device__ __forceinline__ void load_scene(Scene &S, const Scene *__restrict__ g)
{
    static_assert(sizeof(Scene) % 16 == 0, "Scene image is copied in 16-B words");
    const uint4 *src = (const uint4 *)g;
    uint4 *dst = (uint4 *)&S;
    for (int i = threadIdx.x; i < (int)(sizeof(Scene) / 16); i += blockDim.x) dst[i] = src[i];
    __syncthreads();
}

// ---------------------------------------------------------------------------
// Level pass.  count[] layout (zeroed per slab), one counter per 128-B line.
constexpr int C_FIX = 0;                      // pixels listed for fix_kernel
constexpr int C_BASE = 1;                     // + L: pool base of level L (2..5; level 1 at 0)
constexpr int C_SEG = C_BASE + LEVELS;        // + L * NSEG + s: length of segment s of level L (1..5)
constexpr int C_TOTAL = C_SEG + LEVELS * lq::NSEG;
#define QCNT(A, i) ((A).count[(i) * lq::CSTRIDE])

// Node record info word: heap index | origin primitive << 8 | type << 16 | rcode << 20.
__device__ __forceinline__ int pack_info(int node, const Node &n)
{
    return node | ((n.origin & 0xff) << 8) | (n.type << 16) | (n.rcode << 20);
}

// Work-counter word of a node: tests | shadow rays << 16 | undefined-behaviour bit << 24.
constexpr unsigned CNT_UB = 1u << 24;

struct QArgs {
    const Scene *scene;
    float4 *rcol;         // [ntrees] root term.xyz, counter word (bits)
    int2 *rchild;         // [ntrees] pool slots of the root's children, -1 if none
    float4 *psum;         // [npix] the pixel's leading childless trees summed (xyz), first recorded sub (w, bits)
    unsigned *fixbits;    // [ntrees/32 + 1] tree whose records are incomplete or inexact
    unsigned *pixbits;    // [npix/32 + 1] pixel with such a tree: finished by fix_kernel
    int *fixlist;         // [fixcap] those pixels (fix_kernel scans pixbits when more)
    // The record pool (levels 1..5), indexed by pool slot.
    float4 *ia;           // queued ray: o.xyz, d.x
    float4 *ib;           // d.y, d.z, weight, tree (bits)
    float4 *ic;           // transparency.xyz, info (bits, pack_info)
    // A node's record takes its item's place once level_kernel has read it
    // (no other kernel reads an item after its level): ncol aliases ia, and
    // nchild[2 q] the first half of ib[q].
    float4 *ncol;         // node term.xyz, counter word (bits)
    int2 *nchild;         // pool slots of the node's children (levels 1..4), at index 2 q
    int *count;           // [C_TOTAL * CSTRIDE]
    int *ovf;             // host-mapped flag: set when this frame's pool overflowed
    int pool, fixcap, ntrees, npix, w;
    int row_begin, row_stride;   // the slab's rows: see slab_row
};

__device__ __forceinline__ int slab_row(const QArgs &A, int r)
{
    return A.row_begin + ((r >> 4) * A.row_stride << 4) + (r & 15);
}

__device__ __forceinline__ int level_base(const QArgs &A, int L)
{
    return L <= 1 ? 0 : QCNT(A, C_BASE + L);
}

// A tree whose records cannot give the reference's terms -- a node that did
// not fit the pool, or a specular term spec20 could not certify -- is
// re-evaluated with its pixel by fix_kernel.
__device__ void flag_tree(const QArgs &A, int tree)
{
    const unsigned bit = 1u << (tree & 31);
    if (atomicOr(&A.fixbits[tree >> 5], bit) & bit) return;
    const int pix = tree % A.npix;
    const unsigned pb = 1u << (pix & 31);
    if (atomicOr(&A.pixbits[pix >> 5], pb) & pb) return;
    const int k = atomicAdd(&QCNT(A, C_FIX), 1);
    if (k < A.fixcap) A.fixlist[k] = pix;
}

__device__ __forceinline__ bool tree_flagged(const QArgs &A, int tree)
{
    return (A.fixbits[tree >> 5] >> (tree & 31)) & 1u;
}

__device__ __forceinline__ bool pix_flagged(const QArgs &A, int pix)
{
    return (A.pixbits[pix >> 5] >> (pix & 31)) & 1u;
}

__device__ __forceinline__ void put_item(const QArgs &A, int slot, const Node &n, int tree, int node)
{
    A.ia[slot] = make_float4(n.r.o.x, n.r.o.y, n.r.o.z, n.r.d.x);
    A.ib[slot] = make_float4(n.r.d.y, n.r.d.z, n.w, __int_as_float(tree));
    A.ic[slot] = make_float4(n.tr.x, n.tr.y, n.tr.z, __int_as_float(pack_info(node, n)));
}

// Queues the children (flags f) of node `n` (heap index `node` of `tree`,
// hit h) into level L+1 and returns their slots (-1: none).  All lanes of the
// wave call it.
__device__ __forceinline__ int2 queue_children(const QArgs &A, const Scene &S, int L, int nbase, int wave_id,
                                               bool active, int f, const Node &n, const Hit &h, int tree,
                                               int node)
{
    const bool ql = active && (f & 1), qr = active && (f & 2);
    const int seg = wave_id & (lq::NSEG - 1);
    const int lim = lq::seg_limit(A.pool, nbase);
    int j = lq::wave_alloc(&QCNT(A, C_SEG + (L + 1) * lq::NSEG + seg), (int)ql + (int)qr);
    int2 ch = make_int2(-1, -1);
    if (ql) {
        if (j < lim) {
            ch.x = lq::seg_slot(nbase, seg, j);
            put_item(A, ch.x, make_child(S, n, h, false), tree, 2 * node + 1);
        } else {
            flag_tree(A, tree);
        }
        j++;
    }
    if (qr) {
        if (j < lim) {
            ch.y = lq::seg_slot(nbase, seg, j);
            put_item(A, ch.y, make_child(S, n, h, true), tree, 2 * node + 2);
        } else {
            flag_tree(A, tree);
        }
    }
    return ch;
}

// Occupancy of the tracing kernels (waves per SIMD): 8 measured best for
// both (6: 800x600 0.596 -> 0.549 ms, 1080p 2.07 -> 1.82 ms).
#ifndef RT_Q_ROOT_MINWAVES
#define RT_Q_ROOT_MINWAVES 8
#endif
#ifndef RT_Q_LEVEL_MINWAVES
#define RT_Q_LEVEL_MINWAVES 7     // 7: 72 VGPRs, no scratch (8: 64 VGPRs + 28 B/lane scratch since the lean loops); A/B 8/7/6
#endif

// Level 0: the nine primary rays of every pixel of the slab.
template <bool COUNT, bool UNCERT>
__global__ void __launch_bounds__(256, RT_Q_ROOT_MINWAVES)
root_kernel(QArgs A, int row_end, float DX, float DY, unsigned long long *__restrict__ counters)
{
    __shared__ Scene S;
    load_scene(S, A.scene);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int x = blockIdx.x * 16 + (wave & 1) * 8 + (lane & 7);
    const int r = blockIdx.y * 16 + (wave >> 1) * 8 + (lane >> 3);
    const int y = slab_row(A, r);
    const bool active = x < A.w && y < row_end;
    const int pix = r * A.w + x;
    const int wave_id = ((blockIdx.y * gridDim.x + blockIdx.x) << 2) + wave;
    unsigned long long cnt[4] = {0, 0, 0, 0};
    // While the pixel's trees have no children their terms are final: they
    // are summed here in the reference's order; the trees from the first one
    // with children (or with an uncertified term) on are recorded.
    // Two sub-samples' nearest hits are found together (nearest_n<2>: each
    // primitive record read once for both, two dependency chains per lane),
    // then each is shaded, summed or recorded and queued in sub-sample order
    // (1080p -2 %, 800 x 600 level; at 7 or 6 waves per SIMD instead of 8,
    // without the 12-B spill: slower; profiles/r06/queue_root_rays_ab.log).
    float ax = 0.f, ay = 0.f, az = 0.f;
    int kfirst = NSUB;
#pragma unroll 1
    for (int s0 = 0; s0 < NSUB; s0 += 2) {
        const int s1 = min(s0 + 1, NSUB - 1);
        const ray3 rr[2] = {primary(s0, x, y, DX, DY).r, primary(s1, x, y, DX, DY).r};
        float dd[2];
        int pp[2], rs[2];
        if (s0 + 1 < NSUB) {
            nearest_n<2>(S, rr, dd, pp, rs);
        } else {
            const ray3 r1[1] = {rr[0]};
            float d1[1];
            int p1[1], q1[1];
            nearest_n<1>(S, r1, d1, p1, q1);
            dd[0] = d1[0]; pp[0] = p1[0]; rs[0] = q1[0];
        }
#pragma unroll
    for (int j = 0; j < 2; j++) {
        const int sub = s0 + j;
        if (sub >= NSUB) break;
        Node n;
        Hit h;
        int f = 0;
        if (active) {
            n = primary(sub, x, y, DX, DY);
            h = shade_hit<COUNT, false, UNCERT>(S, n.r, dd[j], pp[j], rs[j]);
            f = child_flags(S, n, h);
        }
        const int tree = sub * A.npix + pix;
        const int2 ch = queue_children(A, S, 0, 0, wave_id, active, f, n, h, tree, 0);
        if (active) {
            const v3 c = term(S, n, h);     // weight 1, type ORIGIN: ray_col * 1.0f
            const unsigned cw = h.cnt | ((f & 4) ? CNT_UB : 0u);
            if (kfirst == NSUB && !(f & 3) && !h.amb) {
                ax += c.x; ay += c.y; az += c.z;
                if (COUNT) {
                    cnt[0] += 1; cnt[1] += (cw >> 16) & 0xff; cnt[2] += cw & 0xffff; cnt[3] += cw >> 24;
                }
            } else {
                if (kfirst == NSUB) kfirst = sub;
                A.rcol[tree] = make_float4(c.x, c.y, c.z, __uint_as_float(cw));
                A.rchild[tree] = ch;
                if (h.amb) flag_tree(A, tree);
            }
        }
    }
    }
    if (active) A.psum[pix] = make_float4(ax, ay, az, __int_as_float(kfirst));
    if (COUNT) flush_counters<4>(counters, cnt);
}

// Level L = 1..5: a grid of resident blocks; wave w takes 64-ray pages
// w, w + #waves, ... of the level's queue.
template <bool COUNT, bool UNCERT>
__global__ void __launch_bounds__(256, RT_Q_LEVEL_MINWAVES)
level_kernel(QArgs A, int L)
{
    __shared__ Scene S;
    load_scene(S, A.scene);
    const int base0 = level_base(A, L);
    const lq::SegView v = lq::seg_view(&QCNT(A, C_SEG + L * lq::NSEG), base0, lq::seg_limit(A.pool, base0));
    const int nbase = lq::next_base(v);             // level L+1's pool base
    if (L < LEVELS - 1 && blockIdx.x == 0 && threadIdx.x == 0) QCNT(A, C_BASE + L + 1) = nbase;
    const int lane = __lane_id();
    const int wave_id = (blockIdx.x << 2) + (threadIdx.x >> 6);
    int base, nvalid;
    for (int k = wave_id; lq::seg_chunk(v, k, base, nvalid); k += gridDim.x << 2) {
        const int q = base + lane;
        const bool active = lane < nvalid;
        Node n;
        Hit h;
        int f = 0, tree = 0, node = 0;
        if (active) {
            const float4 a = A.ia[q], b = A.ib[q], c = A.ic[q];
            const int info = __float_as_int(c.w);
            node = info & 0xff;
            n.r.o = mk(a.x, a.y, a.z);
            n.r.d = mk(a.w, b.x, b.y);
            n.w = b.z;
            tree = __float_as_int(b.w);
            n.tr = mk(c.x, c.y, c.z);
            n.origin = (info >> 8) & 0xff;
            n.type = (info >> 16) & 0xf;
            n.rcode = info >> 20;
            h = trace<COUNT, false, UNCERT>(S, n.r);
            if (L < LEVELS - 1) f = child_flags(S, n, h);
            const v3 t = term(S, n, h);
            const unsigned cw = h.cnt | ((f & 4) ? CNT_UB : 0u);
            A.ncol[q] = make_float4(t.x, t.y, t.z, __uint_as_float(cw));
            if (h.amb) flag_tree(A, tree);
        }
        if (L < LEVELS - 1) {
            const int2 ch = queue_children(A, S, L, nbase, wave_id, active, f, n, h, tree, node);
            if (active) A.nchild[2 * q] = ch;
        }
    }
}

// Adds a recorded (unflagged) tree's terms to the pixel's chain, breadth-
// first through the child links, one level at a time: ring (this lane's
// RING-entry column of pool slots) holds the current level's slots, read in
// batches of FOLD whose loads are all in flight together (consecutive nodes
// of a level do not depend on each other: the walk is latency-bound).
#ifndef RT_Q_FOLD
#define RT_Q_FOLD 8         // records per batch of the fold's breadth-first walk (A/B: 2,4,6,8,12,16 -> 8 best)
#endif
constexpr int FOLD = RT_Q_FOLD;

template <bool COUNT, int COLS>
__device__ __forceinline__ void fold_tree_from(const QArgs &A, float4 c0, int2 ch, int (*ring)[COLS], float &ax,
                                               float &ay, float &az, unsigned long long (&cnt)[4])
{
    const int t = threadIdx.x;
    ax += c0.x; ay += c0.y; az += c0.z;
    const auto count = [&](unsigned cw) {
        cnt[0] += 1; cnt[1] += (cw >> 16) & 0xff; cnt[2] += cw & 0xffff; cnt[3] += cw >> 24;
    };
    if (COUNT) count(__float_as_uint(c0.w));
    int head = 0, tail = 0;
    if (ch.x >= 0) ring[tail++ & (RING - 1)][t] = ch.x;
    if (ch.y >= 0) ring[tail++ & (RING - 1)][t] = ch.y;
    for (int lvl = 1; head != tail; lvl++) {
        const int end = tail;                       // level lvl: entries [head, end)
        const bool inner = lvl < LEVELS - 1;
        while (head != end) {
            int q[FOLD];
            float4 c[FOLD];
            int2 cc[FOLD];
#pragma unroll
            for (int i = 0; i < FOLD; i++) q[i] = head + i < end ? ring[(head + i) & (RING - 1)][t] : -1;
#pragma unroll
            for (int i = 0; i < FOLD; i++) {
                if (q[i] >= 0) {
                    c[i] = A.ncol[q[i]];
                    cc[i] = inner ? A.nchild[2 * q[i]] : make_int2(-1, -1);
                }
            }
#pragma unroll
            for (int i = 0; i < FOLD; i++) {
                if (q[i] < 0) break;
                ax += c[i].x; ay += c[i].y; az += c[i].z;
                if (COUNT) count(__float_as_uint(c[i].w));
                if (cc[i].x >= 0) ring[tail++ & (RING - 1)][t] = cc[i].x;
                if (cc[i].y >= 0) ring[tail++ & (RING - 1)][t] = cc[i].y;
                head++;
            }
        }
    }
}

// The tree's root record read here (fix_kernel); final_kernel reads several
// trees' root records together and calls fold_tree_from.
template <bool COUNT, int COLS>
__device__ __forceinline__ void fold_tree(const QArgs &A, int tree, int (*ring)[COLS], float &ax, float &ay,
                                          float &az, unsigned long long (&cnt)[4])
{
    fold_tree_from<COUNT, COLS>(A, A.rcol[tree], A.rchild[tree], ring, ax, ay, az, cnt);
}

// :436-447: (int) as x86 converts (an overflowing or NaN sum packs 0), 255
// clamp, uchar_4 (r, g, b, 0).
__device__ __forceinline__ uint32_t pack_pixel(float ax, float ay, float az)
{
    int red = cvt_i32_x86(ax * 28.0f), green = cvt_i32_x86(ay * 28.0f), blue = cvt_i32_x86(az * 28.0f);
    if (red > 255) red = 255;
    if (green > 255) green = 255;
    if (blue > 255) blue = 255;
    return (uint32_t)(red & 0xff) | ((uint32_t)(green & 0xff) << 8) | ((uint32_t)(blue & 0xff) << 16);
}

// The pixel's sum in the reference's order and the pack, for every pixel
// whose trees' records are complete and exact (the others: fix_kernel).
template <bool COUNT>
__global__ void __launch_bounds__(256)
final_kernel(QArgs A, int row_end, uint32_t *__restrict__ out, unsigned long long *__restrict__ counters)
{
    __shared__ int ring[RING][256];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int x = blockIdx.x * 16 + (wave & 1) * 8 + (lane & 7);
    const int r = blockIdx.y * 16 + (wave >> 1) * 8 + (lane >> 3);
    const int y = slab_row(A, r);
    unsigned long long cnt[4] = {0, 0, 0, 0};
    const int pix = r * A.w + x;
    if (x < A.w && y < row_end && !pix_flagged(A, pix)) {
        const float4 ps = A.psum[pix];
        float ax = ps.x, ay = ps.y, az = ps.z;
        // The remaining trees' root records loaded together (one latency
        // instead of one per tree; reading fewer at a time, 1 / 3 / 5, was
        // slower), then each tree folded in order.
        const int s0 = __float_as_int(ps.w);
        float4 c0[NSUB];
        int2 ch[NSUB];
#pragma unroll
        for (int j = 0; j < NSUB; j++) {
            const int tree = (j >= s0 ? j : NSUB - 1) * A.npix + pix;   // (s0 = NSUB: nothing left)
            c0[j] = A.rcol[tree];
            ch[j] = A.rchild[tree];
        }
#pragma unroll
        for (int j = 0; j < NSUB; j++)
            if (j >= s0) fold_tree_from<COUNT, 256>(A, c0[j], ch[j], ring, ax, ay, az, cnt);
        out[(size_t)y * A.w + x] = pack_pixel(ax, ay, az);
    }
    if (COUNT) flush_counters<4>(counters, cnt);
}

// Node `j` (heap index) of a tree re-derived from its root: the ancestors'
// rays re-traced (uncounted; their spec terms do not shape the children),
// node j traced exactly.  false if node j does not exist.
template <bool COUNT>
__device__ bool derive_node(const Scene &S, const Node &root, int j, Node &n, Hit &h, int &f, Node &cl, Node &cr)
{
    const unsigned hp = (unsigned)j + 1u;
    const int depth = 31 - __builtin_clz(hp);
    n = root;
    for (int k = depth - 1; k >= 0; k--) {
        const Hit ha = trace<false>(S, n.r);
        Node a, b;
        const int fa = expand(S, n, ha, a, b);
        const bool refr_side = (hp >> k) & 1u;
        if (!(fa & (refr_side ? 2 : 1))) return false;
        n = refr_side ? b : a;
    }
    h = trace<COUNT, true>(S, n.r);
    f = depth < LEVELS - 1 ? expand(S, n, h, cl, cr) : 0;
    return true;
}

// The pixels final_kernel skipped: the chain over all nine trees, recorded
// trees from their records, flagged trees node by node in heap order, each
// node's ray re-derived from the root and traced exactly.  Waves take listed
// pixels (or, past the list's capacity, 32-pixel words of pixbits).
template <bool COUNT>
__global__ void __launch_bounds__(64)
fix_kernel(QArgs A, float DX, float DY, uint32_t *__restrict__ out, unsigned long long *__restrict__ counters)
{
    const int nfix = QCNT(A, C_FIX);
    if (nfix == 0) return;
    if (blockIdx.x == 0) {
        // A segment counter past its limit: the pool was too small (the next
        // frame gets a larger one).
        bool over = false;
        for (int L = 1; L < LEVELS; L++) {
            const int base = level_base(A, L);
            over = over || QCNT(A, C_SEG + L * lq::NSEG + (int)threadIdx.x) > lq::seg_limit(A.pool, base);
        }
        if (__builtin_amdgcn_ballot_w64(over) != 0 && threadIdx.x == 0) *(volatile int *)A.ovf = 1;
    }
    // blocks past the work (a handful of flagged pixels) leave before staging the scene
    if ((int)blockIdx.x * 64 >= (nfix > A.fixcap ? (A.npix + 31) >> 5 : nfix)) return;
    __shared__ Scene S;
    __shared__ int ring[RING][64];
    load_scene(S, A.scene);
    const bool scan = nfix > A.fixcap;
    const int nitems = scan ? (A.npix + 31) >> 5 : nfix;
    unsigned long long cnt[4] = {0, 0, 0, 0};
    for (int it = blockIdx.x * 64 + threadIdx.x; it < nitems; it += gridDim.x * 64) {
        unsigned bits = scan ? A.pixbits[it] : 1u;
        while (bits) {
            const int bit = __builtin_ctz(bits);
            bits &= bits - 1u;
            const int pix = scan ? (it << 5) + bit : A.fixlist[it];
            const int x = pix % A.w, y = slab_row(A, pix / A.w);
            const float4 ps = A.psum[pix];
            float ax = ps.x, ay = ps.y, az = ps.z;
            for (int sub = __float_as_int(ps.w); sub < NSUB; sub++) {
                const int tree = sub * A.npix + pix;
                if (!tree_flagged(A, tree)) {
                    fold_tree<COUNT, 64>(A, tree, ring, ax, ay, az, cnt);
                    continue;
                }
                const Node root = primary(sub, x, y, DX, DY);
                unsigned long long todo = 1ull;
                while (todo) {
                    const int j = __builtin_ctzll(todo);
                    todo &= todo - 1ull;
                    Node n, cl, cr;
                    Hit h;
                    int f;
                    if (!derive_node<COUNT>(S, root, j, n, h, f, cl, cr)) continue;
                    const v3 c = term(S, n, h);
                    ax += c.x; ay += c.y; az += c.z;
                    if (COUNT) {
                        const unsigned cw = h.cnt | ((f & 4) ? CNT_UB : 0u);
                        cnt[0] += 1; cnt[1] += (cw >> 16) & 0xff; cnt[2] += cw & 0xffff; cnt[3] += cw >> 24;
                    }
                    if (f & 1) todo |= 1ull << (2 * j + 1);
                    if (f & 2) todo |= 1ull << (2 * j + 2);
                }
            }
            out[(size_t)y * A.w + x] = pack_pixel(ax, ay, az);
        }
    }
    if (COUNT) flush_counters<4>(counters, cnt);
}

}  // namespace queue

}  // namespace rt

// ------------------------------------------------------------------ host side
#include <stdlib.h>
#include <algorithm>
#include "rt_runtime.h"

namespace {

constexpr int SLOT_Q = 8;       // rtrt scratch slots of the queue tracer's arenas (two with two streams)
constexpr int SLOT_Q2 = 10;

// Trees per slab (1080p: three slabs, on two streams) and the record pool as a fraction of
// them: the reference scene needs 0.70 (3.02 M nodes below the roots for
// 4.32 M trees at 800 x 600); a tree with a node that does not fit is
// re-evaluated by final_kernel, exactly, so a denser scene is slower, never
// wrong (and the next frame's pool is 1.25x larger: rtrt::pool_fraction).
constexpr long long SLAB_TREES = 6000000;
constexpr double POOL_FRAC = 0.8;

int wait_frame(rtrt::DeviceState &st)
{
    hipError_t e = hipEventSynchronize(st.wf_done);
    if (e != hipSuccess) return rtrt::fail_hip(e, "rtq frame wait");
    st.wf_pending = false;
    return RT_OK;
}

int arena(rtrt::DeviceState &st, int slot, int w, int rows, rt::queue::QArgs *A)
{
    using namespace rt::queue;
    const size_t T = (size_t)w * rows * NSUB;
    if (T > (size_t)0x7fffffff / 2) return rtrt::fail(RT_ERR_INVALID, "rtq: frame too large");
    int *ovf = nullptr;
    double frac0 = POOL_FRAC;
    if (const char *e = getenv("RT_QUEUE_POOL_FRAC0")) frac0 = atof(e);                            // A/B
    size_t P = (size_t)(T * rtrt::pool_fraction(st, rtrt::POOL_QUEUE, (long long)T, frac0, &ovf));
    if (const char *e = getenv("RT_QUEUE_POOL_CAP")) {      // test hook: exercises the overflow path
        const long long v = atoll(e);
        if (v > 0 && (size_t)v < P) P = (size_t)v;
    }
    P = std::max<size_t>((P + rt::lq::PAGE_ROW - 1) / rt::lq::PAGE_ROW, 1) * rt::lq::PAGE_ROW;
    auto al = [](size_t b) { return (b + 255) & ~(size_t)255; };
    const size_t npix = (size_t)w * rows;
    const size_t FB = (T + 31) / 32 * 4, PB = (npix + 31) / 32 * 4;
    const size_t FC = std::max<size_t>(npix / 64, 4096);       // listed pixels (fix_kernel)
    const size_t bytes = al(sizeof(Scene)) + al(T * 16) + al(T * 8) + al(npix * 16) + al(FB) + al(PB) +
                         al(FC * 4) + al(P * 16) * 3 + al(sizeof(int) * C_TOTAL * rt::lq::CSTRIDE);
    if (st.cap[slot] < bytes && st.wf_pending) {
        int rc = wait_frame(st);
        if (rc) return rc;
    }
    void *base = nullptr;
    int rc = rtrt::scratch(st, slot, bytes, &base);
    if (rc) return rc;
    char *p = (char *)base;
    auto take = [&](size_t b) { char *q = p; p += al(b); return q; };
    A->scene = (const Scene *)take(sizeof(Scene));
    A->rcol = (float4 *)take(T * 16);
    A->rchild = (int2 *)take(T * 8);
    A->psum = (float4 *)take((size_t)w * rows * 16);
    A->fixbits = (unsigned *)take(FB);
    A->pixbits = (unsigned *)take(PB);
    A->fixlist = (int *)take(FC * 4);
    A->ia = (float4 *)take(P * 16);
    A->ib = (float4 *)take(P * 16);
    A->ic = (float4 *)take(P * 16);
    A->ncol = A->ia;
    A->nchild = (int2 *)A->ib;
    A->count = (int *)take(sizeof(int) * C_TOTAL * rt::lq::CSTRIDE);
    if ((size_t)(p - (char *)base) > bytes) return rtrt::fail(RT_ERR_INVALID, "rtq: arena layout exceeds its size");
    A->ovf = ovf;
    A->pool = (int)P;
    A->fixcap = (int)FC;
    A->w = w;
    return RT_OK;
}

template <class K>
int resident_blocks(K kernel)
{
    int dev = 0, cus = 0, per = 0;
    if (hipGetDevice(&dev) != hipSuccess) return 1024;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return 1024;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, kernel, 256, 0) != hipSuccess || per < 1) per = 1;
    return cus * per;
}

template <bool COUNT, bool UNCERT>
int launch(const rt::queue::QArgs &A, int w, int rows, int row_end, float DX, float DY, unsigned long long *cnt,
           hipStream_t s, uint32_t *d_px)
{
    using namespace rt::queue;
    static const int level_blocks = resident_blocks(level_kernel<COUNT, UNCERT>);
    const dim3 tiles((w + 15) / 16, (rows + 15) / 16), block(256);
    hipLaunchKernelGGL((root_kernel<COUNT, UNCERT>), tiles, block, 0, s, A, row_end, DX, DY, cnt);
    for (int L = 1; L < LEVELS; L++)
        hipLaunchKernelGGL((level_kernel<COUNT, UNCERT>), dim3(level_blocks), block, 0, s, A, L);
    hipLaunchKernelGGL(final_kernel<COUNT>, tiles, block, 0, s, A, row_end, d_px, cnt);
    hipLaunchKernelGGL(fix_kernel<COUNT>, dim3(256), dim3(64), 0, s, A, DX, DY, d_px, cnt);
    return rtrt::check_launch("rtq kernels");
}

}  // namespace

extern "C" int rtq_render_async(const rtq_primitive *d_prims, int nprims, uint32_t *d_pixels, int w, int h,
                                int row_begin, int row_end, uint64_t *d_counters, void *stream)
{
    if (!d_prims || !d_pixels || nprims < 1 || nprims > rt::queue::MAXP || w < 1 || h < 1)
        return rtrt::fail(RT_ERR_INVALID, "rtq_render_async: bad arguments");
    if (row_begin < 0 || row_end > h || row_begin >= row_end)
        return rtrt::fail(RT_ERR_INVALID, "rtq_render_async: rows must satisfy 0 <= row_begin < row_end <= h");
    rtrt::DeviceState *st;
    int rc = rtrt::state(&st);
    if (rc) return rc;
    std::lock_guard<std::recursive_mutex> lk(st->mu);
    hipStream_t s = (hipStream_t)stream;
    // The arena belongs to the device: order this frame after the previous
    // level-pass frame (queue tracer or Whitted), whatever stream it ran on.
    if (st->wf_pending) {
        hipError_t e = hipStreamWaitEvent(s, st->wf_done, 0);
        if (e != hipSuccess) return rtrt::fail_hip(e, "rtq_render_async wait");
    }
    const float DX = (3.0f - -3.0f) / w, DY = (-2.25f - 2.25f) / h;     // :299-300
    const int rows = row_end - row_begin;
    const int ngroups = (rows + 15) / 16;
    long long slab_trees = SLAB_TREES;
    if (const char *e = getenv("RT_QUEUE_SLAB_TREES")) slab_trees = std::max(100000LL, atoll(e));   // A/B
    long long nslab = ((long long)w * ngroups * 16 * rt::queue::NSUB + slab_trees - 1) / slab_trees;
    if (const char *e = getenv("RT_QUEUE_SLABS")) nslab = std::max(1, atoi(e));   // test hook
    nslab = std::min<long long>(std::max<long long>(nslab, 1), ngroups);
    // A frame of several slabs alternates them between the caller's stream
    // and a second one, each with its own arena: one slab's latency-bound
    // fold runs beside the other's tracing (1080p, three 6 M-tree slabs:
    // 1.80 -> 1.57 ms at the same 605 MB of arenas; one slab per stream at
    // 12 M: 1.50 ms but 1.2 GB). RT_QUEUE_STREAMS=1/2 overrides (A/B; 2
    // forces at least two slabs).
    int nstream = nslab >= 2 ? 2 : 1;
    if (const char *e = getenv("RT_QUEUE_STREAMS")) nstream = atoi(e) >= 2 ? 2 : 1;
    if (nstream == 2) {
        nslab = std::min<long long>(std::max<long long>(nslab, 2), ngroups);
        if (nslab < 2) nstream = 1;
    }
    const int slab_rows = (int)((ngroups + nslab - 1) / nslab) * 16;
    rt::queue::QArgs A[2];
    hipStream_t ss[2] = {s, s};
    if (nstream == 2) {
        if ((rc = rtrt::aux_stream(*st))) return rc;
        ss[1] = st->aux;
        hipError_t e = hipEventRecord(st->fork_ev, s);
        if (e == hipSuccess) e = hipStreamWaitEvent(st->aux, st->fork_ev, 0);
        if (e != hipSuccess) return rtrt::fail_hip(e, "rtq_render_async fork");
    }
    unsigned long long *cnt = (unsigned long long *)d_counters;
    // (after the fork, an error return still joins the second stream back)
    const auto bail = [&](int code) { return nstream == 2 ? rtrt::join_aux_on_error(*st, s, code) : code; };
    for (int i = 0; i < nstream; i++) {
        if ((rc = arena(*st, i ? SLOT_Q2 : SLOT_Q, w, slab_rows, &A[i]))) return bail(rc);
        A[i].row_stride = (int)nslab;
    }
    // RT_QUEUE_EXACT_ALL=1 (test hook): every specular term uncertified,
    // so fix_kernel's exact path renders nearly every pixel.
    const char *ex = getenv("RT_QUEUE_EXACT_ALL");
    for (int k = 0; k < (int)nslab; k++) {
        rt::queue::QArgs &a = A[k % nstream];
        hipStream_t sk = ss[k % nstream];
        const int srows = (int)((ngroups - k + nslab - 1) / nslab) * 16;
        a.row_begin = row_begin + 16 * k;
        a.npix = w * srows;
        a.ntrees = a.npix * rt::queue::NSUB;
        // counters, tree and pixel flag words zeroed; the arena's scene image
        // built by its first slab (16-B words: the arena rounds every part to 256 B)
        const auto words = [](size_t bytes) { return (int)((bytes + 15) / 16); };
        const int nz0 = words(sizeof(int) * rt::queue::C_TOTAL * rt::lq::CSTRIDE);
        const int nz1 = words(sizeof(unsigned) * (((size_t)a.ntrees + 31) / 32));
        const int nz2 = words(sizeof(unsigned) * (((size_t)a.npix + 31) / 32));
        const int pblocks = std::min(1024, std::max(1, (nz0 + nz1 + nz2 + 255) / 256));
        hipLaunchKernelGGL(rt::queue::prep_kernel, dim3(pblocks), dim3(256), 0, sk, k < nstream ? d_prims : nullptr,
                           nprims, (rt::queue::Scene *)a.scene, (uint4 *)a.count, nz0, (uint4 *)a.fixbits, nz1,
                           (uint4 *)a.pixbits, nz2);
        if (ex && *ex == '1')
            rc = cnt ? launch<true, true>(a, w, srows, row_end, DX, DY, cnt, sk, d_pixels)
                     : launch<false, true>(a, w, srows, row_end, DX, DY, cnt, sk, d_pixels);
        else
            rc = cnt ? launch<true, false>(a, w, srows, row_end, DX, DY, cnt, sk, d_pixels)
                     : launch<false, false>(a, w, srows, row_end, DX, DY, cnt, sk, d_pixels);
        if (rc) return bail(rc);
    }
    if (nstream == 2) {
        hipError_t e = hipEventRecord(st->join_ev, st->aux);
        if (e == hipSuccess) e = hipStreamWaitEvent(s, st->join_ev, 0);
        if (e != hipSuccess) return bail(rtrt::fail_hip(e, "rtq_render_async join"));
    }
    hipError_t e = hipEventRecord(st->wf_done, s);
    if (e != hipSuccess) return rtrt::fail_hip(e, "rtq_render_async record");
    st->wf_pending = true;
    return RT_OK;
}

extern "C" int rtq_render(const rtq_primitive *prims, int nprims, uint32_t *pixels, int w, int h,
                          uint64_t *counters)
{
    if (!prims || !pixels || nprims < 1 || nprims > rt::queue::MAXP || w < 1 || h < 1)
        return rtrt::fail(RT_ERR_INVALID, "rtq_render: bad arguments");
    rtrt::DeviceState *st;
    int rc = rtrt::state(&st);
    if (rc) return rc;
    std::lock_guard<std::recursive_mutex> lk(st->mu);
    // slots 0..2 may still feed a frame issued on another stream
    if (st->wf_pending && (rc = wait_frame(*st))) return rc;
    const size_t frame_bytes = sizeof(uint32_t) * (size_t)w * h;
    void *d_prims, *d_px, *d_cnt;
    if ((rc = rtrt::scratch(*st, 0, sizeof(rtq_primitive) * nprims, &d_prims))) return rc;
    if ((rc = rtrt::scratch(*st, 1, frame_bytes, &d_px))) return rc;
    if ((rc = rtrt::scratch(*st, 2, 4 * sizeof(uint64_t), &d_cnt))) return rc;
    hipStream_t s = st->stream;
    hipError_t e = hipMemcpyAsync(d_prims, prims, sizeof(rtq_primitive) * nprims, hipMemcpyHostToDevice, s);
    if (e == hipSuccess && counters) e = hipMemsetAsync(d_cnt, 0, 4 * sizeof(uint64_t), s);
    if (e != hipSuccess) return rtrt::fail_hip(e, "rtq_render H2D");
    rc = rtq_render_async((const rtq_primitive *)d_prims, nprims, (uint32_t *)d_px, w, h, 0, h,
                          counters ? (uint64_t *)d_cnt : nullptr, s);
    if (rc) return rc;
    e = hipMemcpyAsync(pixels, d_px, frame_bytes, hipMemcpyDeviceToHost, s);
    if (e == hipSuccess && counters)
        e = hipMemcpyAsync(counters, d_cnt, 4 * sizeof(uint64_t), hipMemcpyDeviceToHost, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    if (e != hipSuccess) return rtrt::fail_hip(e, "rtq_render D2H");
    return RT_OK;
}
