// whitted.hip -- gfx950 kernel for the Whitted hot path of raytracer3.0.06.no_rec.samp.
//
// Computes, bit for bit, what the CPU path Engine_Render (raytracer.cpp:301-530)
// writes into the Surface framebuffer: per pixel 3x3 primary sub-samples, each
// expanded into the reference's 63-node breadth-first ray tree
// (raytracer.cpp:398-472), back-accumulated (:476-511), summed (:513-515) and
// packed to 0x00RRGGBB with the x28 scale and 255 clamp (:517-523).
//
// Mapping (MI355X-first, not a port of openCLcode.cl):
//   * the ray trees of all (pixel, sub-sample) pairs are evaluated level by
//     level (see "Level-synchronous" below): one coherent launch for the 9 x
//     W x rows root rays, then one launch per tree level over a compacted
//     queue of child rays, back-accumulation level by level, and a final
//     per-pixel sum.  Every lane traces one ray per step (no lane idles while
//     a neighbour walks a deep glass tree), and the node records live in a
//     device arena written once and read once (no per-lane scratch arrays);
//   * the <= 64 primitives are staged once per block from the reference's
//     96-byte AoS into LDS as SoA (geometry float4, materials, light list);
//     the nearest-hit and occluder loops read them with wave-uniform indices
//     (LDS broadcast, no bank conflicts);
//   * trees the level pass cannot evaluate exactly -- total internal
//     reflection, whose refraction child reuses the previous node's
//     refraction ray (raytracer.cpp:231-233), or a full queue -- are
//     re-evaluated by a sequential per-lane BFS (fixup_kernel);
//   * m_SX / m_SY are sequential float sums in the reference (:309,:524,:526):
//     the host tabulates them once per frame size (exact same float adds);
//   * glibc powf/expf are reproduced by rt_glibc_math.h (double-precision,
//     op-for-op restatement of glibc 2.35's FMA build).
#include "rt_common.h"
#include "rt_glibc_math.h"
#include "rt_levelq.h"

namespace rt {
namespace whitted {

constexpr int MAXP = 64;        // reference allocates 50 (scene.cpp:225)
constexpr int NODES = 63;       // raytracer.cpp:336
constexpr float EPS = 0.001f;   // common.h:24
constexpr int SPHERE = 1, PLANE = 2;

struct Scene {
    // Geometry in dense per-type arrays (no index indirection in the hot
    // loops): the nearest-hit and occlusion results are independent of the
    // visiting order once distance ties go to the lowest primitive index
    // (the reference's strict '<' over ascending s, raytracer.cpp:39-49).
    float4 sph[MAXP];   // sphere centre.xyz, SqRadius
    float4 pln[MAXP];   // plane N.xyz, D
    int sph_id[MAXP], pln_id[MAXP];        // original primitive index
    float4 osph[MAXP];  // non-light spheres (occluders, raytracer.cpp:100)
    float4 opln[MAXP];  // non-light planes
    int osph_pos[MAXP], opln_pos[MAXP];    // position in the non-light order (test counts)
    int ns, np, nos, nop;
    // Per-primitive records for per-lane lookups of the hit primitive.
    float4 geo[MAXP];   // sphere: centre.xyz, SqRadius   plane: N.xyz, D
    float4 mat0[MAXP];  // colour.xyz, refl
    float4 mat1[MAXP];  // refr, diff, spec, rindex
    float4 cen[MAXP];   // m_Centre (light position, raytracer.cpp:80,115)
    float rrad[MAXP];   // RRadius (sphere normal scale)
    int type[MAXP];
    int light[MAXP];
    int lights[MAXP];   // indices of m_Light > 0 primitives, in index order
    int n, nnonlight, nlights;
    int pad_;                                     // sizeof(Scene) % 16 == 0
};

// Sphere half of Primitive_Intersect (scene.cpp:130-169): the candidate
// distance (INPRIM: i2, HIT: i1) or +inf with res = 0.
__device__ __forceinline__ float sphere_cand(float4 g, const ray3 &r, int &res)
{
    const float vx = r.o.x - g.x, vy = r.o.y - g.y, vz = r.o.z - g.z;
    float b = vx * r.d.x + vy * r.d.y + vz * r.d.z;
    b = -b;
    float det = (b * b) - (vx * vx + vy * vy + vz * vz) + g.w;
    res = 0;
    float cand = __builtin_inff();
    if (det > 0) {
        det = sqrt_exact(det);
        const float i1 = b - det, i2 = b + det;
        if (i2 > 0) {
            cand = i1 < 0 ? i2 : i1;
            res = i1 < 0 ? -1 : 1;
        }
    }
    return cand;
}

// Plane half of Primitive_Intersect (scene.cpp:171-185), without branches:
// the division for every lane, its result kept only where the reference
// divides (d != 0) and t > 0.
__device__ __forceinline__ float plane_cand_lean(float4 g, const ray3 &r)
{
    const float d = g.x * r.d.x + g.y * r.d.y + g.z * r.d.z;
    const float t = -((g.x * r.o.x + g.y * r.o.y + g.z * r.o.z) + g.w) / d;
    return (d != 0 && t > 0) ? t : __builtin_inff();
}

// Primitive_GetNormal, scene.cpp:34-53.
__device__ __forceinline__ v3 normal_at(const Scene &S, int p, v3 pos)
{
    int t = S.type[p];
    float4 g = S.geo[p];
    if (t == SPHERE) {
        float rr = S.rrad[p];
        v3 n = mk(pos.x - g.x, pos.y - g.y, pos.z - g.z);
        n.x *= rr; n.y *= rr; n.z *= rr;
        return n;
    }
    if (t == PLANE) return mk(g.x, g.y, g.z);
    return mk(0.f, 0.f, 0.f);
}

struct Hit {
    v3 acc;           // node colour (starts at 0, raytracer.cpp:403-405)
    int prim;         // nearest primitive, -1 on miss
    float dist;       // *a_Dist
    float refl, refr; // *a_refl / *a_refr as the caller sees them
    bool refr_ray_ok; // refraction ray written (false on TIR)
    float rindex_out; // *a_RIndex after the call
    ray3 refl_ray, refr_ray;
};

struct Counts { unsigned long long traced, shadow, tests, tir; };

// Engine_Raytrace's nearest hit (raytracer.cpp:39-49: min distance below 1e6,
// lowest index on ties) for R rays per lane in lock-step: each sphere and
// plane record is read once for all of them and their dependency chains
// interleave (R = 2 in the latency-bound root kernel).  Branch-lean: a
// sphere is one wave-uniform branch (skipped when no lane's det is
// positive) around a straight-line body -- sqrt_nr for every lane, its range
// checked once per loop, a lane outside it redoing its ray with the exact
// per-sphere test -- and a plane test is straight-line (the division for
// every lane, kept where the reference divides).  det <= 0 or NaN needs no
// test of its own: sqrt_nr returns NaN there, so i2 > 0 fails.  (The
// per-lane-branch forms cost more exec-mask instructions than VALU:
// profiles/r04/whitted_lean_loops_ab.log.)  prim = 0x7fffffff: no hit.
template <int R>
__device__ __forceinline__ void nearest_n(const Scene &S, const ray3 (&ray)[R], float (&dist)[R], int (&prim)[R],
                                          int (&result)[R])
{
    bool bad[R];
#pragma unroll
    for (int r = 0; r < R; r++) {
        dist[r] = 1000000.0f;
        prim[r] = 0x7fffffff;
        result[r] = 0;
        bad[r] = false;
    }
    for (int k = 0; k < S.ns; k++) {
        const float4 g = S.sph[k];
        float b[R], det[R];
        bool anyp = false;
#pragma unroll
        for (int r = 0; r < R; r++) {
            const float vx = ray[r].o.x - g.x, vy = ray[r].o.y - g.y, vz = ray[r].o.z - g.z;
            b[r] = vx * ray[r].d.x + vy * ray[r].d.y + vz * ray[r].d.z;
            b[r] = -b[r];
            det[r] = (b[r] * b[r]) - (vx * vx + vy * vy + vz * vz) + g.w;
            anyp = anyp || det[r] > 0;
        }
        if (wave_any(anyp)) {
            const int id = S.sph_id[k];
#pragma unroll
            for (int r = 0; r < R; r++) {
                const float sd = sqrt_nr(det[r]);
                bad[r] = bad[r] || (det[r] > 0 && !sqrt_nr_ok(det[r]));
                const float i1 = b[r] - sd, i2 = b[r] + sd;
                const float c = i1 < 0 ? i2 : i1;
                const bool take = i2 > 0 && (c < dist[r] || (c == dist[r] && id < prim[r]));
                dist[r] = take ? c : dist[r];
                prim[r] = take ? id : prim[r];
                result[r] = take ? (i1 < 0 ? -1 : 1) : result[r];
            }
        }
    }
#pragma unroll
    for (int r = 0; r < R; r++) {
        if (wave_any(bad[r])) {                         // (rare: det outside sqrt_nr's range)
            dist[r] = 1000000.0f;
            prim[r] = 0x7fffffff;
            result[r] = 0;
            for (int k = 0; k < S.ns; k++) {
                int res;
                const float c = sphere_cand(S.sph[k], ray[r], res);
                const int id = S.sph_id[k];
                if (res && (c < dist[r] || (c == dist[r] && id < prim[r]))) { dist[r] = c; prim[r] = id; result[r] = res; }
            }
        }
    }
#pragma unroll 4
    for (int k = 0; k < S.np; k++) {
        const float4 g = S.pln[k];
        const int id = S.pln_id[k];
#pragma unroll
        for (int r = 0; r < R; r++) {
            const float c = plane_cand_lean(g, ray[r]);
            const bool take = c < dist[r] || (c == dist[r] && id < prim[r]);
            dist[r] = take ? c : dist[r];
            prim[r] = take ? id : prim[r];
            result[r] = take ? 1 : result[r];
        }
    }
}

// The rest of Engine_Raytrace (raytracer.cpp:51-271) from its nearest hit
// (a_Depth is always 1 at every call site, so the TRACEDEPTH guards are
// constant-true).  ocl: the device twin of openCLcode.h:150-390 -- a light
// hit adds the light's colour (openCLcode.h:176-182) instead of (1,1,1);
// all else equal.  COUNT = false: the work counters are dead, so a shadow
// test stops as soon as every lane of the wave has found an occluder (the
// reference's own early exit, at wave granularity); only "occluded or not"
// is used then.
template <bool COUNT>
__device__ Hit shade_hit(const Scene &S, const ray3 &ray, float rindex_in, float dist, int prim, int result,
                         Counts &cnt, bool ocl)
{
    Hit h;
    h.acc = mk(0.f, 0.f, 0.f);
    h.prim = -1;
    h.refl = 0.f; h.refr = 0.f;
    h.refr_ray_ok = false;
    h.rindex_out = rindex_in;
    cnt.traced++;
    const int hit_once = prim != 0x7fffffff;
    if (!hit_once) prim = 0;
    cnt.tests += (unsigned long long)S.n;
    h.dist = dist;
    if (!hit_once) return h;                            // :51
    h.prim = prim;
    if (S.light[prim] > 0) {                            // :53-57
        if (ocl) {
            const float4 lc = S.mat0[prim];
            h.acc = mk(lc.x, lc.y, lc.z);
        } else {
            h.acc = mk(1.f, 1.f, 1.f);
        }
        return h;
    }
    v3 pi;                                              // :61-65
    pi.x = ray.d.x * dist; pi.y = ray.d.y * dist; pi.z = ray.d.z * dist;
    pi.x += ray.o.x; pi.y += ray.o.y; pi.z += ray.o.z;

    const float4 m0 = S.mat0[prim];
    const float4 m1 = S.mat1[prim];
    const float pdiff = m1.y, pspec = m1.z;
    const v3 N = normal_at(S, prim, pi);

    for (int li = 0; li < S.nlights; li++) {            // :68-176 lights in index order
        const int l = S.lights[li];
        const float4 lg = S.cen[l];
        const float4 lm = S.mat0[l];
        float shade = 1.0f;
        // pi -> light centre, its length and reciprocal: the same float ops
        // in the shadow test (:76-82) and the shading (:115-125), done once.
        v3 L = mk(lg.x - pi.x, lg.y - pi.y, lg.z - pi.z);
        float len, inv;
        {
            const float d2 = L.x * L.x + L.y * L.y + L.z * L.z;
            if (!wave_any(!sqrt_nr_ok(d2))) {
                len = sqrt_nr(d2);
                inv = rcp_nr(len);
            } else {
                len = sqrt_rn(d2);
                inv = 1.0f / len;
            }
        }
        L.x *= inv; L.y *= inv; L.z *= inv;
        if (S.type[l] == SPHERE) {                      // :76-110
            const float tdist = len;
            ray3 r;
            r.o = mk(pi.x + L.x * EPS, pi.y + L.y * EPS, pi.z + L.z * EPS);
            r.d = L;
            cnt.shadow++;
            // Any non-light primitive nearer than the light centre shades the
            // point (the reference breaks at the first one; which one does not
            // matter, only the count of tests, recovered from its position).
            // The loops are nearest_n's lean forms.  (An all-occluded exit
            // after each sphere measured slower; the planes take one
            // all-occluded check before their loop.)
            int first = 0x7fffffff;
            bool sbad = false;
            for (int k = 0; k < S.nos; k++) {
                const float4 g = S.osph[k];
                const float vx = r.o.x - g.x, vy = r.o.y - g.y, vz = r.o.z - g.z;
                float b = vx * r.d.x + vy * r.d.y + vz * r.d.z;
                b = -b;
                const float det = (b * b) - (vx * vx + vy * vy + vz * vz) + g.w;
                if (wave_any(det > 0)) {
                    const float sd = sqrt_nr(det);
                    sbad = sbad || (det > 0 && !sqrt_nr_ok(det));
                    const float i1 = b - sd, i2 = b + sd;
                    const float c = i1 < 0 ? i2 : i1;
                    const bool occ = i2 > 0 && c < tdist;
                    first = occ ? min(first, S.osph_pos[k]) : first;
                }
            }
            if (wave_any(sbad)) {
                first = 0x7fffffff;
                for (int k = 0; k < S.nos; k++) {
                    int res;
                    const float c = sphere_cand(S.osph[k], r, res);
                    if (res && c < tdist) first = min(first, S.osph_pos[k]);
                    if (!COUNT && !wave_any(first == 0x7fffffff)) break;
                }
            }
            const bool pl_any = COUNT || wave_any(first == 0x7fffffff);   // (all occluded by a sphere: no plane test)
#pragma unroll 4
            for (int k = 0; pl_any && k < S.nop; k++) {
                const float c = plane_cand_lean(S.opln[k], r);
                first = c < tdist ? min(first, S.opln_pos[k]) : first;
            }
            if (first != 0x7fffffff) shade = 0;
            cnt.tests += (unsigned long long)(first != 0x7fffffff ? first + 1 : S.nnonlight);
        }
        if (shade > 0) {                                // :112-174
            if (!(len > 0.0f)) L = mk(0.f, 0.f, 0.f);
            if (pdiff > 0) {
                float dot = L.x * N.x + L.y * N.y + L.z * N.z;
                if (dot > 0) {
                    float diff = dot * pdiff * shade;
                    v3 dv = mk(m0.x, m0.y, m0.z);
                    dv.x *= lm.x; dv.y *= lm.y; dv.z *= lm.z;
                    dv.x *= diff; dv.y *= diff; dv.z *= diff;
                    h.acc.x += dv.x; h.acc.y += dv.y; h.acc.z += dv.z;
                }
            }
            if (pspec > 0) {
                float td = (L.x * N.x + L.y * N.y + L.z * N.z);
                v3 R = mk(L.x - 2.0f * td * N.x, L.y - 2.0f * td * N.y, L.z - 2.0f * td * N.z);
                float dot = (ray.d.x * R.x + ray.d.y * R.y + ray.d.z * R.z);
                if (dot > 0) {
                    float spec = rtm::powf(dot, 20.0f) * pspec * shade;
                    h.acc.x += spec * lm.x; h.acc.y += spec * lm.y; h.acc.z += spec * lm.z;
                }
            }
        }
    }

    h.refr = m1.x;                                      // :181-236
    if (h.refr > 0) {
        const float rindex = m1.w;
        const float nr = rindex_in / rindex;
        h.rindex_out = rindex;
        const float fres = (float)result;
        v3 Nr = mk(N.x * fres, N.y * fres, N.z * fres);
        float cosI = Nr.x * ray.d.x + Nr.y * ray.d.y + Nr.z * ray.d.z;
        cosI = -cosI;
        float cosT2 = 1.0f - nr * nr * (1.0f - cosI * cosI);
        if (cosT2 > 0.0f) {
            float k = nr * cosI - sqrt_exact(cosT2);
            v3 T = mk((nr * ray.d.x) + k * Nr.x, (nr * ray.d.y) + k * Nr.y, (nr * ray.d.z) + k * Nr.z);
            h.refr_ray.o = mk(pi.x + T.x * EPS, pi.y + T.y * EPS, pi.z + T.z * EPS);
            h.refr_ray.d = T;
            h.refr_ray_ok = true;
        }
    }

    h.refl = m0.w;                                      // :241-267
    if (h.refl > 0.0f) {
        float dR = (ray.d.x * N.x + ray.d.y * N.y + ray.d.z * N.z);
        v3 R = mk(ray.d.x - 2.0f * dR * N.x, ray.d.y - 2.0f * dR * N.y, ray.d.z - 2.0f * dR * N.z);
        h.refl_ray.o = mk(pi.x + R.x * EPS, pi.y + R.y * EPS, pi.z + R.z * EPS);
        h.refl_ray.d = R;
    }
    return h;
}

// Engine_Raytrace, raytracer.cpp:30-271.
template <bool COUNT>
__device__ Hit trace(const Scene &S, const ray3 &ray, float rindex_in, Counts &cnt, bool ocl)
{
    const ray3 rr[1] = {ray};
    float dist[1];
    int prim[1], result[1];
    nearest_n<1>(S, rr, dist, prim, result);
    return shade_hit<COUNT>(S, ray, rindex_in, dist[0], prim[0], result[0], cnt, ocl);
}

// Primary ray of sub-sample `sub` (tx outer, ty inner: raytracer.cpp:351,364-367).
// side = 3 (CPU path, tx/ty in -1..1) or 2 (openCLcode.cl:66, tx/ty in -1..0).
__device__ __forceinline__ ray3 primary(int sub, float SX, float SY, float DX, float DY, int side)
{
    const float tx = (float)(sub / side - 1), ty = (float)(sub % side - 1);
    v3 d;
    d.x = (SX + DX * tx / 2.0f) - 0.0f;
    d.y = (SY + DY * ty / 2.0f) - 0.25f;
    d.z = 0.0f - (-7.0f);
    float l = inv_len(d.x * d.x + d.y * d.y + d.z * d.z);
    d.x *= l; d.y *= l; d.z *= l;
    ray3 r;
    r.o = mk(0.0f, 0.25f, -7.0f);
    r.d = d;
    return r;
}

// Builds the SoA scene image from the reference's 96-byte AoS primitives:
// one wave, a lane per primitive (MAXP = 64); each list position is the
// count of the earlier primitives of its kind (ballot prefix), so the lists
// keep the reference's order.
__device__ void build_scene(Scene &S, const rt_primitive *__restrict__ prims, int nprims)
{
    static_assert(MAXP <= 64, "one lane per primitive");
    const int p = __lane_id();
    const bool v = p < nprims;
    rt_primitive q{};
    if (v) q = prims[p];
    const bool light = v && q.m_Light > 0, occluder = v && q.m_Light == 0;
    const bool sph = v && q.type == SPHERE, pln = v && q.type == PLANE;
    const unsigned long long below = (1ull << p) - 1ull;       // lanes before this one
    const auto rank = [&](bool b) { return __popcll(__builtin_amdgcn_ballot_w64(b) & below); };
    const auto total = [](bool b) { return __popcll(__builtin_amdgcn_ballot_w64(b)); };
    const int il = rank(light), in = rank(occluder), is = rank(sph), ip = rank(pln);
    const int ios = rank(sph && occluder), iop = rank(pln && occluder);
    if (v) {
        S.geo[p] = q.type == SPHERE ? make_float4(q.m_Centre.x, q.m_Centre.y, q.m_Centre.z, q.m_SqRadius)
                                    : make_float4(q.plane_N.x, q.plane_N.y, q.plane_N.z, q.plane_D);
        S.mat0[p] = make_float4(q.m_Color.x, q.m_Color.y, q.m_Color.z, q.m_Refl);
        S.mat1[p] = make_float4(q.m_Refr, q.m_Diff, q.m_Spec, q.m_RIndex);
        S.cen[p] = make_float4(q.m_Centre.x, q.m_Centre.y, q.m_Centre.z, 0.f);
        S.rrad[p] = q.m_RRadius;
        S.type[p] = q.type;
        S.light[p] = q.m_Light;
    }
    if (light) S.lights[il] = p;
    if (sph) {
        const float4 g = make_float4(q.m_Centre.x, q.m_Centre.y, q.m_Centre.z, q.m_SqRadius);
        S.sph[is] = g;
        S.sph_id[is] = p;
        if (occluder) { S.osph[ios] = g; S.osph_pos[ios] = in; }
    } else if (pln) {
        const float4 g = make_float4(q.plane_N.x, q.plane_N.y, q.plane_N.z, q.plane_D);
        S.pln[ip] = g;
        S.pln_id[ip] = p;
        if (occluder) { S.opln[iop] = g; S.opln_pos[iop] = in; }
    }
    const int nl = total(light), nn = total(occluder), ns = total(sph), np = total(pln);
    const int nos = total(sph && occluder), nop = total(pln && occluder);
    if (p == 0) {
        S.n = nprims; S.nlights = nl; S.nnonlight = nn;
        S.ns = ns; S.np = np; S.nos = nos; S.nop = nop;
    }
}

// A slab's preparation in one launch: its counters and tree flag words
// zeroed (grid-stride, 16-B stores) and, when `prims` is given, the arena's
// scene image built by the first wave (replaces a one-lane scene pass and
// two fills).
__global__ void __launch_bounds__(256) prep_kernel(const rt_primitive *__restrict__ prims, int nprims,
                                                   Scene *__restrict__ scene, uint4 *__restrict__ z0, int n0,
                                                   uint4 *__restrict__ z1, int n1)
{
    if (prims && blockIdx.x == 0 && threadIdx.x < 64) build_scene(*scene, prims, nprims);
    const uint4 zero = make_uint4(0u, 0u, 0u, 0u);
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n0 + n1; i += gridDim.x * blockDim.x) {
        if (i < n0) z0[i] = zero;
        else z1[i - n0] = zero;
    }
}

// Block-cooperative copy of the scene image into LDS (coalesced 16-B loads).
__device__ __forceinline__ void load_scene(Scene &S, const Scene *__restrict__ g)
{
    static_assert(sizeof(Scene) % 16 == 0, "Scene image is copied in 16-B words");
    const uint4 *src = (const uint4 *)g;
    uint4 *dst = (uint4 *)&S;
    for (int i = threadIdx.x; i < (int)(sizeof(Scene) / 16); i += blockDim.x) dst[i] = src[i];
    __syncthreads();
}

// ---------------------------------------------------------------------------
// Level-synchronous ("wavefront") evaluation of the ray trees.
//
// A tree = one (pixel, sub-sample) of Engine_Render; node i of the reference's
// 63-slot BFS array sits on level floor(log2(i+1)).  The reference traces a
// child of node p iff p < 31 and refl/refr(p) > 0 (:398-472), with p's own
// reflection ray and -- unless p had total internal reflection -- p's own
// refraction ray; the trace of a node depends on nothing else.  So all trees
// advance together one level per launch:
//   root_kernel    level 0 of every tree (coherent: one launch, lanes = pixels);
//   level_kernel   level L = 1..5 from a compacted queue of child rays that
//                  level L-1 appended (wave-aggregated atomics);
//   tir_kernel     after level L: the refraction children of its TIR nodes
//                  (see below), appended to level L+1;
//   backacc_kernel node colour += refraction child (Beer factor) then +=
//                  reflection child (:476-511), children final first: levels
//                  3 and 1, each folding the two levels below it in registers;
//   final_kernel   level 0 of the nine trees of a pixel + the sum / x28 pack.
// Records hold what back-accumulation needs (colour, distance, primitive, TIR)
// and the queue slots of the node's two children.
//
// Queue memory.  Levels 1..5 share ONE pool of records.  Each level's queue
// is split into NSEG segments with their own counters (a producing wave
// appends to segment wave_id mod NSEG, so thousands of waves finishing a step
// together do not queue on one atomic address); a segment's items are laid
// out in 64-slot pages, page c of segment s at level base + (c*NSEG + s)*64.
// Level L+1 starts right after level L's last page (base_{L+1} = base_L +
// NSEG*64*max_s pages_s, computed by level_kernel(L) once level L is final),
// so the pool holds the levels' actual node counts (14.2 M at 1080p for 17.1 M
// trees), not a per-level worst case.
//
// Exceptions go to fixup_kernel, which re-evaluates the whole tree in the
// reference's sequential BFS order (per-lane records): a tree with a node
// that does not fit in the pool, or a TIR whose stale ray (below) is not in
// the pool.  The fixup counts only the nodes the wavefront did not trace, so
// counters stay exactly the reference's.
constexpr int LEVELS = 6;
constexpr int INFO_TIR = 0x100;       // refr > 0 but no refraction ray (TIR)
constexpr int INFO_REFR_OK = 0x200;   // the node wrote a refraction ray
constexpr int TREE_BITS = 25;         // queued item: tree | node << TREE_BITS (node 0..62; < 2^25 trees a slab)
constexpr int TREE_MASK = (1 << TREE_BITS) - 1;
using lq::NSEG;
using lq::PAGE;
using lq::PAGE_ROW;
using lq::CSTRIDE;
using lq::SegView;
using lq::seg_slot;
using lq::wave_alloc;
using lq::next_base;
using lq::seg_chunk;
// count[] layout (zeroed per slab), one counter per 128-B line (lq::CSTRIDE).
constexpr int C_FIX = 0;                      // trees flagged for fixup
constexpr int C_TIR = 1;                      // + L: TIR list length of level L (0..4)
constexpr int C_BASE = C_TIR + LEVELS;        // + L: pool base of level L (2..5; level 1 at 0)
constexpr int C_SEG = C_BASE + LEVELS;        // + L * NSEG + s: length of segment s of level L (1..5)
constexpr int C_TOTAL = C_SEG + LEVELS * NSEG;
#define CNT(A, i) ((A).count[(i) * CSTRIDE])

struct WfArgs {
    const Scene *scene;       // scene image (prep_kernel, the arena's first slab)
    float4 *rcol;             // [ntrees] root colour.xyz, dist
    int *rinfo;               // [ntrees] hit primitive | INFO_*
    float4 *psum;             // [npix] sum (xyz) of the colours of the pixel's leading childless trees,
                              //   in sub-sample order, and (w, int bits) the first sub-sample not in it
    int2 *rchild;             // [ntrees] pool slots (level 1) of refl / refr child, -1 if none
    unsigned *fixbits;        // [ntrees/32 + 1] tree flagged for fixup
    int *fixlist;             // [fixcap] flagged trees (fixup scans fixbits when more)
    // The record pool (levels 1..5), indexed by pool slot.
    float4 *ia;               // queued ray: o.xyz, d.x
    float4 *ib;               // d.y, d.z, rindex, tree | node << TREE_BITS (int bits)
    float4 *lcol;             // node colour.xyz, dist
    int *linfo;               // traced node: hit primitive | INFO_*
    int2 *lchild;             // pool slots of the node's children
    int4 *tir[LEVELS];        // [tcap] TIR nodes of level L (0..4): slot, tree, node, rindex (bits)
    int *count;               // [C_TOTAL * CSTRIDE]
    int *ovf;                 // host-mapped flag: set when this frame's pool or a TIR list overflowed
    int pool, fixcap, tcap, ntrees, npix, w;
    int row_begin, row_stride;   // the slab's rows: see slab_row
    int row_count;               //   (row_count 16-row groups per row_stride)
    int side, nsub;           // sub-sample grid: 3 x 3 (CPU path) or 2 x 2 (openCLcode.cl)
    bool ocl;                 // openCLcode.cl semantics (light colour, refl-first folding, x64)
};

// Row y of the slab's local row r: slabs interleave in groups of 16 rows (a
// root block's height).  Local group g of the slab is frame group
// (g / row_count) * row_stride + g % row_count, counted from row_begin =
// the first row + 16 x the slab's offset in the period: row_count = 1 for
// slabs of one group per period (slab k of n: offset k, period n), more for
// the unequal pair of a two-stream frame (render_async).
__device__ __forceinline__ int slab_row(const WfArgs &A, int r)
{
    const int g = r >> 4;
    const int pg = A.row_count == 1 ? g * A.row_stride : (g / A.row_count) * A.row_stride + g % A.row_count;
    return A.row_begin + (pg << 4) + (r & 15);
}

// Per-segment item limit of a level based at `base` (the pages left in the pool).
__device__ __forceinline__ int seg_limit(const WfArgs &A, int base)
{
    return lq::seg_limit(A.pool, base);
}
__device__ __forceinline__ int level_base(const WfArgs &A, int L)
{
    return L <= 1 ? 0 : CNT(A, C_BASE + L);
}

__device__ void flag_tree(const WfArgs &A, int tree)
{
    const unsigned bit = 1u << (tree & 31);
    if (!(atomicOr(&A.fixbits[tree >> 5], bit) & bit)) {
        const int s = atomicAdd(&CNT(A, C_FIX), 1);
        if (s < A.fixcap) A.fixlist[s] = tree;
    }
}

__device__ __forceinline__ bool flagged(const WfArgs &A, int tree)
{
    return (A.fixbits[tree >> 5] >> (tree & 31)) & 1u;
}

__device__ __forceinline__ void put_item(const WfArgs &A, int L, int slot, const ray3 &r, float rin, int tree,
                                         int node)
{
    A.ia[slot] = make_float4(r.o.x, r.o.y, r.o.z, r.d.x);
    // The node index rides in the item's tree word (no separate 4-B write here
    // and read at trace time: 8 B per queued node).
    (void)L;
    A.ib[slot] = make_float4(r.d.y, r.d.z, rin, __int_as_float(tree | (node << TREE_BITS)));
}

// Queues the children of node `node` (level L < 5, record `slot_self`) into
// level L+1 (pool base `nbase`) and returns their slots (-1: not queued).  A
// TIR node's refraction child is queued later by tir_kernel, once every node
// before it in BFS order has been traced.  All lanes of the wave call it.
__device__ __forceinline__ int2 queue_children(const WfArgs &A, int L, int nbase, int wave_id, bool active,
                                               int slot_self, int tree, int node, const Hit &hh, bool tir)
{
    const bool cl = active && hh.refl > 0, cr = active && hh.refr > 0;
    const bool qr = cr && !tir;
    const int seg = wave_id & (NSEG - 1);
    const int lim = seg_limit(A, nbase);
    int j = wave_alloc(&CNT(A, C_SEG + (L + 1) * NSEG + seg), (int)cl + (int)qr);
    int2 ch = make_int2(-1, -1);
    if (cl) {
        if (j < lim) {
            ch.x = seg_slot(nbase, seg, j);
            put_item(A, L + 1, ch.x, hh.refl_ray, hh.rindex_out, tree, 2 * node + 1);
        } else {
            flag_tree(A, tree);
        }
        j++;
    }
    if (qr) {
        if (j < lim) {
            ch.y = seg_slot(nbase, seg, j);
            put_item(A, L + 1, ch.y, hh.refr_ray, hh.rindex_out, tree, 2 * node + 2);
        } else {
            flag_tree(A, tree);
        }
    }
    if (cr && tir) {
        const int t = atomicAdd(&CNT(A, C_TIR + L), 1);
        if (t < A.tcap) A.tir[L][t] = make_int4(slot_self, tree, node, __float_as_int(hh.rindex_out));
        else flag_tree(A, tree);
    }
    return ch;
}

__device__ __forceinline__ int node_info(const Hit &hh, bool tir)
{
    return (hh.prim & 0xff) | (tir ? INFO_TIR : 0) | (hh.refr_ray_ok ? INFO_REFR_OK : 0);
}

// Consumer view of level L's segmented queue (rt_levelq.h).
__device__ __forceinline__ SegView seg_view(const WfArgs &A, int L)
{
    const int base = level_base(A, L);
    return lq::seg_view(&CNT(A, C_SEG + L * NSEG), base, seg_limit(A, base));
}

#ifndef RT_WH_MINWAVES
#define RT_WH_MINWAVES 6    // root/level kernels: occupancy 5 -> 6 (86 -> 79 VGPRs, no spills): -2 %
#endif
#ifndef RT_WH_ROOT_RAYS
#define RT_WH_ROOT_RAYS 2   // root kernel: sub-sample rays per lane whose nearest hits are found together
#endif
#ifndef RT_WH_ROOT_MINWAVES
#define RT_WH_ROOT_MINWAVES 6 // (R = 2: 80 VGPRs + 20 B scratch; 5 waves / 3 rays: level, profiles/r06/whitted_root_rays_ab.log)
#endif

template <bool COUNT>
__global__ void __launch_bounds__(256, RT_WH_ROOT_MINWAVES)
root_kernel(WfArgs A, int row_end, const float *__restrict__ sx_tab, const float *__restrict__ sy_tab,
            float DX, float DY, unsigned long long *__restrict__ counters)
{
    __shared__ Scene S;
    load_scene(S, A.scene);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int x = blockIdx.x * 16 + (wave & 1) * 8 + (lane & 7);
    const int r = blockIdx.y * 16 + (wave >> 1) * 8 + (lane >> 3);   // the slab's row r
    const int y = slab_row(A, r);
    const bool active = x < A.w && y < row_end;
    const int pix = r * A.w + x;
    const float SX = active ? sx_tab[x] : 0.f, SY = active ? sy_tab[y] : 0.f;
    Counts cnt = {0, 0, 0, 0};
    // A tree without children (a plane, a light, a miss) is final at its
    // root: while the pixel's trees are childless their colours are summed
    // here, in sub-sample order with the same float adds as final_kernel
    // (:513-515), and only the trees from the first one with children on
    // are recorded for the later passes.
    float tr = 0.f, tg = 0.f, tb = 0.f;
    int kfirst = A.nsub;
    const int wave_id = ((blockIdx.y * gridDim.x + blockIdx.x) << 2) + wave;
    // The nearest hits of RT_WH_ROOT_RAYS sub-samples at a time (nearest_n:
    // their chains interleave -- this pass is latency-bound), then each
    // sub-sample shaded, recorded and queued in sub-sample order.
    for (int sub0 = 0; sub0 < A.nsub; sub0 += RT_WH_ROOT_RAYS) {
        ray3 rp[RT_WH_ROOT_RAYS];
        float nd[RT_WH_ROOT_RAYS];
        int np_[RT_WH_ROOT_RAYS], nr[RT_WH_ROOT_RAYS];
#pragma unroll
        for (int j = 0; j < RT_WH_ROOT_RAYS; j++) rp[j] = primary(min(sub0 + j, A.nsub - 1), SX, SY, DX, DY, A.side);
        nearest_n<RT_WH_ROOT_RAYS>(S, rp, nd, np_, nr);
#pragma unroll
        for (int j = 0; j < RT_WH_ROOT_RAYS; j++) {
            const int sub = sub0 + j;
            if (sub >= A.nsub) break;                   // (uniform)
            Hit hh;
            bool tir = false;
            if (active) {
                hh = shade_hit<COUNT>(S, rp[j], 1.0f, nd[j], np_[j], nr[j], cnt, A.ocl);
                tir = hh.refr > 0 && !hh.refr_ray_ok;
                if (tir) cnt.tir++;
            }
            const int tree = sub * A.npix + pix;
            const int2 ch = queue_children(A, 0, 0, wave_id, active, tree, tree, 0, hh, tir);
            if (active) {
                if (kfirst == A.nsub && !(hh.refl > 0 || hh.refr > 0)) {
                    tr += hh.acc.x; tg += hh.acc.y; tb += hh.acc.z;
                } else {
                    if (kfirst == A.nsub) kfirst = sub;
                    A.rcol[tree] = make_float4(hh.acc.x, hh.acc.y, hh.acc.z, hh.dist);
                    A.rinfo[tree] = node_info(hh, tir);
                    A.rchild[tree] = ch;
                }
            }
        }
    }
    if (active) A.psum[pix] = make_float4(tr, tg, tb, __int_as_float(kfirst));
    if (COUNT) {
        const unsigned long long c[4] = {cnt.traced, cnt.shadow, cnt.tests, cnt.tir};
        flush_counters<4>(counters, c);
    }
}

// Level L = 1..5: a grid of resident blocks; wave w takes 64-ray pages
// w, w + #waves, ... of the level's queue.
#ifndef RT_WH_LEVEL_MINWAVES
#define RT_WH_LEVEL_MINWAVES RT_WH_MINWAVES
#endif
template <bool COUNT>
__global__ void __launch_bounds__(256, RT_WH_LEVEL_MINWAVES)
level_kernel(WfArgs A, int L, unsigned long long *__restrict__ counters)
{
    __shared__ Scene S;
    load_scene(S, A.scene);
    const SegView v = seg_view(A, L);
    const int nbase = next_base(v);                 // level L+1's pool base
    if (L < LEVELS - 1 && blockIdx.x == 0 && threadIdx.x == 0) CNT(A, C_BASE + L + 1) = nbase;
    const int lane = __lane_id();
    const int wave_id = (blockIdx.x << 2) + (threadIdx.x >> 6);
    Counts cnt = {0, 0, 0, 0};
    int base, nvalid;
    for (int k = wave_id; seg_chunk(v, k, base, nvalid); k += gridDim.x << 2) {
        const int q = base + lane;
        const bool active = lane < nvalid;
        Hit hh;
        bool tir = false;
        int tree = 0, node = 0;
        if (active) {
            const float4 a = A.ia[q], b = A.ib[q];
            ray3 r;
            r.o = mk(a.x, a.y, a.z);
            r.d = mk(a.w, b.x, b.y);
            tree = __float_as_int(b.w) & TREE_MASK;
            node = __float_as_int(b.w) >> TREE_BITS;
            hh = trace<COUNT>(S, r, b.z, cnt, A.ocl);
            tir = hh.refr > 0 && !hh.refr_ray_ok;
            if (tir && L < 5) cnt.tir++;                // node index < 31 (:398)
            A.lcol[q] = make_float4(hh.acc.x, hh.acc.y, hh.acc.z, hh.dist);
            if (L < LEVELS - 1) A.linfo[q] = node_info(hh, tir);   // level 5's info has no reader
        }
        if (L < LEVELS - 1) {
            const int2 ch = queue_children(A, L, nbase, wave_id, active, q, tree, node, hh, tir);
            if (active) A.lchild[q] = ch;
        }
    }
    if (COUNT) {
        const unsigned long long c[4] = {cnt.traced, cnt.shadow, cnt.tests, cnt.tir};
        flush_counters<4>(counters, c);
    }
}

// Record of node `j` of `tree`, walking the child links from the root
// (heap position j+1: after its leading 1, bit 0 = reflection child, bit 1 =
// refraction child).  Returns false if the node was not traced.
__device__ bool find_node(const WfArgs &A, int tree, int j, int &lvl, int &slot)
{
    const unsigned h = (unsigned)j + 1u;
    const int depth = 31 - __builtin_clz(h);
    slot = tree;
    lvl = 0;
    for (int k = depth - 1; k >= 0; k--) {
        const int2 ch = lvl == 0 ? A.rchild[slot] : A.lchild[slot];
        slot = ((h >> k) & 1u) ? ch.y : ch.x;
        lvl++;
        if (slot < 0) return false;
    }
    return true;
}

// TIR nodes of level L (0..4): the reference traces their refraction child
// with its refr_Ray variable as the previous calls left it -- the refraction
// ray of the last node before this one in BFS order that wrote one, or the
// primary ray (raytracer.cpp:231-233, :373-374, :412).  Every node before it
// has been traced by now (levels <= L); queue that child into level L+1.
__global__ void __launch_bounds__(64)
tir_kernel(WfArgs A, int L, const float *__restrict__ sx_tab, const float *__restrict__ sy_tab, float DX,
           float DY)
{
    const int nt = min(CNT(A, C_TIR + L), A.tcap);
    const int nbase = level_base(A, L + 1);
    const int lim = seg_limit(A, nbase);
    for (int t = blockIdx.x * blockDim.x + threadIdx.x; t < nt; t += gridDim.x * blockDim.x) {
        const int4 e = A.tir[L][t];
        const int slot_self = e.x, tree = e.y, node = e.z;
        const float rin = __int_as_float(e.w);
        ray3 r;
        bool found = false, broken = false;
        for (int j = node - 1; j >= 0 && !found && !broken; j--) {
            int lv, sl;
            if (!find_node(A, tree, j, lv, sl)) continue;
            const int info = lv == 0 ? A.rinfo[sl] : A.linfo[sl];
            if (!(info & INFO_REFR_OK)) continue;
            const int c = (lv == 0 ? A.rchild[sl] : A.lchild[sl]).y;   // its own refraction child
            if (c < 0) { broken = true; break; }                       // not queued (overflow)
            const float4 a = A.ia[c], b = A.ib[c];
            r.o = mk(a.x, a.y, a.z);
            r.d = mk(a.w, b.x, b.y);
            found = true;
        }
        if (broken) { flag_tree(A, tree); continue; }
        if (!found) {
            const int sub = tree / A.npix, pix = tree % A.npix;
            const int x = pix % A.w, y = slab_row(A, pix / A.w);
            r = primary(sub, sx_tab[x], sy_tab[y], DX, DY, A.side);
        }
        const int seg = tree & (NSEG - 1);
        const int k = atomicAdd(&CNT(A, C_SEG + (L + 1) * NSEG + seg), 1);
        if (k >= lim) { flag_tree(A, tree); continue; }
        const int q = seg_slot(nbase, seg, k);
        put_item(A, L + 1, q, r, rin, tree, 2 * node + 2);
        if (L == 0) A.rchild[slot_self].y = q;
        else A.lchild[slot_self].y = q;
    }
}

// Back-accumulation of one node (raytracer.cpp:476-511): the refraction child
// (Beer factor from the node's own distance and colour, unless TIR) first,
// then the reflection child (colour x refl).  cx / cy: the children's final
// colours (read only where ch.x / ch.y >= 0).
__device__ __forceinline__ float4 accumulate(const Scene &S, float4 pc, int pinfo, int2 ch, float4 cx, float4 cy,
                                             bool ocl)
{
    const float4 pm = S.mat0[pinfo & 0xff];
    const auto refr = [&]() {
        if (ch.y < 0) return;
        float ax = cy.x, ay = cy.y, az = cy.z;
        if (!(pinfo & INFO_TIR)) {
            const float nd = -pc.w;
            ax = cy.x * rtm::expf(pm.x * 0.15f * nd);
            ay = cy.y * rtm::expf(pm.y * 0.15f * nd);
            az = cy.z * rtm::expf(pm.z * 0.15f * nd);
        }
        pc.x += ax; pc.y += ay; pc.z += az;
    };
    const auto refl = [&]() {
        if (ch.x < 0) return;
        pc.x += cx.x * pm.x * pm.w;
        pc.y += cx.y * pm.y * pm.w;
        pc.z += cx.z * pm.z * pm.w;
    };
    if (ocl) {                     // openCLcode.cl:199-233: reflection child first
        refl();
        refr();
    } else {
        refr();
        refl();
    }
    return pc;
}

// Final colour of pool node c, whose descendants D levels down are final:
// the D levels between are folded in registers, bottom-up per child, and
// never written back (nothing but their parent reads them).  D = 0: the
// node's colour as stored.  A level-5 node (no lchild record) is only ever
// reached with D = 0.
template <int D>
__device__ __forceinline__ float4 folded(const WfArgs &A, const Scene &S, int c)
{
    float4 cc = A.lcol[c];
    if constexpr (D > 0) {
        const int2 g = A.lchild[c];
        if (g.x >= 0 || g.y >= 0) {
            const float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
            const float4 cx = g.x >= 0 ? folded<D - 1>(A, S, g.x) : z;
            const float4 cy = g.y >= 0 ? folded<D - 1>(A, S, g.y) : z;
            cc = accumulate(S, cc, A.linfo[c], g, cx, cy, A.ocl);
        }
    }
    return cc;
}

// Back-accumulation of level L's nodes with their D levels below
// (folded<D>), written back: D = 1 is a launch per level (4, 3, 2, 1); D = 2
// folds levels (3 <- 4 <- 5) and (1 <- 2 <- 3) in two launches, the default
// (WF_BACKACC_LEVELS).  Levels written: only those a later launch or
// final_kernel reads as final.
template <int D>
__global__ void __launch_bounds__(256)
backacc_kernel(WfArgs A, int L)
{
    __shared__ Scene S;
    load_scene(S, A.scene);
    const SegView v = seg_view(A, L);
    const int lane = __lane_id();
    int base, nvalid;
    for (int k = (blockIdx.x << 2) + (threadIdx.x >> 6); seg_chunk(v, k, base, nvalid); k += gridDim.x << 2) {
        const int q = base + lane;
        if (lane >= nvalid) continue;
        const int2 ch = A.lchild[q];
        if (ch.x < 0 && ch.y < 0) continue;
        const float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
        const float4 cx = ch.x >= 0 ? folded<D - 1>(A, S, ch.x) : z;
        const float4 cy = ch.y >= 0 ? folded<D - 1>(A, S, ch.y) : z;
        A.lcol[q] = accumulate(S, A.lcol[q], A.linfo[q], ch, cx, cy, A.ocl);
    }
}

// Level 0 of the pixel's nine trees, folded with the FD levels below it
// (level FD's colours final), the sum over sub-samples (:513-515) and the
// x28 / clamp / XRGB pack (:517-523).
template <int FD>
__global__ void __launch_bounds__(256)
final_kernel(WfArgs A, int row_end, uint32_t *__restrict__ out)
{
    __shared__ Scene S;
    load_scene(S, A.scene);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int x = blockIdx.x * 16 + (wave & 1) * 8 + (lane & 7);
    const int r = blockIdx.y * 16 + (wave >> 1) * 8 + (lane >> 3);
    const int y = slab_row(A, r);
    if (x >= A.w || y >= row_end) return;
    const int pix = r * A.w + x;
    const float4 ps = A.psum[pix];                          // the leading childless trees, summed by root_kernel
    float tr = ps.x, tg = ps.y, tb = ps.z;
    // The root records of all the pixel's remaining trees read in one round
    // (they do not depend on each other; a round per tree: final_kernel<1>
    // 39.6 us against 33.6), then each tree's children and its share of the
    // sum in sub-sample order.
    constexpr int T = 9;                                   // nsub <= 9 (3 x 3; 2 x 2 for openCLcode.cl)
    const int kf = __float_as_int(ps.w);
    float4 c0[T];
    int2 ch[T];
    int info[T];
    bool fl[T];
#pragma unroll
    for (int j = 0; j < T; j++) {
        const int sub = kf + j < A.nsub ? kf + j : kf;
        const int tree = sub * A.npix + pix;
        if (kf + j < A.nsub) {
            c0[j] = A.rcol[tree];
            ch[j] = A.rchild[tree];
            info[j] = A.rinfo[tree];
            fl[j] = flagged(A, tree);
        }
    }
#pragma unroll
    for (int j = 0; j < T; j++) {
        if (kf + j >= A.nsub) continue;
        float4 c = c0[j];
        if (!fl[j] && (ch[j].x >= 0 || ch[j].y >= 0)) {
            const float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
            const float4 cx = ch[j].x >= 0 ? folded<FD - 1>(A, S, ch[j].x) : z;
            const float4 cy = ch[j].y >= 0 ? folded<FD - 1>(A, S, ch[j].y) : z;
            c = accumulate(S, c, info[j], ch[j], cx, cy, A.ocl);
        }
        tr += c.x; tg += c.y; tb += c.z;
    }
    const float scale = A.ocl ? 64.0f : 28.0f;            // 256/4 (openCLcode.cl:238) or 256/9 (:517)
    int red = cvt_i32_x86(tr * scale), green = cvt_i32_x86(tg * scale), blue = cvt_i32_x86(tb * scale);
    if (red > 255) red = 255;
    if (green > 255) green = 255;
    if (blue > 255) blue = 255;
    out[(size_t)y * A.w + x] = (uint32_t)((red << 16) + (green << 8) + blue);
}

struct NodeStore {       // per-lane private tree records (only traced nodes touched)
    float4 col[NODES];   // colour.xyz, dist
    int info[NODES];     // hit primitive | INFO_TIR
    float4 ra[NODES];    // refl ray o.xyz, d.x
    float4 rb[NODES];    // refl ray d.yz, refr ray o.xy
    float4 rc[NODES];    // refr ray o.z, d.xyz
    float rin[NODES];    // *a_RIndex after the node's call
    int wf[NODES];       // the node's record slot in the wavefront pass, -1 if it did not trace it
};

__device__ __forceinline__ int level_of(int i) { return 31 - __builtin_clz(i + 1); }

// Sequential re-evaluation, in the reference's BFS order, of trees the level
// pass could not finish (a full queue): a 64-bit to-do mask (ctz = next node;
// children 2i+1 / 2i+2 are always later), the caller's refr_Ray variable
// carried across nodes (cur_refr), back-accumulation in decreasing index.
// Writes the tree's final level-0 colour into rcol[tree]; counts only the
// nodes the level pass did not trace.
template <bool COUNT>
__global__ void __launch_bounds__(64)
fixup_kernel(WfArgs A, const float *__restrict__ sx_tab, const float *__restrict__ sy_tab, float DX, float DY,
             unsigned long long *__restrict__ counters)
{
    const int nfix = CNT(A, C_FIX);
    if (nfix == 0) return;
    if (blockIdx.x == 0) {
        // Tell the host when a queue asked for more than its pages (a segment
        // counter past its limit) or a TIR list for more than its capacity:
        // the next frame gets a larger pool.
        const int lane = threadIdx.x;
        bool over = lane < LEVELS - 1 && CNT(A, C_TIR + lane) > A.tcap;
        for (int L = 1; L < LEVELS; L++) {
            const int base = level_base(A, L);
            over = over || CNT(A, C_SEG + L * NSEG + lane) > seg_limit(A, base);
        }
        if (__builtin_amdgcn_ballot_w64(over) != 0 && lane == 0) *(volatile int *)A.ovf = 1;
    }
    // blocks past the work leave before staging the scene
    if ((int)(blockIdx.x * blockDim.x) >= (nfix > A.fixcap ? (A.ntrees + 31) >> 5 : nfix)) return;
    __shared__ Scene S;
    load_scene(S, A.scene);
    const bool scan = nfix > A.fixcap;                  // the list overflowed: walk the bitmask
    const int nitems = scan ? (A.ntrees + 31) >> 5 : nfix;
    Counts cnt = {0, 0, 0, 0};
    for (int f = blockIdx.x * blockDim.x + threadIdx.x; f < nitems; f += gridDim.x * blockDim.x) {
      unsigned bits = scan ? A.fixbits[f] : 1u;
      while (bits) {
        const int bit = __builtin_ctz(bits);
        bits &= bits - 1u;
        const int tree = scan ? (f << 5) + bit : A.fixlist[f];
        const int sub = tree / A.npix, pix = tree % A.npix;
        const int x = pix % A.w, y = slab_row(A, pix / A.w);
        NodeStore ns;
        unsigned long long todo = 1, traced = 0;
        const ray3 root = primary(sub, sx_tab[x], sy_tab[y], DX, DY, A.side);
        ray3 cur_refr = root;          // the caller's refr_Ray variable (:373-374)
        while (todo) {
            const int i = __builtin_ctzll(todo);
            todo &= todo - 1;
            traced |= 1ull << i;
            ray3 r;
            float rin;
            int wf = -1;
            if (i == 0) {
                r = root; rin = 1.0f; wf = tree;
            } else {
                const int p = (i - 1) >> 1;
                const float4 a = ns.ra[p], b = ns.rb[p], c = ns.rc[p];
                if (i & 1) { r.o = mk(a.x, a.y, a.z); r.d = mk(a.w, b.x, b.y); }
                else       { r.o = mk(b.z, b.w, c.x); r.d = mk(c.y, c.z, c.w); }
                rin = ns.rin[p];
                if (ns.wf[p] >= 0) {
                    const int lp = level_of(p);
                    const int2 ch = lp == 0 ? A.rchild[ns.wf[p]] : A.lchild[ns.wf[p]];
                    wf = (i & 1) ? ch.x : ch.y;
                }
            }
            Counts c1 = {0, 0, 0, 0};
            Hit hh = trace<COUNT>(S, r, rin, c1, A.ocl);
            const bool tir = hh.refr > 0 && !hh.refr_ray_ok;
            if (wf < 0) {                  // not traced by the level pass: count it here
                cnt.traced += c1.traced; cnt.shadow += c1.shadow; cnt.tests += c1.tests;
                if (tir && i < NODES / 2) cnt.tir++;
            }
            ns.col[i] = make_float4(hh.acc.x, hh.acc.y, hh.acc.z, hh.dist);
            ns.info[i] = (hh.prim & 0xff) | (tir ? INFO_TIR : 0);
            ns.wf[i] = wf;
            if (hh.refr_ray_ok) cur_refr = hh.refr_ray;
            if (i < NODES / 2) {
                const bool cl = hh.refl > 0, cr = hh.refr > 0;
                if (cl || cr) {
                    const ray3 fl = hh.refl_ray, fr = cur_refr;
                    ns.ra[i] = make_float4(fl.o.x, fl.o.y, fl.o.z, fl.d.x);
                    ns.rb[i] = make_float4(fl.d.y, fl.d.z, fr.o.x, fr.o.y);
                    ns.rc[i] = make_float4(fr.o.z, fr.d.x, fr.d.y, fr.d.z);
                    ns.rin[i] = hh.rindex_out;
                    if (cl) todo |= 1ull << (2 * i + 1);
                    if (cr) todo |= 1ull << (2 * i + 2);
                }
            }
        }
        // Back-accumulation (:476-511): parents in decreasing index order; per
        // parent the refraction child then the reflection child (the CPU
        // path) or the reverse (openCLcode.cl:199-233).
        for (int p = NODES / 2 - 1; p >= 0; p--) {
            if (!((traced >> p) & 1ull)) continue;
            float4 pc = ns.col[p];
            const int pinfo = ns.info[p];
            const float4 pm = S.mat0[pinfo & 0xff];
            for (int k = 0; k < 2; k++) {
                const bool refr_side = A.ocl ? (k == 1) : (k == 0);
                const int c = refr_side ? 2 * p + 2 : 2 * p + 1;
                if (!((traced >> c) & 1ull)) continue;
                const float4 cc = ns.col[c];
                float ax = cc.x, ay = cc.y, az = cc.z;
                if (refr_side) {
                    if (!(pinfo & INFO_TIR)) {
                        const float nd = -pc.w;
                        ax = cc.x * rtm::expf(pm.x * 0.15f * nd);
                        ay = cc.y * rtm::expf(pm.y * 0.15f * nd);
                        az = cc.z * rtm::expf(pm.z * 0.15f * nd);
                    }
                } else {
                    ax = cc.x * pm.x * pm.w;
                    ay = cc.y * pm.y * pm.w;
                    az = cc.z * pm.z * pm.w;
                }
                pc.x += ax; pc.y += ay; pc.z += az;
            }
            ns.col[p] = pc;
        }
        A.rcol[tree] = ns.col[0];
      }
    }
    if (COUNT) {
        const unsigned long long c[4] = {cnt.traced, cnt.shadow, cnt.tests, cnt.tir};
        flush_counters<4>(counters, c);
    }
}

}  // namespace whitted
}  // namespace rt

// ------------------------------------------------------------------ host side
#include <stdlib.h>
#include <algorithm>
#include "rt_runtime.h"

namespace {

constexpr int SLOT_WF = 6;      // rtrt scratch slots of the level-pass arenas (two with two streams)
constexpr int SLOT_WF2 = 9;

// Trees per slab of the level pass.  A frame with more trees is rendered as
// several slabs, one after the other on the stream, so the arena is sized
// for one slab whatever the frame size (1080p: one slab; 4K: four).  Slabs
// interleave in groups of 16 rows (slab_row), so every slab holds the
// frame's mix of sphere / plane / background rows and so its queue fill.
constexpr long long SLAB_TREES = 18000000;
constexpr long long STREAM2_TREES = 4000000;   // frames from this size on: two slabs on two streams
#ifndef WF_SPLIT_P
#define WF_SPLIT_P 1                            // row groups of the first / second of those slabs per period
#define WF_SPLIT_Q 1
#endif
#ifndef WF_BACKACC_LEVELS
#define WF_BACKACC_LEVELS 2                     // levels folded per back-accumulation launch (1 or 2)
#endif
// Record pool (levels 1..5 together) as a fraction of the slab's trees, to
// start with.  The reference scene needs 0.83 at 1080p (14.2 M nodes for
// 17.1 M trees) but 0.94 at 640 x 480 (its rows [20, 410) hold more of the
// spheres); a tree whose node does not fit is finished by fixup_kernel,
// exactly but ~5x slower per frame, and the next frame's pool is 1.25x
// larger (rtrt::pool_fraction), so a denser scene costs a frame or two.
constexpr double POOL_FRAC = 0.9;

// m_SX / m_SY (Engine_InitRender raytracer.cpp:278-294, then the sequential
// m_SX += m_DX (:524) per pixel and m_SY += m_DY (:526) per row): lane 0
// runs the x recurrence, lane 1 the y one, with the reference's float adds.
// openCLcode.cl:22-23 semantics: SX = WX1 + x*DX, SY = WY1 + y*DY.
__global__ void __launch_bounds__(64) view_kernel(float *__restrict__ tab, int w, int h, float DX, float DY, int ocl)
{
    const float WX1 = -3.0f, WY1 = 2.25f;
    if (ocl) {
        for (int i = threadIdx.x; i < w + h; i += 64)
            tab[i] = i < w ? WX1 + i * DX : WY1 + (i - w) * DY;
        return;
    }
    if (threadIdx.x == 0) {
        float sx = WX1;
        for (int x = 0; x < w; x++) { tab[x] = sx; sx += DX; }
    } else if (threadIdx.x == 1) {
        float sy = WY1;
        sy += 20 * DY;
        for (int y = 0; y < h && y < 20; y++) tab[w + y] = 0.f;
        for (int y = 20; y < h; y++) { tab[w + y] = sy; sy += DY; }
    }
}

// Host wait for the previous frame (its arena, tables and staging slots).
int wait_frame(rtrt::DeviceState &st)
{
    hipError_t e = hipEventSynchronize(st.wf_done);
    if (e != hipSuccess) return rtrt::fail_hip(e, "rtw frame wait");
    st.wf_pending = false;
    return RT_OK;
}

// Device slot of at least `bytes` that the previous frame may still read:
// regrowing frees it, so wait for that frame first.
int frame_scratch(rtrt::DeviceState &st, int slot, size_t bytes, void **out)
{
    if (st.cap[slot] < bytes && st.wf_pending) {
        int rc = wait_frame(st);
        if (rc) return rc;
    }
    return rtrt::scratch(st, slot, bytes, out);
}

// View tables for (w, h, ocl) in slot SLOT_VIEW, (re)computed on `s` only
// when the frame size or semantics change (ordered after earlier frames by
// the caller's wait on wf_done).
int view_tables(rtrt::DeviceState &st, hipStream_t s, int w, int h, bool ocl, float DX, float DY,
                const float **d_sx, const float **d_sy)
{
    void *d = nullptr;
    int rc = frame_scratch(st, rtrt::SLOT_VIEW, sizeof(float) * ((size_t)w + h), &d);
    if (rc) return rc;
    if (st.vt_w != w || st.vt_h != h || st.vt_ocl != (int)ocl) {
        hipLaunchKernelGGL(view_kernel, dim3(1), dim3(64), 0, s, (float *)d, w, h, DX, DY, (int)ocl);
        if ((rc = rtrt::check_launch("rtw view_kernel"))) return rc;
        st.vt_w = w; st.vt_h = h; st.vt_ocl = (int)ocl;
    }
    *d_sx = (const float *)d;
    *d_sy = (const float *)d + w;
    return RT_OK;
}

// Device arena of the level pass (scratch slot SLOT_WF, grow-only) for a slab
// of `rows` rows: per tree a root record and a fixup bit; the record pool of
// levels 1..5; per level 0..4 a TIR list.
int wavefront_arena(rtrt::DeviceState &st, int slot, int w, int rows, int nsub, rt::whitted::WfArgs *A)
{
    using namespace rt::whitted;
    const size_t T = (size_t)w * rows * nsub;
    if (T > (size_t)TREE_MASK + 1) return rtrt::fail(RT_ERR_INVALID, "rtw: slab too large");   // item tree word
    // RT_WHITTED_QUEUE_CAP lowers the pool (test hook: exercises the
    // overflow -> fixup path).
    int *ovf = nullptr;
    size_t P = (size_t)(T * rtrt::pool_fraction(st, rtrt::POOL_WHITTED, (long long)T, POOL_FRAC, &ovf));
    if (const char *e = getenv("RT_WHITTED_QUEUE_CAP")) {
        const long long v = atoll(e);
        if (v > 0 && (size_t)v < P) P = (size_t)v;
    }
    P = std::max<size_t>((P + PAGE_ROW - 1) / PAGE_ROW, 1) * PAGE_ROW;
    const size_t TC = std::max<size_t>(P / 64, 1024);   // TIR list per level
    const size_t FC = std::max<size_t>(T / 16, 1024);   // fixup list
    const size_t FB = (T + 31) / 32 * 4;                // fixup bits
    auto al = [](size_t b) { return (b + 255) & ~(size_t)255; };
    const size_t root_b = al(T * 16) + al(T * 4) + al((size_t)w * rows * 16) + al(T * 8) + al(FB) + al(FC * 4);
    const size_t pool_b = al(P * 16) * 3 + al(P * 4) + al(P * 8);
    const size_t bytes = al(sizeof(Scene)) + root_b + pool_b + (LEVELS - 1) * al(TC * 16) +
                         al(sizeof(int) * C_TOTAL * CSTRIDE);
    void *base = nullptr;
    int rc = frame_scratch(st, slot, bytes, &base);
    if (rc) return rc;
    char *p = (char *)base;
    auto take = [&](size_t b) { char *q = p; p += al(b); return q; };
    A->scene = (const Scene *)take(sizeof(Scene));
    A->rcol = (float4 *)take(T * 16);
    A->rinfo = (int *)take(T * 4);
    A->psum = (float4 *)take((size_t)w * rows * 16);
    A->rchild = (int2 *)take(T * 8);
    A->fixbits = (unsigned *)take(FB);
    A->fixlist = (int *)take(FC * 4);
    A->ia = (float4 *)take(P * 16);
    A->ib = (float4 *)take(P * 16);
    A->lcol = (float4 *)take(P * 16);
    A->linfo = (int *)take(P * 4);
    A->lchild = (int2 *)take(P * 8);
    for (int L = 0; L < LEVELS; L++) A->tir[L] = L < LEVELS - 1 ? (int4 *)take(TC * 16) : nullptr;
    A->count = (int *)take(sizeof(int) * C_TOTAL * CSTRIDE);
    A->ovf = ovf;
    A->pool = (int)P;
    A->fixcap = (int)FC;
    A->tcap = (int)TC;
    A->ntrees = (int)T;
    A->npix = w * rows;
    A->w = w;
    return RT_OK;
}

// Resident blocks of a 256-thread kernel on this device (persistent grids).
template <class K>
int resident_blocks(K kernel)
{
    int dev = 0, cus = 0, per = 0;
    if (hipGetDevice(&dev) != hipSuccess) return 1024;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return 1024;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, kernel, 256, 0) != hipSuccess || per < 1) per = 1;
    return cus * per;
}

template <bool COUNT>
int launch_wavefront(const rt::whitted::WfArgs &A, int w, int rows, int row_end, const float *d_sx,
                     const float *d_sy, float DX, float DY, unsigned long long *cnt, hipStream_t s, uint32_t *d_xrgb)
{
    using namespace rt::whitted;
    static const int level_blocks = resident_blocks(level_kernel<COUNT>);
    const dim3 tiles((w + 15) / 16, (rows + 15) / 16), block(256);
    const int qblocks = (int)std::min<long long>(((long long)A.pool + 255) / 256, 2048);
    hipLaunchKernelGGL(root_kernel<COUNT>, tiles, block, 0, s, A, row_end, d_sx, d_sy, DX, DY, cnt);
    for (int L = 1; L < LEVELS; L++) {
        hipLaunchKernelGGL(tir_kernel, dim3(64), dim3(64), 0, s, A, L - 1, d_sx, d_sy, DX, DY);   // (256 / 1024 blocks: level)
        hipLaunchKernelGGL(level_kernel<COUNT>, dim3(level_blocks), block, 0, s, A, L, cnt);
    }
    hipLaunchKernelGGL(fixup_kernel<COUNT>, dim3(256), dim3(64), 0, s, A, d_sx, d_sy, DX, DY, cnt);
    // Back-accumulation schedule (RT_WHITTED_BACKACC, A/B): 1 = a launch per
    // level 4..1; 2 = levels (3 <- 4 <- 5), (1 <- 2 <- 3); 3 = (2 <- 3 <- 4 <- 5)
    // and the final kernel folds 0 <- 1 <- 2; 4 = (3 <- 4 <- 5) and the final
    // kernel folds 0 <- 1 <- 2 <- 3.
    static const int backacc = [] {
        const char *e = getenv("RT_WHITTED_BACKACC");
        const int v = e ? atoi(e) : WF_BACKACC_LEVELS;
        return v >= 1 && v <= 4 ? v : WF_BACKACC_LEVELS;
    }();
    static_assert(LEVELS == 6, "the back-accumulation schedules assume levels 0..5");
    if (backacc == 1) {
        for (int L = LEVELS - 2; L >= 1; L--)
            hipLaunchKernelGGL(backacc_kernel<1>, dim3(qblocks), block, 0, s, A, L);
        hipLaunchKernelGGL(final_kernel<1>, tiles, block, 0, s, A, row_end, d_xrgb);
    } else if (backacc == 2) {
        hipLaunchKernelGGL(backacc_kernel<2>, dim3(qblocks), block, 0, s, A, 3);
        hipLaunchKernelGGL(backacc_kernel<2>, dim3(qblocks), block, 0, s, A, 1);
        hipLaunchKernelGGL(final_kernel<1>, tiles, block, 0, s, A, row_end, d_xrgb);
    } else if (backacc == 3) {
        hipLaunchKernelGGL(backacc_kernel<3>, dim3(qblocks), block, 0, s, A, 2);
        hipLaunchKernelGGL(final_kernel<2>, tiles, block, 0, s, A, row_end, d_xrgb);
    } else {
        hipLaunchKernelGGL(backacc_kernel<2>, dim3(qblocks), block, 0, s, A, 3);
        hipLaunchKernelGGL(final_kernel<3>, tiles, block, 0, s, A, row_end, d_xrgb);
    }
    return rtrt::check_launch("rtw wavefront kernels");
}

int render_async(const rt_primitive *d_prims, int nprims, uint32_t *d_xrgb, int w, int h, int row_begin,
                 int row_end, uint64_t *d_counters, void *stream, bool ocl)
{
    rtrt::DeviceState *st;
    int rc = rtrt::state(&st);
    if (rc) return rc;
    std::lock_guard<std::recursive_mutex> lk(st->mu);
    hipStream_t s = (hipStream_t)stream;
    // The arena and view tables belong to the device: order this frame after
    // the previous one, whatever stream that ran on.
    if (st->wf_pending) {
        hipError_t e = hipStreamWaitEvent(s, st->wf_done, 0);
        if (e != hipSuccess) return rtrt::fail_hip(e, "rtw_render_async wait");
    }
    const float DX = (3.0f - -3.0f) / w, DY = (-2.25f - 2.25f) / h;    // Engine_InitRender / openCLcode.cl:20-21
    const float *d_sx, *d_sy;
    if ((rc = view_tables(*st, s, w, h, ocl, DX, DY, &d_sx, &d_sy))) return rc;
    const int rows = row_end - row_begin;
    const int side = ocl ? 2 : 3, nsub = side * side;
    const int ngroups = (rows + 15) / 16;                // 16-row groups (slab_row)
    long long nslab = ((long long)w * ngroups * 16 * nsub + SLAB_TREES - 1) / SLAB_TREES;
    if (const char *e = getenv("RT_WHITTED_SLABS")) nslab = std::max(1, atoi(e));   // test hook
    {   // at most 2^TREE_BITS trees a slab (the queued items' tree word)
        const long long max_groups = std::max<long long>(1, ((long long)rt::whitted::TREE_MASK + 1) / ((long long)w * 16 * nsub));
        nslab = std::max<long long>(nslab, (ngroups + max_groups - 1) / max_groups);
    }
    nslab = std::min<long long>(std::max<long long>(nslab, 1), ngroups);
    // Frames of >= 4 M trees run as (at least) two slabs that alternate
    // between the caller's stream and a second one, each with its own arena:
    // one slab's launches fill the tails of the other's, and its
    // HBM-bound back-accumulation runs beside the other's tracing (1080p:
    // 2.00 -> 1.85 ms; the same two slabs on one stream: 2.15 ms).
    // RT_WHITTED_STREAMS=1/2 overrides (A/B).
    int nstream = (long long)w * ngroups * 16 * nsub >= STREAM2_TREES ? 2 : 1;
    if (const char *e = getenv("RT_WHITTED_STREAMS")) nstream = atoi(e) >= 2 ? 2 : 1;
    if (nstream == 2) {
        // Two arenas are live at once: each slab holds at most SLAB_TREES / 2
        // trees, so both together stay within one single-stream arena (1080p
        // window: 2 slabs as before; full-height 1080p 3, 3840x2400 10).
        const long long half_groups = std::max<long long>(1, (SLAB_TREES / 2) / ((long long)w * 16 * nsub));
        nslab = std::max<long long>(nslab, std::max<long long>(2, (ngroups + half_groups - 1) / half_groups));
        nslab = std::min<long long>(nslab, ngroups);
        if (nslab < 2) nstream = 1;
    }
    // Two slabs on two streams: the second slab's root kernel can start only
    // once the first's root grid is dispatched (~0.37 ms in at 1080p), so
    // with equal slabs the second ends ~0.16 ms after the first
    // (profiles/r03/whitted_two_stream_timeline.txt).  The first takes p of
    // every p + q row groups (RT_WHITTED_SPLIT=p,q; 1,1: equal).  The
    // two-arena memory bound above holds for the equal split only: an
    // unequal one gives the larger slab p / (p + q) of the groups, up to
    // 2 max(p, q) / (p + q) of a half arena (an A/B hook; the default is 1,1).
    int sp_p = 1, sp_q = 1;
    if (nstream == 2 && nslab == 2) {
        sp_p = WF_SPLIT_P;
        sp_q = WF_SPLIT_Q;
        if (const char *e = getenv("RT_WHITTED_SPLIT")) sscanf(e, "%d,%d", &sp_p, &sp_q);   // A/B
        sp_p = std::min(std::max(sp_p, 1), 64);
        sp_q = std::min(std::max(sp_q, 1), 64);
    }
    const int period = sp_p + sp_q;
    const auto split_groups = [&](int k) {      // 16-row groups of slab k of an unequal pair
        const int full = ngroups / period, rem = ngroups % period;
        return k == 0 ? full * sp_p + std::min(rem, sp_p) : full * sp_q + std::max(0, std::min(rem - sp_p, sp_q));
    };
    const bool unequal = nstream == 2 && nslab == 2 && !(sp_p == 1 && sp_q == 1);
    const int slab_rows = unequal ? std::max(split_groups(0), split_groups(1)) * 16
                                  : (int)((ngroups + nslab - 1) / nslab) * 16;
    rt::whitted::WfArgs A[2];
    hipStream_t ss[2] = {s, s};
    if (nstream == 2) {
        if ((rc = rtrt::aux_stream(*st))) return rc;
        ss[1] = st->aux;
        hipError_t e = hipEventRecord(st->fork_ev, s);
        if (e == hipSuccess) e = hipStreamWaitEvent(st->aux, st->fork_ev, 0);
        if (e != hipSuccess) return rtrt::fail_hip(e, "rtw_render_async fork");
    }
    unsigned long long *cnt = (unsigned long long *)d_counters;
    // (after the fork, an error return still joins the second stream back)
    const auto bail = [&](int code) { return nstream == 2 ? rtrt::join_aux_on_error(*st, s, code) : code; };
    for (int i = 0; i < nstream; i++) {
        if ((rc = wavefront_arena(*st, i ? SLOT_WF2 : SLOT_WF, w, slab_rows, nsub, &A[i]))) return bail(rc);
        A[i].side = side;
        A[i].nsub = nsub;
        A[i].ocl = ocl;
        A[i].row_stride = unequal ? period : (int)nslab;
        A[i].row_count = unequal ? (i == 0 ? sp_p : sp_q) : 1;
    }
    for (int k = 0; k < (int)nslab; k++) {
        rt::whitted::WfArgs &a = A[k % nstream];
        hipStream_t sk = ss[k % nstream];
        const int srows = unequal ? split_groups(k) * 16 : (int)((ngroups - k + nslab - 1) / nslab) * 16;
        if (srows == 0) continue;                // (an unequal pair over fewer groups than its period)
        a.row_begin = row_begin + 16 * (unequal && k == 1 ? sp_p : k);
        a.npix = w * srows;
        a.ntrees = a.npix * nsub;
        // counters and tree flag words zeroed; the arena's scene image built by
        // its first slab (16-B words: the arena rounds every part to 256 B)
        const auto words = [](size_t bytes) { return (int)((bytes + 15) / 16); };
        const int nz0 = words(sizeof(int) * rt::whitted::C_TOTAL * rt::whitted::CSTRIDE);
        const int nz1 = words(sizeof(unsigned) * (((size_t)a.ntrees + 31) / 32));
        const int pblocks = std::min(1024, std::max(1, (nz0 + nz1 + 255) / 256));
        hipLaunchKernelGGL(rt::whitted::prep_kernel, dim3(pblocks), dim3(256), 0, sk, k < nstream ? d_prims : nullptr,
                           nprims, (rt::whitted::Scene *)a.scene, (uint4 *)a.count, nz0, (uint4 *)a.fixbits, nz1);
        rc = cnt ? launch_wavefront<true>(a, w, srows, row_end, d_sx, d_sy, DX, DY, cnt, sk, d_xrgb)
                 : launch_wavefront<false>(a, w, srows, row_end, d_sx, d_sy, DX, DY, cnt, sk, d_xrgb);
        if (rc) return bail(rc);
    }
    if (nstream == 2) {
        hipError_t e = hipEventRecord(st->join_ev, st->aux);
        if (e == hipSuccess) e = hipStreamWaitEvent(s, st->join_ev, 0);
        if (e != hipSuccess) return bail(rtrt::fail_hip(e, "rtw_render_async join"));
    }
    hipError_t e = hipEventRecord(st->wf_done, s);
    if (e != hipSuccess) return rtrt::fail_hip(e, "rtw_render_async record");
    st->wf_pending = true;
    return RT_OK;
}

}  // namespace

extern "C" int rtw_render_async(const rt_primitive *d_prims, int nprims, uint32_t *d_xrgb, int w,
                                int h, int row_begin, int row_end, uint64_t *d_counters,
                                void *stream)
{
    if (!d_prims || !d_xrgb || nprims < 1 || nprims > rt::whitted::MAXP || w < 1 || h < 1)
        return rtrt::fail(RT_ERR_INVALID, "rtw_render_async: bad arguments");
    if (row_begin < 20 || row_end > h || row_begin >= row_end)
        return rtrt::fail(RT_ERR_INVALID, "rtw_render_async: rows must satisfy 20 <= row_begin < row_end <= h");
    return render_async(d_prims, nprims, d_xrgb, w, h, row_begin, row_end, d_counters, stream, false);
}

extern "C" int rtw_render_ocl_async(const rt_primitive *d_prims, int nprims, uint32_t *d_xrgb, int w, int h,
                                    uint64_t *d_counters, void *stream)
{
    if (!d_prims || !d_xrgb || nprims < 1 || nprims > rt::whitted::MAXP || w < 1 || h < 1)
        return rtrt::fail(RT_ERR_INVALID, "rtw_render_ocl_async: bad arguments");
    const int row_end = std::min(h, 530);
    if (row_end <= 20) return RT_OK;                 // the kernel's window is empty
    return render_async(d_prims, nprims, d_xrgb, w, h, 20, row_end, d_counters, stream, true);
}

extern "C" int rtw_render_ocl(const rt_primitive *prims, int nprims, uint32_t *xrgb, int w, int h,
                              uint64_t *counters)
{
    if (!prims || !xrgb || nprims < 1 || nprims > rt::whitted::MAXP || w < 1 || h < 1)
        return rtrt::fail(RT_ERR_INVALID, "rtw_render_ocl: bad arguments");
    const int row_end = std::min(h, 530);
    if (row_end <= 20) {
        if (counters) counters[0] = counters[1] = counters[2] = counters[3] = 0;
        return RT_OK;
    }
    rtrt::DeviceState *st;
    int rc = rtrt::state(&st);
    if (rc) return rc;
    std::lock_guard<std::recursive_mutex> lk(st->mu);
    // slots 0..2 may still feed a frame issued on another stream
    if (st->wf_pending && (rc = wait_frame(*st))) return rc;
    const size_t frame_bytes = sizeof(uint32_t) * (size_t)w * h;
    void *d_prims, *d_frame, *d_cnt;
    if ((rc = rtrt::scratch(*st, 0, sizeof(rt_primitive) * nprims, &d_prims))) return rc;
    if ((rc = rtrt::scratch(*st, 1, frame_bytes, &d_frame))) return rc;
    if ((rc = rtrt::scratch(*st, 2, 4 * sizeof(uint64_t), &d_cnt))) return rc;
    hipStream_t s = st->stream;
    hipError_t e = hipMemcpyAsync(d_prims, prims, sizeof(rt_primitive) * nprims, hipMemcpyHostToDevice, s);
    if (e == hipSuccess && counters) e = hipMemsetAsync(d_cnt, 0, 4 * sizeof(uint64_t), s);
    if (e != hipSuccess) return rtrt::fail_hip(e, "rtw_render_ocl H2D");
    rc = render_async((const rt_primitive *)d_prims, nprims, (uint32_t *)d_frame, w, h, 20, row_end,
                      counters ? (uint64_t *)d_cnt : nullptr, s, true);
    if (rc) return rc;
    const size_t off = sizeof(uint32_t) * (size_t)20 * w, len = sizeof(uint32_t) * (size_t)(row_end - 20) * w;
    e = hipMemcpyAsync((char *)xrgb + off, (char *)d_frame + off, len, hipMemcpyDeviceToHost, s);
    if (e == hipSuccess && counters)
        e = hipMemcpyAsync(counters, d_cnt, 4 * sizeof(uint64_t), hipMemcpyDeviceToHost, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    if (e != hipSuccess) return rtrt::fail_hip(e, "rtw_render_ocl D2H");
    return RT_OK;
}

extern "C" int rtw_render(const rt_primitive *prims, int nprims, uint32_t *xrgb, int w, int h,
                          int row_begin, int row_end, uint64_t *counters)
{
    if (!prims || !xrgb || nprims < 1 || nprims > rt::whitted::MAXP || w < 1 || h < 1)
        return rtrt::fail(RT_ERR_INVALID, "rtw_render: bad arguments");
    if (row_begin < 20 || row_end > h || row_begin >= row_end)
        return rtrt::fail(RT_ERR_INVALID, "rtw_render: rows must satisfy 20 <= row_begin < row_end <= h");
    rtrt::DeviceState *st;
    int rc = rtrt::state(&st);
    if (rc) return rc;
    std::lock_guard<std::recursive_mutex> lk(st->mu);
    // slots 0..2 may still feed a frame issued on another stream
    if (st->wf_pending && (rc = wait_frame(*st))) return rc;
    const size_t frame_bytes = sizeof(uint32_t) * (size_t)w * h;
    void *d_prims, *d_frame, *d_cnt;
    if ((rc = rtrt::scratch(*st, 0, sizeof(rt_primitive) * nprims, &d_prims))) return rc;
    if ((rc = rtrt::scratch(*st, 1, frame_bytes, &d_frame))) return rc;
    if ((rc = rtrt::scratch(*st, 2, 4 * sizeof(uint64_t), &d_cnt))) return rc;
    hipStream_t s = st->stream;
    hipError_t e = hipMemcpyAsync(d_prims, prims, sizeof(rt_primitive) * nprims, hipMemcpyHostToDevice, s);
    if (e != hipSuccess) return rtrt::fail_hip(e, "rtw_render H2D prims");
    // Rows outside [row_begin,row_end) are left untouched: copy only the window back.
    if (counters && (e = hipMemsetAsync(d_cnt, 0, 4 * sizeof(uint64_t), s)) != hipSuccess)
        return rtrt::fail_hip(e, "rtw_render memset");
    rc = rtw_render_async((const rt_primitive *)d_prims, nprims, (uint32_t *)d_frame, w, h, row_begin,
                          row_end, counters ? (uint64_t *)d_cnt : nullptr, s);
    if (rc) return rc;
    const size_t off = sizeof(uint32_t) * (size_t)row_begin * w;
    const size_t len = sizeof(uint32_t) * (size_t)(row_end - row_begin) * w;
    e = hipMemcpyAsync((char *)xrgb + off, (char *)d_frame + off, len, hipMemcpyDeviceToHost, s);
    if (e != hipSuccess) return rtrt::fail_hip(e, "rtw_render D2H frame");
    if (counters && (e = hipMemcpyAsync(counters, d_cnt, 4 * sizeof(uint64_t), hipMemcpyDeviceToHost, s)) != hipSuccess)
        return rtrt::fail_hip(e, "rtw_render D2H counters");
    e = hipStreamSynchronize(s);
    if (e != hipSuccess) return rtrt::fail_hip(e, "rtw_render sync");
    return RT_OK;
}
