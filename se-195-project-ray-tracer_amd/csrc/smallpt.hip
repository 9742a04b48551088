// smallpt.hip -- gfx950 kernel for the Monte-Carlo hot path of smallptgpu-v1.6.
//
// Computes what nsamples successive UpdateRenderingCPU passes
// (smallptCPU.cpp:77-132) compute: per pixel a camera ray from the pixel's
// own MWC RNG (simplernd.h:34-48), RadiancePathTracing (geomfunc.h:167-338)
// or RadianceDirectLighting (:340-483), the running average into the
// flipped colour slot (smallptCPU.cpp:110-118) and the toInt pack
// (vec.h:62, smallptCPU.cpp:120-122).  Results match the CPU path bit for bit
// (the float ops are the reference's, in its order; glibc sinf/cosf/powf are
// reproduced by rt_glibc_math.h), well inside the 1e-4 HDR tolerance.
//
// Mapping (MI355X-first, not a port of rendering_kernel.cl):
//   * one lane per pixel, a wave per 8x8 tile (launch_shape: 4 or 16 waves
//     per block, a block's waves spread over the row window);
//   * ALL samples of a launch run in-lane with path regeneration: the per-
//     lane loop advances one bounce per iteration and a lane whose path ended
//     immediately starts its next sample, so a wave's cost is the max over
//     lanes of the total bounces of nsamples paths (~ the mean for spp >> 1),
//     not the sum over samples of the per-sample max;
//   * RNG state, the colour accumulator and the path state stay in VGPRs for
//     the whole launch: HBM traffic is 32 B per pixel per launch, whatever
//     nsamples is;
//   * spheres are staged once per block into LDS as SoA float4 (centre,
//     rad^2) + material records and read with wave-uniform indices (LDS
//     broadcast); scenes larger than the LDS budget are read from global
//     memory through the same wave-uniform loop (L2/scalar-cache resident).
#include "rt_common.h"
#include "rt_glibc_math.h"

namespace rt {
namespace smallpt {

constexpr int MAX_LDS_BYTES = 96 * 1024; // per-block scene copy: 48 B per sphere + 48 B per light
constexpr float EPS = 0.01f;             // geom.h:29
constexpr float PI_F = 3.14159265358979323846f;
constexpr int DIFF = 0, SPEC = 1;   // REFR = 2 is the remaining case
#ifndef RT_SPT_QUNROLL
#define RT_SPT_QUNROLL 3
#endif

struct SphereGeo { float4 g; };          // centre.xyz, rad*rad (same float product as :42)

// GetRandom, simplernd.h:34-48, returning f = the float in [2, 4) that the
// reference maps to (f - 2) / 2.  Callers finish with fma(f, .5, c): for
// c = -1 that is (f - 2) / 2 and for c = -1.5 it is (f - 2) / 2 - .5f, exact
// (f / 2 - 1 and f / 2 - 1.5 are representable, as are the reference's two
// steps each), in one op instead of two or three.
__device__ __forceinline__ float get_random_f(uint32_t &s0, uint32_t &s1)
{
    s0 = 36969u * (s0 & 65535u) + (s0 >> 16);
    s1 = 18000u * (s1 & 65535u) + (s1 >> 16);
    const uint32_t ires = (s0 << 16) + s1;
    return __uint_as_float((ires & 0x007fffffu) | 0x40000000u);
}
__device__ __forceinline__ float get_random(uint32_t &s0, uint32_t &s1)
{
    return __builtin_fmaf(get_random_f(s0, s1), .5f, -1.f);
}

__device__ __forceinline__ float vdot(v3 a, v3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
__device__ __forceinline__ v3 vsmul(float k, v3 b) { return mk(k * b.x, k * b.y, k * b.z); }
__device__ __forceinline__ v3 vadd(v3 a, v3 b) { return mk(a.x + b.x, a.y + b.y, a.z + b.z); }
__device__ __forceinline__ v3 vsub(v3 a, v3 b) { return mk(a.x - b.x, a.y - b.y, a.z - b.z); }
__device__ __forceinline__ v3 vmul(v3 a, v3 b) { return mk(a.x * b.x, a.y * b.y, a.z * b.z); }
__device__ __forceinline__ v3 vnorm(v3 v) { const float l = inv_len(vdot(v, v)); return vsmul(l, v); }
__device__ __forceinline__ v3 vxcross(v3 a, v3 b)
{
    return mk(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}

// SphereIntersect, geomfunc.h:32-59 (g = centre.xyz, rad*rad), except that a
// miss returns +inf instead of 0: every caller tests "d != 0 && d < t" with a
// finite t, which for +inf is the single test "d < t".  The early return on
// det < 0 is kept as a branch: when no lane of the wave reaches the sphere's
// line the square root is skipped (measured +8 % over a branch-free select
// form).  NaN det is a miss, as in the reference.
constexpr float MISS = __builtin_inff();
__device__ __forceinline__ float sphere_hit(float4 g, const ray3 &r)
{
    const float opx = g.x - r.o.x, opy = g.y - r.o.y, opz = g.z - r.o.z;
    const float b = opx * r.d.x + opy * r.d.y + opz * r.d.z;
    const float det = b * b - (opx * opx + opy * opy + opz * opz) + g.w;
    if (det < 0.f) return MISS;
    const float sd = sqrt_exact(det);
    const float t1 = b - sd, t2 = b + sd;
    return t1 > EPS ? t1 : (t2 > EPS ? t2 : MISS);
}

// Sphere geometry for the nearest-hit / any-hit loops: LDS (per-block copy)
// or global-memory float4 array (scenes above MAX_LDS_BYTES), runtime count.
struct DynGeo {
    const float4 *g;
    int n;
    __device__ __forceinline__ int count() const { return n; }
    __device__ __forceinline__ float4 at(int i) const { return g[i]; }
};

struct Scene {                // per-block LDS copy (or global view for big scenes)
    const float4 *geo;        // centre, rad^2 (per-lane lookups of the hit sphere)
    const float4 *emi;        // emission.xyz, refl (as int bits)
    const float4 *col;        // colour.xyz, rad
    const float4 *lrec;       // per light (!viszero(e), ascending index): geo, col, emi
    int n, nlights;
};

// One ray query over the spheres, i descending, update iff d != 0 && d < t.
// With t = 1e20f on entry this is Intersect (geomfunc.h:71-92: nearest hit,
// highest index wins ties); with t = maxt on entry "some update happened" is
// IntersectP (:94-110: any d != 0 && d < maxt), and the first update is at
// the index where IntersectP's early exit stops (kept for the test counter).
// Returns the last updated index, -1 if none.
template <bool COUNT, class G>
__device__ __forceinline__ int query(const G &geo, const ray3 &r, float &t, int &first)
{
    int id = -1;
#pragma unroll 1
    for (int i = geo.count() - 1; i >= 0; i--) {
        const float d = sphere_hit(geo.at(i), r);
        const bool take = d < t;                           // d != 0 && d < t (miss = +inf)
        t = take ? d : t;
        id = take ? i : id;
        if (COUNT) first = (first < 0 && take) ? i : first;
    }
    return id;
}

// The same query with a branch-free sphere test and the next sphere's record
// loaded while the current one is tested (one LDS / scalar-load latency per
// query instead of one per sphere).  sqrt_nr is exact for det in [2^-96,
// inf); for det < 0 or NaN it returns NaN, and NaN roots fail both "> EPS"
// tests -- the reference's miss; for det = +inf it returns NaN where sqrtf
// returns +inf, whose root b + inf is never "< t" for the finite t of
// every caller -- a miss either way.  Only |det| < 2^-96 (where sqrt_nr
// is not sqrtf, e.g. det = +-0) is unsafe: any lane that meets one in the
// whole query has the wave redo the query with the exact per-sphere test.
template <bool COUNT, class G>
__device__ __forceinline__ int query_bf(const G &geo, const ray3 &r, float &t, int &first)
{
    const float t_in = t;
    int id = -1;
    bool bad = false;
#pragma unroll RT_SPT_QUNROLL
    for (int i = geo.count() - 1; i >= 0; i--) {
        const float4 g = geo.at(i);
        const float opx = g.x - r.o.x, opy = g.y - r.o.y, opz = g.z - r.o.z;
        const float b = opx * r.d.x + opy * r.d.y + opz * r.d.z;
        const float det = b * b - (opx * opx + opy * opy + opz * opz) + g.w;
        bad = bad || fabsf(det) < 0x1p-96f;
        const float sd = sqrt_nr(det);
        const float t1 = b - sd, t2 = b + sd;
        // SphereIntersect's distance is t1 if t1 > EPS, else t2 if t2 > EPS,
        // else a miss: d = t1 > EPS ? t1 : t2, taken iff d > EPS && d < t
        // (false for NaN) -- one select fewer than materialising the miss.
        const float d = t1 > EPS ? t1 : t2;
        const bool take = d > EPS && d < t;
        t = take ? d : t;
        id = take ? i : id;
        if (COUNT) first = (first < 0 && take) ? i : first;
    }
    if (wave_any(bad)) {
        t = t_in;
        first = -1;
        id = query<COUNT>(geo, r, t, first);
    }
    return id;
}

// Two queries in one pass over the spheres (single-light scenes, see
// render_kernel<..., DUAL>): the path ray's nearest hit (t = 1e20f on entry,
// as query_bf) and, for lanes with sh set, the pending shadow ray's any hit
// (ts = maxt on entry; "some update happened" = IntersectP true, the first
// update = its early-exit index for the test counter).  Each sphere record
// is loaded once for both rays, and the two dependency chains interleave.
// Uncounted, the shadow ray only needs "some distance in (EPS, maxt)"
// (geomfunc.h:94-110 with a fixed maxt): an occluded flag, not a running
// minimum and index -- three VALU operations fewer per sphere.
template <bool COUNT, class G>
__device__ __forceinline__ void query2_bf(const G &geo, const ray3 &r, float &t, int &id, const ray3 &rs, bool sh,
                                          float &ts, int &ids, int &firsts)
{
    const float t_in = t, ts_in = ts;
    int first = -1;
    id = -1;
    ids = -1;
    bool bad = false, occ = false;
#pragma unroll RT_SPT_QUNROLL
    for (int i = geo.count() - 1; i >= 0; i--) {
        const float4 g = geo.at(i);
        {
            const float opx = g.x - r.o.x, opy = g.y - r.o.y, opz = g.z - r.o.z;
            const float b = opx * r.d.x + opy * r.d.y + opz * r.d.z;
            const float det = b * b - (opx * opx + opy * opy + opz * opz) + g.w;
            bad = bad || fabsf(det) < 0x1p-96f;
            const float sd = sqrt_nr(det);
            const float t1 = b - sd, t2 = b + sd;
            const float d = t1 > EPS ? t1 : t2;          // (query_bf: taken iff d > EPS && d < t)
            const bool take = d > EPS && d < t;
            t = take ? d : t;
            id = take ? i : id;
        }
        {
            const float opx = g.x - rs.o.x, opy = g.y - rs.o.y, opz = g.z - rs.o.z;
            const float b = opx * rs.d.x + opy * rs.d.y + opz * rs.d.z;
            const float det = b * b - (opx * opx + opy * opy + opz * opz) + g.w;
            bad = bad || (sh && fabsf(det) < 0x1p-96f);
            const float sd = sqrt_nr(det);
            const float t1 = b - sd, t2 = b + sd;
            const float d = t1 > EPS ? t1 : t2;
            const bool take = d > EPS && d < ts;
            if (COUNT) {
                ts = take ? d : ts;
                ids = take ? i : ids;
                firsts = (firsts < 0 && take) ? i : firsts;
            } else {
                occ = occ || take;
            }
        }
    }
    if (!COUNT) ids = occ ? 0 : -1;
    if (wave_any(bad)) {
        t = t_in;
        id = query<COUNT>(geo, r, t, first);
        ts = ts_in;
        firsts = -1;
        ids = query<COUNT>(geo, rs, ts, firsts);
    }
}

// ---------------------------------------------------------------------------
// Bounding-volume hierarchy for large scenes (BASELINE configs[4]: 10k
// spheres).  The reference tests every sphere for every ray (geomfunc.h:71-
// 110); the result is the minimum over spheres of the float distance d_i of
// SphereIntersect, ties to the highest index (Intersect), or "some d_i <
// maxt" (IntersectP).  Both are order-independent, so a traversal that
// computes d_i with the reference's exact float formula for every sphere it
// visits, and skips a sphere only when d_i provably cannot matter, returns
// identical bits.
//
// Skipping rule.  For a sphere (radius r, |c - o| = |op|) inside box B
// (centre C, half-diagonal R), a float distance t* puts the point o + t*.d
// within  m = 1.04e-3 * (|op| + r) + sqrt(e) * t*  of the sphere, hence of B:
//   * the float root b -+ sqrt(det) differs from the geometric one by at most
//     sqrt(|det error|) + |b error|, with |det error| <= ~18u max(|op|, r)^2
//     (u = 2^-24; det = b*b - op.op + rad^2 cancels in float) -> 1.04e-3 *
//     max(|op|, r);
//   * a direction with |d|^2 = 1 + e puts the formula's roots on a sphere of
//     radius sqrt(r^2 + e t*^2), i.e. sqrt(e) * t* further out.
// With |op| <= |o - C| + R, r <= R and t* <= |o - C| + 2R this is below
// (1.04e-3 + sqrt(e)) |o - C| + (1.04e-3 + 2 sqrt(e)) R.  The margin is
// alpha * |o - C| + BVH_ALPHA_R * R + BETA with a per-ray alpha = 2 x
// (1.04e-3 + sqrt(e' + 2^-22)) (e' the float-computed e, whose rounding the
// 2^-22 covers): twice the bound's first coefficient; BVH_ALPHA_R = 1/64 is
// 1.7 .. 7x the second for e < 2^-16, and beyond that nothing is culled
// (rays here are normalised or built from unit vectors: e ~ 1e-7, alpha ~
// 1/270).  tests/test_bvh_margin.py measures the float roots of grazing rays
// at ~0.57 of the bound.  So a node whose box, grown by m on every side, is not
// crossed by the ray between 0 and lim (the current nearest distance, or
// maxt) holds no sphere that could be taken; its spheres are skipped.  BETA
// and the same slack absorb the slab test's own rounding (approximate
// reciprocals and square root, relative ~1e-6) and the box corners'.
// Spheres whose radius dwarfs the rest (the ground) are tested first, for
// every ray, outside the hierarchy.
struct BvhView {
    const float4 *node;   // 8 octant layouts x 2 per node: (centre.xyz, link) (half-extent.xyz, ALPHA*R + BETA)
    const float4 *geo;    // spheres in hierarchy order: centre, rad^2
    const int *id;        // their reference indices
    const float4 *ageo;   // "always" spheres (tested first)
    const int *aid;
    int nalways, nnodes;
    const uint4 *wnode;   // the 8-wide layout (spt_bvh.h WideBuild: 7 x 16 B per node), staged in LDS
    const uint4 *wmax;    //   per node and slot the highest reference index below (2 x 16 B per node;
                          //   staged by the counted kernels only)
    int wnodes, wdepth;   //   its node count and depth (levels of wide nodes)
};
// (BVH_ALPHA_R = spt_bvh.h's ALPHA_R: applied on the host, in the node records' margin terms)
#ifndef RT_BVH_K
#define RT_BVH_K 2.f
#endif

#ifndef RT_BVH_BUDGET
#define RT_BVH_BUDGET 32    // walk steps per render-loop iteration before a lane's query is suspended
#endif
constexpr float BVH_K = RT_BVH_K;           // per-ray alpha: K x the bound's |o - C| coefficient
constexpr int BVH_LEAF_MAX = 4;             // spheres per leaf (host build: BVH_LEAF)

// One ray query through the hierarchy.  Nearest hit (shadow = false): t in
// = 1e20f, out = nearest distance, returns its index (highest on ties) or
// -1.  Any hit (shadow = true): t = maxt, returns an occluder index or -1;
// with COUNT the highest one (IntersectP's early-exit position, for the test
// counter), without COUNT the traversal stops at the first.
//
// The walk is latency-bound (one dependent node load per step, L1/L2 hits):
// every step loads both halves of the node record together and runs the slab
// test before branching on the node kind -- leaves are tested against their
// own grown box too -- and a leaf issues the loads of all its spheres and
// indices before the first test, so a step costs one memory latency (a first
// form that branched on the link word first and loaded per sphere paid two
// to five: configs[4] 11.1 -> 8.5 ms per 4 spp).

// A query's walk state, kept across loop iterations of render_kernel: the
// walk is resumable, so a lane whose walk is long does not hold up the
// other lanes of its wave (they shade and start their next queries while it
// continues).  t = nearest distance so far (any hit: maxt, unchanged), id =
// the result so far, node = next node in the ray's octant layout (nnodes:
// finished), pend = a crossed leaf not yet tested (first | count << 24).
// Leaf postponement: a lane may hold two crossed leaves and keeps stepping
// while it holds one; the wave tests pending leaves once >= BVH_BATCH/64 of
// its lanes in the walk cannot step (hold two, or reached the end with one).
constexpr int BVH_BATCH = 16;
struct BvhWalk {
    float t;
    int id, node, pend;
    unsigned m;             // 8-wide walk: node = the current node (-1: root not yet visited), m = its
    int sp, bpos;           //   children still to visit (visit order), sp = stacked (node, mask) entries,
                            //   bpos = hierarchy position of the best leaf hit so far (-1: none)
    int pend2;              // a second crossed leaf (only while pend holds one)
#ifdef RT_SPT_TRACE
    unsigned tr_leaf, tr_trips, tr_leafruns;   // tools-only phase stamps (s_memtime cycles, counts)
#endif
#ifdef RT_SPT_PROF
    unsigned pf_l[3], pf_w[3];   // tools-only: lanes / wave-executions of wide_walk calls, node steps, leaf passes
#endif
};
#ifdef RT_SPT_PROF
#define WALK_PROF(W, b)                                                                    \
    do {                                                                                   \
        (W).pf_l[b]++;                                                                     \
        if ((int)(threadIdx.x & 63) == __builtin_ctzll(__builtin_amdgcn_read_exec())) (W).pf_w[b]++; \
    } while (0)
#else
#define WALK_PROF(W, b) do {} while (0)
#endif

// Starts a query: the "always" spheres, then the walk from the root.
// Nearest hit (shadow = false): t = 1e20f on entry; any hit: t = maxt.
template <bool COUNT>
__device__ __forceinline__ void bvh_begin(const BvhView &B, const ray3 &r, bool shadow, float t, BvhWalk &W)
{
    const float maxt = t;
    int id = -1;
    for (int k = 0; k < B.nalways; k++) {
        const float d = sphere_hit(B.ageo[k], r);
        const int i = B.aid[k];
        if (shadow) {
            if (d < maxt && i > id) id = i;
        } else if (d < t || (d == t && i > id)) {
            t = d;
            id = i;
        }
    }
    W.t = t;
    W.id = id;
    W.node = (!COUNT && shadow && id >= 0) ? B.nnodes : 0;
    W.pend = 0;
    W.pend2 = 0;
}

// Advances the walks of the wave's lanes by up to RT_BVH_BUDGET steps
// (node visits); returns true for a lane whose query is complete: W.id is
// then the nearest sphere (highest index on ties) with W.t its distance, or
// for any hit an occluder index (COUNT: the highest one, IntersectP's
// early-exit position, for the test counter; without COUNT the walk stops
// at the first) or -1.
template <bool COUNT>
__device__ bool bvh_walk(const BvhView &B, const ray3 &r, bool shadow, BvhWalk &W)
{
    const float maxt = W.t;
    float t = W.t;
    int id = W.id, node = W.node, pend = W.pend, pend2 = W.pend2;
    // Slab test (culling only: its rounding is inside the margin; fused ops
    // are fine here and nowhere else).  Zero direction components become
    // +-1e-30 so no 0 * inf appears.
    const float dx = fabsf(r.d.x) < 1e-30f ? copysignf(1e-30f, r.d.x) : r.d.x;
    const float dy = fabsf(r.d.y) < 1e-30f ? copysignf(1e-30f, r.d.y) : r.d.y;
    const float dz = fabsf(r.d.z) < 1e-30f ? copysignf(1e-30f, r.d.z) : r.d.z;
    const float ix = __builtin_amdgcn_rcpf(dx), iy = __builtin_amdgcn_rcpf(dy), iz = __builtin_amdgcn_rcpf(dz);
    const float e = fabsf(r.d.x * r.d.x + r.d.y * r.d.y + r.d.z * r.d.z - 1.f);
    const float alpha = e < 0x1p-16f ? BVH_K * (1.04e-3f + __builtin_amdgcn_sqrtf(e + 0x1p-22f)) : 1e30f;
    // Layout of this ray's direction octant: near children first.  A 32-bit
    // element offset from the uniform base (one VGPR, not a 64-bit pointer).
    const unsigned lay = 2u * (unsigned)B.nnodes * ((dx < 0.f ? 1u : 0u) | (dy < 0.f ? 2u : 0u) | (dz < 0.f ? 4u : 0u));
    // Crossed leaves are postponed: a lane that reaches one keeps it pending
    // and steps on until it holds a second; the wave tests one pending leaf
    // per lane together once at least BVH_BATCH/64 of its lanes still in the
    // walk cannot step (or
    // none can), instead of running the leaf block for the one or two lanes
    // that reach a leaf in a given step.  The result does not depend on the
    // order spheres are tested in (minimum, ties to the highest index; or
    // "some occluder"); a leaf tested later than it was crossed only makes
    // the culling limit t of the steps in between looser, never wrong.
    int trips = 0;
    while (true) {
        if (node < B.nnodes && pend2 == 0) {
            const float4 a = B.node[lay + 2u * (unsigned)node], b = B.node[lay + 2u * (unsigned)node + 1u];
            const int link = __float_as_int(a.w);
            const float lim = shadow ? maxt : t;
            const float cx = a.x - r.o.x, cy = a.y - r.o.y, cz = a.z - r.o.z;
            const float dist = __builtin_amdgcn_sqrtf(__builtin_fmaf(cx, cx, __builtin_fmaf(cy, cy, cz * cz)));
            const float m = __builtin_fmaf(alpha, dist, b.w);
            const float tcx = cx * ix, tcy = cy * iy, tcz = cz * iz;                // slab centres
            const float hx = (b.x + m) * fabsf(ix), hy = (b.y + m) * fabsf(iy), hz = (b.z + m) * fabsf(iz);  // slab half-widths
            const float tn = fmaxf(fmaxf(tcx - hx, tcy - hy), tcz - hz);
            const float tf = fminf(fminf(tcx + hx, tcy + hy), tcz + hz);
            const bool cross = tn <= tf && tf >= 0.f && tn <= lim;
            int next = cross ? node + 1 : link;
            if (link < 0) {                              // leaf ~(first | count << 24); escape = next node
                next = node + 1;
                if (cross) {
                    if (pend == 0) pend = ~link;
                    else pend2 = ~link;
                }
            }
            node = next;
        }
        trips++;
        const unsigned long long pm = __builtin_amdgcn_ballot_w64(pend != 0);
        const unsigned long long sm = __builtin_amdgcn_ballot_w64(node < B.nnodes && pend2 == 0);
        if (pm == 0) {
            if (sm == 0 || trips >= RT_BVH_BUDGET) break;
            continue;
        }
        if (sm != 0 && trips < RT_BVH_BUDGET &&
            64 * __builtin_popcountll(pm & ~sm) < BVH_BATCH * __builtin_popcountll(pm | sm))
            continue;
#ifdef RT_SPT_TRACE
        const unsigned long long tr_l0 = __builtin_amdgcn_s_memtime();
        W.tr_leafruns++;
#endif
        if (pend != 0) {
            const int f = pend & 0xffffff, c = pend >> 24;
            float4 g[BVH_LEAF_MAX];
#pragma unroll
            for (int q = 0; q < BVH_LEAF_MAX; q++)        // all loads first: one latency per leaf
                g[q] = B.geo[f + (q < c ? q : 0)];
            // Branch-free sphere tests (as query_bf): sqrt_nr is exact for det
            // in [2^-96, inf) and NaN below 0 (a miss); a wave with a lane
            // meeting 0 <= |det| < 2^-96 redoes the leaf with sphere_hit.
            float dq[BVH_LEAF_MAX];
            bool bad = false;
#pragma unroll
            for (int q = 0; q < BVH_LEAF_MAX; q++) {
                const float opx = g[q].x - r.o.x, opy = g[q].y - r.o.y, opz = g[q].z - r.o.z;
                const float bb = opx * r.d.x + opy * r.d.y + opz * r.d.z;
                const float det = bb * bb - (opx * opx + opy * opy + opz * opz) + g[q].w;
                bad = bad || (q < c && fabsf(det) < 0x1p-96f);
                const float sd = sqrt_nr(det);
                const float t1 = bb - sd, t2 = bb + sd;
                dq[q] = t1 > EPS ? t1 : (t2 > EPS ? t2 : MISS);
            }
            if (wave_any(bad)) {
#pragma unroll
                for (int q = 0; q < BVH_LEAF_MAX; q++) dq[q] = sphere_hit(g[q], r);
            }
            // The spheres' reference indices are not loaded with the leaf
            // (four VGPRs less across the walk): the leaf's new best is kept
            // as its hierarchy position and its index loaded once, after the
            // tests; only ties (and the counted any-hit's highest occluder)
            // load an index on the spot.
            int bpos = -1;
#pragma unroll
            for (int q = 0; q < BVH_LEAF_MAX; q++) {
                if (q < c) {
                    const float d = dq[q];
                    if (shadow) {
                        if (d < maxt) {
                            if (COUNT) {
                                const int i = B.id[f + q];
                                if (i > id) id = i;
                            } else {
                                bpos = f + q;
                            }
                        }
                    } else if (d < t) {
                        t = d;
                        bpos = f + q;
                    } else if (d == t) {
                        const int cur = bpos >= 0 ? B.id[bpos] : id;
                        if (B.id[f + q] > cur) bpos = f + q;
                    }
                }
            }
            if (bpos >= 0) id = B.id[bpos];
            if (!COUNT && shadow && id >= 0) {
                node = B.nnodes;
                pend2 = 0;
            }
            pend = pend2;
            pend2 = 0;
        }
#ifdef RT_SPT_TRACE
        W.tr_leaf += (unsigned)(__builtin_amdgcn_s_memtime() - tr_l0);
#endif
        if (trips >= RT_BVH_BUDGET) break;
    }
#ifdef RT_SPT_TRACE
    W.tr_trips += trips;
#endif
    W.t = t;
    W.id = id;
    W.node = node;
    W.pend = pend;
    W.pend2 = pend2;
    return node >= B.nnodes && pend == 0;
}

// ---------------------------------------------------------------------------
// 8-wide hierarchy in LDS (GEO_WIDE; spt_bvh.h WideBuild).  The binary tree
// above collapsed to 8 children per node with the child boxes quantised to 8
// bits per plane (rounded outward on the host): configs[4]'s 10k spheres,
// leaves of <= 8, make 528 nodes = 59 KB, which every block stages in LDS.
// A query visits ~7 wide nodes instead of ~15 binary ones, and each visit is
// an LDS read instead of a dependent L2 access: the binary walk's trip cost
// ~1,300 cycles even with its wave alone on the chip (tools/c5_phase.py), its
// latency, not contention, set configs[4]'s critical path.
//
// Culling is the binary walk's rule with the margin taken over the node: a
// child box is skipped when the ray misses it grown by m = alpha * (|o - p| +
// D0) + K, where |o - p| + D0 >= |o - C| for every child centre C and K is the
// largest child's ALPHA_R * R + BETA -- m is at least each child's own binary
// margin.  The slab test in the node's quantisation frame rounds within
// ~2^-22 (|o - p| + D0) of the exact box planes, far inside alpha's factor-2
// slack.  Visit order: the child in slot p ^ octant at position p (the host
// put each octant's front child in the slot of that octant); the per-lane
// stack holds (node << 8 | remaining mask) entries in LDS, one per level.
// idmin >= 0 (the counted any-hit): only children holding a reference index
// above idmin (hid: the node's eight highest-index words) are crossed.
__device__ __forceinline__ unsigned wide_visit(const uint4 *__restrict__ N, const ray3 &r, float ix, float iy,
                                               float iz, float alpha, int oct, float lim,
                                               const unsigned *__restrict__ hid = nullptr, int idmin = -1)
{
    const uint4 h0 = N[0];
    const float2 h1 = *(const float2 *)(N + 1);
    const float cx = __uint_as_float(h0.x) - r.o.x, cy = __uint_as_float(h0.y) - r.o.y,
                cz = __uint_as_float(h0.z) - r.o.z;
    const float dist = __builtin_amdgcn_sqrtf(__builtin_fmaf(cx, cx, __builtin_fmaf(cy, cy, cz * cz)));
    const float m = __builtin_fmaf(alpha, dist + h1.x, h1.y);
    const float ax = __uint_as_float((h0.w & 255u) << 23) * ix;
    const float ay = __uint_as_float(((h0.w >> 8) & 255u) << 23) * iy;
    const float az = __uint_as_float(((h0.w >> 16) & 255u) << 23) * iz;
    const float bx = cx * ix, by = cy * iy, bz = cz * iz;
    const float mx = m * fabsf(ix), my = m * fabsf(iy), mz = m * fabsf(iz);
    const float bnx = bx - mx, bfx = bx + mx, bny = by - my, bfy = by + my, bnz = bz - mz, bfz = bz + mz;
    unsigned valid = h0.w >> 24;
    if (hid && idmin >= 0) {
#pragma unroll
        for (int sl = 0; sl < 8; sl++) valid &= ((int)hid[sl] > idmin ? 1u : 0u) << sl | ~(1u << sl);
    }
    // The child boxes, a half (four slots) at a time: words 16 + 6 h ..
    // 21 + 6 h hold lo_x, lo_y, lo_z, hi_x, hi_y, hi_z of slots 4h .. 4h+3.
    // The near plane of an axis is the low byte for a positive direction.
    const unsigned *W = (const unsigned *)N;
    unsigned hm = 0;
#pragma unroll
    for (int hf = 0; hf < 2; hf++) {
        const unsigned *q = W + 16 + 6 * hf;
        const unsigned lx = q[0], ly = q[1], lz = q[2], ux = q[3], uy = q[4], uz = q[5];
        const unsigned nxw = (oct & 1) ? ux : lx, fxw = (oct & 1) ? lx : ux;
        const unsigned nyw = (oct & 2) ? uy : ly, fyw = (oct & 2) ? ly : uy;
        const unsigned nzw = (oct & 4) ? uz : lz, fzw = (oct & 4) ? lz : uz;
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const int sh = 8 * j, sl = 4 * hf + j;
            const float tnx = __builtin_fmaf((float)((nxw >> sh) & 255u), ax, bnx);
            const float tfx = __builtin_fmaf((float)((fxw >> sh) & 255u), ax, bfx);
            const float tny = __builtin_fmaf((float)((nyw >> sh) & 255u), ay, bny);
            const float tfy = __builtin_fmaf((float)((fyw >> sh) & 255u), ay, bfy);
            const float tnz = __builtin_fmaf((float)((nzw >> sh) & 255u), az, bnz);
            const float tfz = __builtin_fmaf((float)((fzw >> sh) & 255u), az, bfz);
            const float tn = fmaxf(fmaxf(tnx, tny), fmaxf(tnz, 0.f));
            const float tf = fminf(fminf(tfx, tfy), fminf(tfz, lim));
            hm |= ((tn <= tf && ((valid >> sl) & 1u)) ? 1u : 0u) << (sl ^ oct);
        }
    }
    return hm;
}

#ifndef RT_SPT_COOP_NL
#define RT_SPT_COOP_NL 2    // cooperative walk: leaves tested per pass (loads in flight together)
#endif
// (wide_walk's trip budget per call (16), leaf batch threshold (16/64) and
// early stop (end the call once <= 32/64 of its lanes still walk: configs[4]
// 36.3 -> 29.0 ms) come from the host, SptTune.)
constexpr int WIDE_WORDS = 28;   // per node (spt_bvh.h)

template <bool COUNT>
__device__ __forceinline__ void wide_begin(const BvhView &B, const ray3 &r, bool shadow, float t, BvhWalk &W)
{
    bvh_begin<COUNT>(B, r, shadow, t, W);
    W.node = -1;                                        // the root is visited by the first trip
    W.bpos = -1;
    W.m = (!COUNT && shadow && W.id >= 0) ? 0u : 1u;
    W.sp = 0;
}

// Advances the wave's wide walks by up to `budget` trips; returns true
// for a lane whose query is complete (results as bvh_walk).  L: the block's
// LDS copy of the nodes; stk: this wave's LDS stack (entry k of lane l at
// stk[64 k + l]).  Crossed leaves are postponed and tested together as in
// bvh_walk (two pending per lane); a leaf of more than four spheres is tested
// four at a time.
// opts: trip budget per call (bits 8..15), leaf batch threshold in 1/64 of
// the walking lanes (16..23), early stop (24..31): the call ends once at most
// stop/64 of the lanes that entered it are still walking (64: never).
template <bool COUNT>
__device__ bool wide_walk(const BvhView &B, const uint4 *__restrict__ L, unsigned *__restrict__ stk, const ray3 &r,
                          bool shadow, BvhWalk &W, int opts)
{
    const int budget = (opts >> 8) & 255, batch = (opts >> 16) & 255, stop = (opts >> 24) & 255;
    const float maxt = W.t;
    float t = W.t;
    // The best leaf hit so far is kept as its hierarchy position (bpos) and
    // its reference index loaded once, when the query completes -- not after
    // every leaf pass (a dependent global load: ~1/3 of a lone wave's leaf
    // pass, tools/c5_phase.py).  Ties and the counted any-hit's highest
    // occluder still load indices on the spot.
    int id = W.id, cur = W.node, pend = W.pend, pend2 = W.pend2, sp = W.sp, bpos = W.bpos;
    unsigned m = W.m;
    const float dx = fabsf(r.d.x) < 1e-30f ? copysignf(1e-30f, r.d.x) : r.d.x;
    const float dy = fabsf(r.d.y) < 1e-30f ? copysignf(1e-30f, r.d.y) : r.d.y;
    const float dz = fabsf(r.d.z) < 1e-30f ? copysignf(1e-30f, r.d.z) : r.d.z;
    const float ix = __builtin_amdgcn_rcpf(dx), iy = __builtin_amdgcn_rcpf(dy), iz = __builtin_amdgcn_rcpf(dz);
    const float e = fabsf(r.d.x * r.d.x + r.d.y * r.d.y + r.d.z * r.d.z - 1.f);
    const float alpha = e < 0x1p-16f ? BVH_K * (1.04e-3f + __builtin_amdgcn_sqrtf(e + 0x1p-22f)) : 1e30f;
    const int oct = (dx < 0.f ? 1 : 0) | (dy < 0.f ? 2 : 0) | (dz < 0.f ? 4 : 0);
    const unsigned *Lw = (const unsigned *)L;
    const unsigned *Lmax = COUNT ? (const unsigned *)(L + 7 * B.wnodes) : nullptr;   // (counted kernels)
    unsigned *my = stk + (threadIdx.x & 63);
    const int n0 = __builtin_popcountll(__builtin_amdgcn_ballot_w64(true));   // lanes in this call
    int trips = 0;
    WALK_PROF(W, 0);
    while (true) {
        if (m != 0 && pend2 == 0) {
            WALK_PROF(W, 1);
            int cw;
            if (cur < 0) {
                cw = 0;                                  // the root
                m = 0;
            } else {
                const int p = __builtin_ctz(m);
                m &= m - 1;
                cw = (int)Lw[cur * WIDE_WORDS + 8 + (p ^ oct)];
            }
            if (cw < 0) {
                if (pend == 0) pend = ~cw;
                else pend2 = ~cw;
            } else {
                const unsigned hm =
                    COUNT ? wide_visit(L + 7 * cw, r, ix, iy, iz, alpha, oct, shadow ? maxt : t,
                                       Lmax + 8 * cw, shadow ? id : -1)
                          : wide_visit(L + 7 * cw, r, ix, iy, iz, alpha, oct, shadow ? maxt : t);
                if (hm) {
                    if (m) {
                        my[64 * sp] = ((unsigned)cur << 8) | m;
                        sp++;
                    }
                    cur = cw;
                    m = hm;
                }
            }
            if (m == 0 && sp > 0) {
                sp--;
                const unsigned e2 = my[64 * sp];
                cur = (int)(e2 >> 8);
                m = e2 & 255u;
            }
        }
        trips++;
        const unsigned long long pm = __builtin_amdgcn_ballot_w64(pend != 0);
        const unsigned long long sm = __builtin_amdgcn_ballot_w64(m != 0 && pend2 == 0);
        const bool out = trips >= budget || 64 * __builtin_popcountll(pm | sm) <= stop * n0;
        if (pm == 0) {
            if (sm == 0 || out) break;
            continue;
        }
        if (sm != 0 && !out && 64 * __builtin_popcountll(pm & ~sm) < batch * __builtin_popcountll(pm | sm))
            continue;
#ifdef RT_SPT_TRACE
        const unsigned long long tr_l0 = __builtin_amdgcn_s_memtime();
        W.tr_leafruns++;
#endif
        if (pend != 0) {
            WALK_PROF(W, 2);
            const int f = pend & 0xffffff, c = pend >> 24, c4 = c < BVH_LEAF_MAX ? c : BVH_LEAF_MAX;
            float4 g[BVH_LEAF_MAX];
#pragma unroll
            for (int q = 0; q < BVH_LEAF_MAX; q++)        // all loads first: one latency per leaf
                g[q] = B.geo[f + (q < c4 ? q : 0)];
            float dq[BVH_LEAF_MAX];
            bool bad = false;
#pragma unroll
            for (int q = 0; q < BVH_LEAF_MAX; q++) {
                const float opx = g[q].x - r.o.x, opy = g[q].y - r.o.y, opz = g[q].z - r.o.z;
                const float bb = opx * r.d.x + opy * r.d.y + opz * r.d.z;
                const float det = bb * bb - (opx * opx + opy * opy + opz * opz) + g[q].w;
                bad = bad || (q < c4 && fabsf(det) < 0x1p-96f);
                const float sd = sqrt_nr(det);
                const float t1 = bb - sd, t2 = bb + sd;
                dq[q] = t1 > EPS ? t1 : (t2 > EPS ? t2 : MISS);
            }
            if (wave_any(bad)) {
#pragma unroll
                for (int q = 0; q < BVH_LEAF_MAX; q++) dq[q] = sphere_hit(g[q], r);
            }
#pragma unroll
            for (int q = 0; q < BVH_LEAF_MAX; q++) {
                if (q < c4) {
                    const float d = dq[q];
                    if (shadow) {
                        if (d < maxt) {
                            if (COUNT) {
                                const int i = B.id[f + q];
                                if (i > id) id = i;
                            } else {
                                bpos = f + q;
                            }
                        }
                    } else if (d < t) {
                        t = d;
                        bpos = f + q;
                    } else if (d == t) {
                        const int cur_id = bpos >= 0 ? B.id[bpos] : id;
                        if (B.id[f + q] > cur_id) bpos = f + q;
                    }
                }
            }
            if (c > BVH_LEAF_MAX) {
                pend = (f + BVH_LEAF_MAX) | ((c - BVH_LEAF_MAX) << 24);
            } else {
                pend = pend2;
                pend2 = 0;
            }
            if (!COUNT && shadow && (id >= 0 || bpos >= 0)) {
                m = 0;
                sp = 0;
                pend = pend2 = 0;
            }
        }
#ifdef RT_SPT_TRACE
        W.tr_leaf += (unsigned)(__builtin_amdgcn_s_memtime() - tr_l0);
#endif
        if (out) break;
    }
#ifdef RT_SPT_TRACE
    W.tr_trips += trips;
#endif
    const bool done = m == 0 && pend == 0;
    // (an uncounted any-hit only needs "some occluder": no index load)
    if (done && bpos >= 0) id = (!COUNT && shadow) ? 0x7fffffff : B.id[bpos];
    W.t = t;
    W.id = id;
    W.bpos = bpos;
    W.node = cur;
    W.m = m;
    W.sp = sp;
    W.pend = pend;
    W.pend2 = pend2;
    return done;
}

// ---------------------------------------------------------------------------
// Cooperative 8-wide walk: EIGHT lanes per ray (the heaviest tiles).
//
// A heavy tile's critical path is one pixel's 64-sample RNG chain of ~900
// loop iterations, each ~24 dependent walk trips; a lone wave issues one VALU
// instruction per ~4 cycles, and a per-lane trip (eight child slab tests, the
// stack, the pending-leaf bookkeeping) costs it ~250 of them.  Here the eight
// lanes of a lane group (lanes 8g .. 8g+7) hold the same pixel -- the same
// ray, RNG words and path state, computed redundantly and identically -- and
// split each trip: lane k tests child slot k ^ oct of the node (its bit of the
// visit mask, gathered with one ballot), or sphere k of a leaf (the group's
// nearest / any hit by a 3-step DPP reduction).  A trip is ~40 VALU
// instructions instead of ~250, a leaf is one pass instead of up to four, and
// the wave walks the maximum over 8 rays instead of 64.  Group-uniform state
// (node, mask, stack, t, bpos, id) is held identically by the 8 lanes; each
// lane keeps its own copy of the stack column, as in wide_walk.  Results are
// the reference's: every sphere a per-lane walk would test is tested with
// the same float formula, and the nearest hit is the minimum distance with
// the highest reference index on ties, an order-independent choice.
// G = 4 (COOP4): four lanes per pixel, two child slots / spheres per lane --
// half the waves per heavy tile for a somewhat longer trip.
// Minimum over the group of non-negative floats (leaf distances: > EPS or
// +inf), compared as integers: the same order, and no NaN canonicalisation.
template <int G>
__device__ __forceinline__ float grp_min(float v)
{
    // (the identity as the DPP's old value lets the compiler fold each move
    // into its v_min_i32)
    constexpr int ID = 0x7fffffff;
    int i = __float_as_int(v);
    i = min(i, __builtin_amdgcn_update_dpp(ID, i, 0xB1, 0xF, 0xF, false));
    if (G >= 4) i = min(i, __builtin_amdgcn_update_dpp(ID, i, 0x4E, 0xF, 0xF, false));
    if (G == 8) i = min(i, __builtin_amdgcn_update_dpp(ID, i, 0x141, 0xF, 0xF, false));
    return __int_as_float(i);
}
template <int G>
__device__ __forceinline__ int grp_max(int v)
{
    constexpr int ID = (int)0x80000000;
    v = max(v, __builtin_amdgcn_update_dpp(ID, v, 0xB1, 0xF, 0xF, false));
    if (G >= 4) v = max(v, __builtin_amdgcn_update_dpp(ID, v, 0x4E, 0xF, 0xF, false));
    if (G == 8) v = max(v, __builtin_amdgcn_update_dpp(ID, v, 0x141, 0xF, 0xF, false));
    return v;
}
// The group's G bits of a predicate (bit k = lane gbase + k).
template <int G>
__device__ __forceinline__ unsigned grp_bits(bool p, int gbase)
{
    return (unsigned)(__builtin_amdgcn_ballot_w64(p) >> gbase) & ((1u << G) - 1u);
}

// wide_visit split over the group: lane k tests the child at visit
// positions k, k + G, ... (slot position ^ oct) and the group's visit mask
// comes back from ballots.  The float operations are wide_visit's, so the
// culling decisions are its own.
template <int G>
__device__ __forceinline__ unsigned wide_visit_coop(const uint4 *__restrict__ N, const ray3 &r, float ix, float iy,
                                                    float iz, float alpha, int oct, float lim, int pos, int gbase,
                                                    unsigned &lm, const unsigned *__restrict__ hid = nullptr,
                                                    int idmin = -1)
{
    const uint4 h0 = N[0];
    const float2 h1 = *(const float2 *)(N + 1);
    uint2 w[8 / G][3];
    int cwk[8 / G];                       // this lane's children's words (< 0: a leaf)
#pragma unroll
    for (int j = 0; j < 8 / G; j++) cwk[j] = (int)((const unsigned *)N)[8 + ((pos + j * G) ^ oct)];
#pragma unroll
    for (int j = 0; j < 8 / G; j++) {
        const unsigned *q = (const unsigned *)N + 16 + 6 * (((pos + j * G) ^ oct) >> 2);
        w[j][0] = *(const uint2 *)q;
        w[j][1] = *(const uint2 *)(q + 2);
        w[j][2] = *(const uint2 *)(q + 4);
    }
    const float cx = __uint_as_float(h0.x) - r.o.x, cy = __uint_as_float(h0.y) - r.o.y,
                cz = __uint_as_float(h0.z) - r.o.z;
    const float dist = __builtin_amdgcn_sqrtf(__builtin_fmaf(cx, cx, __builtin_fmaf(cy, cy, cz * cz)));
    const float m = __builtin_fmaf(alpha, dist + h1.x, h1.y);
    const float ax = __uint_as_float((h0.w & 255u) << 23) * ix;
    const float ay = __uint_as_float(((h0.w >> 8) & 255u) << 23) * iy;
    const float az = __uint_as_float(((h0.w >> 16) & 255u) << 23) * iz;
    const float bx = cx * ix, by = cy * iy, bz = cz * iz;
    const float mx = m * fabsf(ix), my = m * fabsf(iy), mz = m * fabsf(iz);
    const float bnx = bx - mx, bfx = bx + mx, bny = by - my, bfy = by + my, bnz = bz - mz, bfz = bz + mz;
    unsigned hm = 0;
    lm = 0;
#pragma unroll
    for (int j = 0; j < 8 / G; j++) {
        const int sl = (pos + j * G) ^ oct;
        const unsigned lx = w[j][0].x, ly = w[j][0].y, lz = w[j][1].x, ux = w[j][1].y, uy = w[j][2].x,
                       uz = w[j][2].y;
        const unsigned nxw = (oct & 1) ? ux : lx, fxw = (oct & 1) ? lx : ux;
        const unsigned nyw = (oct & 2) ? uy : ly, fyw = (oct & 2) ? ly : uy;
        const unsigned nzw = (oct & 4) ? uz : lz, fzw = (oct & 4) ? lz : uz;
        const int sh = 8 * (sl & 3);
        const float tnx = __builtin_fmaf((float)((nxw >> sh) & 255u), ax, bnx);
        const float tfx = __builtin_fmaf((float)((fxw >> sh) & 255u), ax, bfx);
        const float tny = __builtin_fmaf((float)((nyw >> sh) & 255u), ay, bny);
        const float tfy = __builtin_fmaf((float)((fyw >> sh) & 255u), ay, bfy);
        const float tnz = __builtin_fmaf((float)((nzw >> sh) & 255u), az, bnz);
        const float tfz = __builtin_fmaf((float)((fzw >> sh) & 255u), az, bfz);
        const float tn = fmaxf(fmaxf(tnx, tny), fmaxf(tnz, 0.f));
        const float tf = fminf(fminf(tfx, tfy), fminf(tfz, lim));
        bool hit = tn <= tf && ((h0.w >> (24 + sl)) & 1u);
        if (hid && idmin >= 0) hit = hit && (int)hid[sl] > idmin;
        hm |= grp_bits<G>(hit, gbase) << (j * G);
        lm |= grp_bits<G>(hit && cwk[j] < 0, gbase) << (j * G);
    }
    return hm;
}

// Applies one leaf pass's distances d[j] (sphere b + pos + j G of the leaf
// at f; MISS past its end) to the group's query.  Nearest hit: t / bpos
// updated to the minimum distance, highest reference index on ties (ids
// loaded only then).  Any hit: COUNT -- id = the highest occluder index so
// far; otherwise returns true (occluded: bpos = f) and the caller ends the walk.
template <bool COUNT, int G>
__device__ __forceinline__ bool leaf_apply(const BvhView &B, bool shadow, float maxt, int f, int b, int pos,
                                           int gbase, const float (&d)[8 / G], float &t, int &bpos, int &id)
{
    constexpr int S = 8 / G;
    if (shadow) {
        bool occ[S];
        unsigned any = 0;
#pragma unroll
        for (int j = 0; j < S; j++) {
            occ[j] = d[j] < maxt;
            any |= grp_bits<G>(occ[j], gbase);
        }
        if (COUNT) {
            if (any) {
                int i = -1;
#pragma unroll
                for (int j = 0; j < S; j++)
                    if (occ[j]) i = max(i, B.id[f + b + pos + j * G]);
                i = grp_max<G>(i);
                if (i > id) id = i;
            }
        } else if (any) {
            bpos = f;
            return true;
        }
        return false;
    }
    float dl = d[0];
#pragma unroll
    for (int j = 1; j < S; j++) dl = fminf(dl, d[j]);
    const float dm = grp_min<G>(dl);
    if (dm <= t) {                              // (dm finite: t < +inf)
        unsigned cm[S];
        int nc = 0;
#pragma unroll
        for (int j = 0; j < S; j++) {
            cm[j] = grp_bits<G>(d[j] == dm, gbase);
            nc += __builtin_popcount(cm[j]);
        }
        if (dm < t && nc == 1) {
            int k = 0;
#pragma unroll
            for (int j = 0; j < S; j++)
                if (cm[j]) k = j * G + __builtin_ctz(cm[j]);
            t = dm;
            bpos = f + b + k;
        } else {                                // a tie: within the leaf, or with the best so far
            int il[S], i = -1;
#pragma unroll
            for (int j = 0; j < S; j++) {
                il[j] = d[j] == dm ? B.id[f + b + pos + j * G] : -1;
                i = max(i, il[j]);
            }
            const int im = grp_max<G>(i);
            const int cur_id = dm == t ? (bpos >= 0 ? B.id[bpos] : id) : -1;
            if (im > cur_id) {
                int k = 0;
#pragma unroll
                for (int j = 0; j < S; j++) {
                    const unsigned wm = grp_bits<G>(il[j] == im, gbase);
                    if (wm) k = j * G + __builtin_ctz(wm);
                }
                t = dm;
                bpos = f + b + k;
            }
        }
    }
    return false;
}

// Up to NL leaves (first sphere f[l], c[l] spheres; c = 0: none) for the
// group, sphere b + k + j G of each on lane k: the sphere loads of all of
// them are issued before the first test (one memory latency per pass), the
// leaves then applied in order.  Returns true when an uncounted any-hit
// found an occluder.
// LOCAL (nearest hit): each lane keeps its own best (t, bpos) over the
// spheres it tests -- no group reduction per leaf; wide_walk_coop reduces the
// lanes' bests to the group's culling limit once per leaf section and to the
// result once per query (the minimum with ties to the highest index: the
// same choice, made once).
template <bool COUNT, int G, int NL, bool LOCAL = false>
__device__ __forceinline__ bool leaf_coop(const BvhView &B, const ray3 &r, bool shadow, float maxt,
                                          const int (&f)[NL], const int (&c)[NL], int pos, int gbase, float &t,
                                          int &bpos, int &id)
{
    constexpr int S = 8 / G;
    int cmax = c[0];
#pragma unroll
    for (int l = 1; l < NL; l++) cmax = max(cmax, c[l]);
    for (int b = 0; b < cmax; b += 8) {
        float4 g[NL][S];
#pragma unroll
        for (int l = 0; l < NL; l++)
#pragma unroll
            for (int j = 0; j < S; j++) {
                const int q = b + pos + j * G;
                g[l][j] = B.geo[f[l] + (q < c[l] ? q : 0)];
            }
#pragma unroll
        for (int l = 0; l < NL; l++) {
            if (b >= c[l]) continue;
            float d[S];
            bool bad = false;
#pragma unroll
            for (int j = 0; j < S; j++) {
                const float opx = g[l][j].x - r.o.x, opy = g[l][j].y - r.o.y, opz = g[l][j].z - r.o.z;
                const float bb = opx * r.d.x + opy * r.d.y + opz * r.d.z;
                const float det = bb * bb - (opx * opx + opy * opy + opz * opz) + g[l][j].w;
                bad = bad || (b + pos + j * G < c[l] && fabsf(det) < 0x1p-96f);
                const float sd = sqrt_nr(det);
                const float t1 = bb - sd, t2 = bb + sd;
                d[j] = t1 > EPS ? t1 : (t2 > EPS ? t2 : MISS);
            }
            if (wave_any(bad)) {
#pragma unroll
                for (int j = 0; j < S; j++) d[j] = sphere_hit(g[l][j], r);
            }
#pragma unroll
            for (int j = 0; j < S; j++)
                if (b + pos + j * G >= c[l]) d[j] = MISS;
            if (LOCAL && !shadow) {
#pragma unroll
                for (int j = 0; j < S; j++) {
                    const int q = f[l] + b + pos + j * G;
                    if (d[j] < t) {
                        t = d[j];
                        bpos = q;
                    } else if (d[j] == t) {             // (d finite: a tie)
                        const int cur_id = bpos >= 0 ? B.id[bpos] : id;
                        if (B.id[q] > cur_id) bpos = q;
                    }
                }
            } else if (leaf_apply<COUNT, G>(B, shadow, maxt, f[l], b, pos, gbase, d, t, bpos, id)) {
                return true;
            }
        }
    }
    return false;
}

// The crossed leaves l1 of node n1 and l2 of node n2, RT_SPT_COOP_NL per
// pass; true when an uncounted any-hit found an occluder.
template <bool COUNT, int G, bool LOC>
__device__ __forceinline__ bool coop_leaves(const BvhView &B, const ray3 &r, bool shadow, float maxt,
                                            const unsigned *Lw, int oct, int n1, unsigned l1, int n2, unsigned l2,
                                            int pos, int gbase, float &t, int &bpos, int &id)
{
    constexpr int NL = G == 2 ? 1 : RT_SPT_COOP_NL;   // (two lanes: four spheres a lane per leaf already)
    while (l1 | l2) {
        int fa[NL], ca[NL];
#pragma unroll
        for (int q = 0; q < NL; q++) {
            fa[q] = ca[q] = 0;
            if (l1 | l2) {
                const bool first = l1 != 0;
                const unsigned lq = first ? l1 : l2;
                const int iq = __builtin_ctz(lq);
                l1 = first ? (l1 & (l1 - 1u)) : l1;
                l2 = first ? l2 : (l2 & (l2 - 1u));
                const int wq = ~(int)Lw[(first ? n1 : n2) * WIDE_WORDS + 8 + (iq ^ oct)];
                fa[q] = wq & 0xffffff;
                ca[q] = wq >> 24;
            }
        }
        if (leaf_coop<COUNT, G, NL, LOC>(B, r, shadow, maxt, fa, ca, pos, gbase, t, bpos, id))
            return true;
    }
    return false;
}

template <bool COUNT, int G>
__device__ bool wide_walk_coop(const BvhView &B, const uint4 *__restrict__ L, unsigned *__restrict__ stk,
                               const ray3 &r, bool shadow, BvhWalk &W, int opts)
{
    const int budget = (opts >> 8) & 255, stop = (opts >> 24) & 255;
    const float maxt = W.t;
    float t = W.t;
    int id = W.id, cur = W.node, sp = W.sp, bpos = W.bpos;
    unsigned m = W.m;
    const float dx = fabsf(r.d.x) < 1e-30f ? copysignf(1e-30f, r.d.x) : r.d.x;
    const float dy = fabsf(r.d.y) < 1e-30f ? copysignf(1e-30f, r.d.y) : r.d.y;
    const float dz = fabsf(r.d.z) < 1e-30f ? copysignf(1e-30f, r.d.z) : r.d.z;
    const float ix = __builtin_amdgcn_rcpf(dx), iy = __builtin_amdgcn_rcpf(dy), iz = __builtin_amdgcn_rcpf(dz);
    const float e = fabsf(r.d.x * r.d.x + r.d.y * r.d.y + r.d.z * r.d.z - 1.f);
    const float alpha = e < 0x1p-16f ? BVH_K * (1.04e-3f + __builtin_amdgcn_sqrtf(e + 0x1p-22f)) : 1e30f;
    const int oct = (dx < 0.f ? 1 : 0) | (dy < 0.f ? 2 : 0) | (dz < 0.f ? 4 : 0);
    const unsigned *Lw = (const unsigned *)L;
    const unsigned *Lmax = COUNT ? (const unsigned *)(L + 7 * B.wnodes) : nullptr;
    unsigned *my = stk + (threadIdx.x & 63);
    const int pos = threadIdx.x & (G - 1), gbase = threadIdx.x & (64 - G);
    const int n0 = __builtin_popcountll(__builtin_amdgcn_ballot_w64(true));
    int trips = 0;
    // One trip as straight-line selects: the next child's word and the
    // stack top are read together at the trip's start (the pop can only
    // need the entry below the current top: a trip that descends does not
    // pop), every group's lanes run the visit (a group with nothing to visit
    // masks its result), and only the leaf passes sit behind a wave-uniform
    // branch.  The old form's per-group branches cost the lone heavy wave
    // ~40 exec-mask and branch instructions per trip (c4_coop_phase_n8_spread.log).
    // (G = 8, nearest hits: t / bpos are the lane's own best -- reduced to
    // the group's culling limit tg once per leaf section and to the result
    // once per query instead of per leaf: N = 8 / 4 shares -2 to -3 %)
    constexpr bool LOC = G == 8;
    float tg = LOC ? grp_min<G>(t) : t;
    unsigned pl = 0u;                           // the previous trip's crossed leaves (of node pn), pending
    int pn = 0;
    while (true) {
        const bool has = m != 0;
        const int p = __builtin_ctz(m | 256u);
        const unsigned mr = cur < 0 ? 0u : (m & (m - 1u));
        const int cwl = (int)Lw[max(cur, 0) * WIDE_WORDS + 8 + ((p & 7) ^ oct)];
        const unsigned e2 = my[64 * max(sp - 1, 0)];
        const int cw = cur < 0 ? 0 : cwl;
        bool occl = false;
        const bool rootleaf = has && cw < 0;    // (a root leaf: child leaves are tested at their parent)
        if (wave_any(rootleaf)) {
            if (rootleaf) {
                const int lf = ~cw;
                const int fa[1] = {lf & 0xffffff}, ca[1] = {lf >> 24};
                occl = leaf_coop<COUNT, G, 1, LOC>(B, r, shadow, maxt, fa, ca, pos, gbase, t, bpos, id);
            }
            if (LOC) tg = grp_min<G>(t);
        }
        const bool vis = has && cw >= 0;
        const int cv = vis ? cw : 0;
        unsigned lm;
        unsigned hm = COUNT ? wide_visit_coop<G>(L + 7 * cv, r, ix, iy, iz, alpha, oct, shadow ? maxt : (LOC ? tg : t), pos, gbase,
                                                 lm, Lmax + 8 * cv, shadow ? id : -1)
                            : wide_visit_coop<G>(L + 7 * cv, r, ix, iy, iz, alpha, oct, shadow ? maxt : (LOC ? tg : t), pos, gbase,
                                                 lm);
        hm = vis ? hm : 0u;
        lm = vis ? lm : 0u;
        // A trip's crossed leaves wait one trip, so one leaf section serves
        // two trips' leaves of every group: the lone heavy wave of an N = 8
        // share runs half as many leaf sections (~50 % of its chain).  Exact:
        // the nearest hit is order-independent; the culling limit tg lags
        // one trip.  N = 8 shares 9.8-10.1 -> 9.3-9.65 ms, N = 4 13.6-14.2
        // -> 13.0-13.5 ms (profiles/r06/c4_coop_defer_ab.log).
        bool run = wave_any(pl != 0);
        if (!run && wave_any(lm != 0)) {
            pl = lm;
            pn = cv;
        } else if (run) {
#ifdef RT_SPT_TRACE
            const unsigned long long tr_l0 = __builtin_amdgcn_s_memtime();
            W.tr_leafruns++;
#endif
            occl = coop_leaves<COUNT, G, LOC>(B, r, shadow, maxt, Lw, oct, pn, pl, cv, lm, pos, gbase, t, bpos, id) || occl;
            pl = 0u;
            if (LOC) tg = grp_min<G>(t);
#ifdef RT_SPT_TRACE
            W.tr_leaf += (unsigned)(__builtin_amdgcn_s_memtime() - tr_l0);
#endif
        }
        const unsigned nm = hm & ~lm;
        const bool desc = vis && nm != 0 && !occl;
        if (desc && mr != 0) my[64 * sp] = ((unsigned)cur << 8) | mr;
        sp = occl ? 0 : sp + ((desc && mr != 0) ? 1 : 0);
        cur = desc ? cw : cur;
        m = occl ? 0u : (desc ? nm : mr);
        const bool pop = m == 0 && sp > 0;      // (then no push this trip: e2 is the top)
        sp -= pop ? 1 : 0;
        cur = pop ? (int)(e2 >> 8) : cur;
        m = pop ? (e2 & 255u) : m;
        trips++;
        const unsigned long long am = __builtin_amdgcn_ballot_w64(m != 0);
        if (am == 0 || trips >= budget || 64 * __builtin_popcountll(am) <= stop * n0) {
            if (wave_any(pl != 0)) {                    // (no leaf is left pending past the call)
                if (coop_leaves<COUNT, G, LOC>(B, r, shadow, maxt, Lw, oct, pn, pl, 0, 0u, pos, gbase, t, bpos, id)) {
                    m = 0u;
                    sp = 0;
                }
            }
            break;
        }
    }
    if (LOC && m == 0 && !shadow) {
        // the group's result from its lanes' bests: the minimum distance,
        // ties to the highest reference index (bpos -1: the query's first id)
        const float tf = grp_min<G>(t);
        const bool cand = t == tf;
        int wb;
        if (__builtin_popcount(grp_bits<G>(cand, gbase)) <= 1) {
            wb = grp_max<G>(cand ? bpos : -1);
        } else {
            const int cid = cand ? (bpos >= 0 ? B.id[bpos] : id) : (int)0x80000000;
            const int im = grp_max<G>(cid);
            wb = grp_max<G>((cand && cid == im) ? bpos : -1);
        }
        t = tf;
        bpos = wb;
    }
#ifdef RT_SPT_TRACE
    W.tr_trips += trips;
#endif
    const bool done = m == 0;
    if (done && bpos >= 0) id = (!COUNT && shadow) ? 0x7fffffff : B.id[bpos];
    W.t = t;
    W.id = id;
    W.bpos = bpos;
    W.node = cur;
    W.m = m;
    W.sp = sp;
    return done;
}

// Per-lane work counters: calls and samples in 32 bits (a lane adds a few per
// sample; render_kernel flushes a lane's calls with an atomic before they
// could wrap), sphere tests in 64.  Four VGPRs fewer than four u64 words.
struct Counts { unsigned isect, isectp, samples; unsigned long long tests; };

// Tools-only block profile (build with -DRT_SPT_PROF; tools/ab.py PROF=1):
// per code block, the lanes that executed it and the wave-executions
// (iterations in which at least one lane of the wave did).  Never in the
// product build.
#ifdef RT_SPT_PROF
enum { PB_ITER, PB_SHADOW, PB_NEAREST, PB_DIFF, PB_SPEC, PB_REFR, PB_LIGHT, PB_BOUNCE, PB_DONE,
       PB_WCALL, PB_WSTEP, PB_WLEAF, PB_WSHADE, PB_N };
__device__ unsigned long long g_spt_prof[2 * PB_N];
#define SPT_PROF(b)                                                                        \
    do {                                                                                   \
        prof_l[b]++;                                                                       \
        if ((int)(threadIdx.x & 63) == __builtin_ctzll(__builtin_amdgcn_read_exec())) prof_w[b]++; \
    } while (0)
#else
#define SPT_PROF(b) do {} while (0)
#endif

// Tools-only wave timeline (build with -DRT_SPT_TRACE): per wave of the grid
// {start, end} (s_memrealtime, 100 MHz), HW_ID, XCC_ID and {sum, max} over
// its lanes of the loop iterations, at g_spt_trace[4 * (linear block * 4 +
// wave) + 0/1].  Never in the product build.
// Phase stamps (s_memtime, shader clock), hierarchy kernels: per wave, the
// max over its lanes of the cycles spent in the walk (bvh_begin + bvh_walk),
// of those in leaf blocks, walk trips, leaf-block passes and queries; at
// g_spt_trace[4 * wave + 2/3].  g_spt_only_group >= 0 renders only that tile
// group (the other waves exit at once): the group's waves run alone on the
// chip, which splits contention from latency.
#ifdef RT_SPT_TRACE
__device__ uint4 *g_spt_trace;
__device__ int g_spt_only_group = -1;
#endif

// toInt, vec.h:62 (clamp macro keeps -0.0; glibc powf via rt_glibc_math.h).
__device__ __forceinline__ int to_int(float x)
{
    const float c = (x < 0.f) ? 0.f : ((x > 1.f) ? 1.f : x);
    return (int)(rtm::powf(c, 1.f / 2.2f) * 255.f + .5f);
}

// Occupancy of the kernel variants (__launch_bounds__ minimum waves per
// SIMD; every bound measured against its neighbours):
//   full-scan one-query kernels: unbounded (1);
//   the uncounted two-query kernel (DUAL): 7 -- 85 -> 72 VGPRs, no VGPR
//     spills, occupancy 5 -> 7: Cornell 1080p 17.87 -> 17.3 ms;
//   binary-hierarchy (GEO_BVH) kernels: 6 -- 93 -> 80 VGPRs (2 spilled): the
//     latency-bound walk gains more from the sixth wave than the spills cost;
//   8-wide (GEO_WIDE) kernels: 4 -- 126 VGPRs unbounded; 5 or 6 spill;
//   counted hierarchy kernels (not timed): 4, room for the counters.
constexpr int SPT_MINWAVES = 1, SPT_DUAL_MINWAVES = 7, BVH_MINWAVES = 6, WIDE_MINWAVES = 4, BVH_MINWAVES_COUNT = 4;
constexpr int GEO_LDS = 0, GEO_GLOBAL = 1, GEO_BVH = 2, GEO_WIDE = 3;
constexpr int GS_BYTES = 6160;      // GEO_BVH group staging strip: 8 x 96 colour floats, 8 x 64 seed words, 8 x 32 pixels, count

// DUAL (path tracing, full-scan geometry, scenes with exactly one light): a
// DIFF vertex builds its light sample's shadow ray AND its bounce ray in the
// same iteration -- SampleLights' draws do not depend on the shadow test, so
// the bounce's draws follow them in the reference's order either way -- and
// the next iteration queries both (query2_bf) and applies the shadow result
// (rad += thr * Ld, geomfunc.h:229-230) before it shades the bounce's hit.
// One iteration per path vertex instead of two for a lit DIFF vertex.
// COUNT: all four counters (the sphere-test count needs IntersectP's early-
// exit position, so a counted shadow query finds the highest-index
// occluder).  RAYS (SPT_COUNT_RAYS): Intersect / IntersectP calls and samples
// only, with the uncounted queries (any occluder ends a shadow query).
// CG (8-wide kernels): lanes per pixel of the cooperative walk this kernel
// carries (8 or 4), or 0 -- no cooperative code (windows without a
// cooperative tier: the full frame, N = 2 shares).
template <bool DL, bool COUNT, int GEO, bool DUAL = false, bool RAYS = false, int CG = 0>
__global__ void __launch_bounds__(1024, GEO == 2 ? ((COUNT || RAYS) ? BVH_MINWAVES_COUNT : BVH_MINWAVES)
                                              : GEO == 3 ? ((COUNT || RAYS) ? BVH_MINWAVES_COUNT : WIDE_MINWAVES)
                                              : ((DUAL && !COUNT && !RAYS) ? SPT_DUAL_MINWAVES : SPT_MINWAVES))
render_kernel(const rt_sphere *__restrict__ spheres, int nspheres, rt_camera cam,
              float *__restrict__ colors, const uint32_t *seeds_in,
              uint32_t *seeds_out, uint32_t *__restrict__ pixels, int w, int h,
              int row_begin, int row_end, int tiles_x, int ntiles, int nslots, int gstride, int first_sample,
              int nsamples, int prio_sched, const int *__restrict__ group_order, unsigned *__restrict__ group_cost,
              const float4 *__restrict__ g_geo, const float4 *__restrict__ g_emi,
              const float4 *__restrict__ g_col, const float4 *__restrict__ g_lrec, int nlights,
              BvhView bvh, unsigned long long *__restrict__ counters, int *__restrict__ work, int split,
              int nheavy, int sflags)
{
    constexpr bool LDS = GEO == GEO_LDS;
    // GEO_WIDE: persistent waves -- each wave takes 8x8 tiles from a work
    // counter (in the adaptive order's slot sequence, heaviest groups first)
    // until the window is done, so a block's LDS copy of the hierarchy is
    // made once and a CU never idles behind one block's slowest wave.
    constexpr bool PERSIST = GEO == GEO_WIDE;
    // Dynamic LDS carve (16-B multiples): geo | emi | col (n each) | lrec (3 per light),
    // a copy of the scene's global SoA (spt_scene_create).
    extern __shared__ __attribute__((aligned(16))) char smem[];
    Scene S;
    if (LDS) {
        float4 *s = (float4 *)smem;
        const int nrec = 3 * nspheres + 3 * (nlights > 0 ? nlights : 1);   // a light-free scene: one zero record
        for (int i = threadIdx.x; i < nrec; i += blockDim.x) s[i] = g_geo[i];
        __syncthreads();
        S.geo = s; S.emi = s + nspheres; S.col = s + 2 * nspheres; S.lrec = s + 3 * nspheres;
    } else {
        S.geo = g_geo; S.emi = g_emi; S.col = g_col; S.lrec = g_lrec;
    }
    S.nlights = nlights;
    S.n = nspheres;
    const DynGeo geo{S.geo, S.n};
    // GEO_WIDE LDS carve: the wide nodes (7 x 16 B each), then per wave of the
    // block its lanes' stacks ((wdepth - 1) entries x 64 lanes x 4 B).
    const uint4 *wL = (const uint4 *)smem;
    unsigned *wstk = nullptr;
    if (GEO == GEO_WIDE) {
        uint4 *d = (uint4 *)smem;
        for (int i = threadIdx.x; i < 7 * bvh.wnodes; i += blockDim.x) d[i] = bvh.wnode[i];
        if (COUNT)
            for (int i = threadIdx.x; i < 2 * bvh.wnodes; i += blockDim.x) d[7 * bvh.wnodes + i] = bvh.wmax[i];
        wstk = (unsigned *)(smem + (size_t)(COUNT ? 144 : 112) * bvh.wnodes) +
               (size_t)(threadIdx.x >> 6) * 64 * (bvh.wdepth - 1);
        __syncthreads();
    }

    // 8x8 pixel tiles of the row window, one per wave, in groups of four
    // side by side (a 32x8 strip: whole 128-B lines of the seed, colour and
    // pixel rows, so no line is fetched by two XCDs); group j of block b is
    // j * gridDim.x + b, so the groups of a 16-wave block sample the whole
    // window (per-CU work evens out when one block fills a CU).
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    // group_order (optional): dispatch slot -> group, heaviest groups of the
    // previous launch first (host: adaptive schedule); results do not depend
    // on it.
    // Compiled into the hierarchy kernels only: in the full-scan kernels
    // (Cornell) the order/cost plumbing cost 1.4 % of the frame and 8 % of an
    // N = 8 band (measured A/B) although it is never used there.
    constexpr bool SCHED = GEO == GEO_BVH || GEO == GEO_WIDE;
    constexpr bool CALLS = COUNT || RAYS;           // the call / sample counters are kept
    Counts cnt = {0, 0, 0, 0};
#ifdef RT_SPT_PROF
    unsigned prof_l[PB_N] = {}, prof_w[PB_N] = {};
#endif
    // Work item: tile (item & 3) of dispatch slot item >> 2.  Static launches:
    // one item per wave, slot (wave >> 2) * gridDim.x + blockIdx.x.
    // Persistent launches fetch work indices f: the first nheavy items in
    // dispatch order (the heaviest, with a learnt order) as 2^hs sub-items of
    // 64 >> hs pixels each (lanes beyond them idle: a heavy tile's pixels run
    // on several SIMDs), f = (nheavy << hs) + ... the rest whole.
    // (split: hs in bits 0..1; the wide walk's options above them, wide_walk)
    const int hs = PERSIST ? (split & 3) : 0;
    // waves of a block that take tier-1 sub-items first (split bits 3..7; 0: 4 << hs)
    const int hw = ((split >> 3) & 31) ? ((split >> 3) & 31) : (4 << hs);
    const int nitems = 4 * nslots;
    // Three tiers, in dispatch order (heaviest first with a learnt order):
    // nheavy bits 0..15 = n1 tiles split into 2^hs sub-items each (the
    // cooperative walk with split bit 2), bits 16..31 = n2 tiles routed one
    // per SIMD, then the rest.
    const int n1 = PERSIST ? min(nheavy & 0xffff, nitems) : 0;
    const int n2 = PERSIST ? min((nheavy >> 16) & 0xffff, nitems - n1) : 0;
    const int nwork = (n1 << hs) + (nitems - n1);
    // Persistent fetch: waves 0..hw - 1 of a block take tier-1 sub-items
    // first (work[2]); waves 0..3 -- one per SIMD -- then take tier-2 tiles
    // (work[1]): a heavy tile's SIMD shares its issue slots with lighter,
    // lower-priority waves instead of with three other heavy tiles; every
    // wave then takes the rest in order (work[0]).
    // (by the wave's first active lane: refill claims fetch from inside the
    // pixel loop, where lanes that ran out of work have left)
    // (below: the first min(hw, waves per block) x #blocks tier-1 sub-items are assigned statically)
    const int nstatic = PERSIST ? min(min(hw, (int)(blockDim.x >> 6)) * (int)gridDim.x, n1 << hs) : 0;
    const auto fetch = [&]() {
        int v = 0;
        if (lane == __builtin_ctzll(__builtin_amdgcn_read_exec())) {
            v = -1;
            if (wave < hw && n1 > 0) {
                const int hv = atomicAdd(work + 2, 1) + nstatic;
                if (hv < (n1 << hs)) v = hv;
            }
            if (v < 0 && wave < 4 && n2 > 0) {
                const int hv = atomicAdd(work + 1, 1);
                if (hv < n2) v = (n1 << hs) + hv;
            }
            if (v < 0) v = (n1 << hs) + n2 + atomicAdd(work, 1);
        }
        return __builtin_amdgcn_readfirstlane(v);
    };
    int f = ((wave >> 2) * (int)gridDim.x + (int)blockIdx.x) * 4 + (wave & 3);
    if (PERSIST) {
        // The first tier-1 sub-item of wave w of block b is
        // w * #blocks + b, not the next one a shared counter hands out: the
        // heaviest tiles' sub-items (dispatch order) land one per CU, beside
        // lighter ones on their SIMD, where the counter gave a whole heavy
        // tile's rows to the waves of the first block to start.
        const int fs = wave * (int)gridDim.x + (int)blockIdx.x;
        f = (wave < hw && fs < (n1 << hs)) ? fs : __builtin_amdgcn_readfirstlane(fetch());
    }
    while (!PERSIST || f < nwork) {
    const bool heavy_ = f < (n1 << hs);
    // Tier-1 (heavy) items are cooperative (the host sends them only to a
    // kernel carrying the walk, CG != 0, with hs = log2(CG)): hs = 3 (G = 8):
    // a heavy tile's 8 sub-items are 8 rows of 8 pixels with eight lanes per
    // pixel (lane group g = pixel g of the row), walking the hierarchy
    // cooperatively (wide_walk_coop); hs = 2 (G = 4): 4 sub-items of 16
    // pixels, four lanes per pixel.
    const bool coop = GEO == GEO_WIDE && CG != 0 && heavy_;
    const int cg = coop ? CG : 0;
    const int item = heavy_ ? f >> hs : f - (n1 << hs) + n1;
    const int sub = heavy_ ? f & ((1 << hs) - 1) : 0;
    const int slot = item >> 2;
    // group_order: the learnt order (hierarchy kernels) or the caller's
    // group list (spt_scene_render_list_async, every kernel) of nslots
    // entries; a slot past it or an entry outside the frame renders nothing.
    const int grp = group_order ? (slot < nslots ? group_order[slot] : -1) : slot;
    const bool gvalid = (unsigned)grp < (unsigned)((ntiles + 3) >> 2);
    const int tile = grp * 4 + (item & 3);
    const int li = coop ? (sub << (6 - hs)) + (lane >> hs) : lane;   // pixel of the 8x8 tile
    const bool lead = !coop || (lane & (cg - 1)) == 0;  // the lane that stores the pixel and counts
    unsigned long long t_start = 0;
    if (SCHED) t_start = __builtin_amdgcn_s_memrealtime();
    // GSTORE (hierarchy kernels): per group of the block a 32x8 staging
    // strip in LDS -- colours, seeds, pixels -- and an arrival count.
    // (Addresses recomputed where used: held across the loop they spilled.)
    constexpr bool GSTORE = GEO == GEO_BVH;
#define GS_BASE() (smem + (size_t)((threadIdx.x >> 6) >> 2) * GS_BYTES)
    if (GSTORE) {
        if ((threadIdx.x & 255) == 0) *(int *)(GS_BASE() + 6144) = 0;
        __syncthreads();
    }
    int x = (tile % tiles_x) * 8 + (li & 7);
    // gstride > 1: the window is every gstride-th 8-row group from row_begin
    // (spt_scene_render_groups_async, multi-GPU load balance).
    int y = row_begin + (tile / tiles_x) * 8 * gstride + (li >> 3);
    // Refill (full-counter 8-wide kernels, items past the cooperative
    // tier): the wave starts on this item's 64 pixels, and from then on a
    // lane whose pixel has taken all its samples stores it and takes the next
    // pixel of the dispatch sequence (the rest of the wave's current item,
    // then further items), until the window's work is gone.  A tile of
    // configs[4] mixes pixels whose sample chains differ several-fold (sky
    // beside the fractal): waiting for the tile's slowest pixel left 28 % of
    // the lanes idle (tools/c4_lanes.py).  Every pixel's computation is
    // unchanged -- only which lane runs it, and when.
    // Counted kernels only: there the tile tail, not the levelling,
    // dominates -- 28 of 64 lanes per iteration without refill, 52 with,
    // profiles/r05/c4_counted_refill.log; on the uncounted frame refill
    // measured +7 % (its waves lose the levelled priority).
    const bool refill = COUNT && PERSIST && !heavy_;
#ifdef RT_SPT_TRACE
    bool active = gvalid && tile < ntiles && x < w && y < row_end &&
                  (g_spt_only_group < 0 || grp == g_spt_only_group);
    unsigned tr_walk = 0, tr_leaf = 0, tr_trips = 0, tr_leafruns = 0, tr_queries = 0;
    const unsigned long long tr_c0 = __builtin_amdgcn_s_memtime();
    const unsigned long long tr_t0 = __builtin_amdgcn_s_memrealtime();
#else
    bool active = gvalid && tile < ntiles && x < w && y < row_end;
#endif

#ifdef RT_SPT_TRACE
    unsigned tr_iters = 0;
#endif
    if (active || refill) {
        int i = (h - y - 1) * w + x;                            // smallptCPU.cpp:86
        uint32_t s0 = 0, s1 = 0;
        v3 col = mk(0.f, 0.f, 0.f);
        if (active) {
            s0 = seeds_in[2 * (size_t)i];
            s1 = seeds_in[2 * (size_t)i + 1];
            if (first_sample > 0)
                col = mk(colors[3 * (size_t)i], colors[3 * (size_t)i + 1], colors[3 * (size_t)i + 2]);
        }
        const float invW = 1.f / w, invH = 1.f / h;             // :80-81
        // Refill state: the lane's pixel is px_ok (its group pgrp, started at
        // pix_t0), exhausted once the window has no pixel left for it; the
        // wave's dispatch cursor is item rf_f, pixel rf_p (wave-uniform: only
        // updated at the loop top, where every lane still looping is active).
        bool px_ok = active, exhausted = false;
        int pgrp = grp;
        unsigned pix_t0 = (unsigned)__builtin_amdgcn_s_memrealtime();
        int rf_f = f, rf_p = 64;

        // Per-lane path state.  Every loop iteration issues exactly ONE ray
        // query for every live lane -- the path ray (nearest hit) or, while a
        // DIFF vertex is sampling its lights, that light's shadow ray (any hit)
        // -- so the sphere loop runs with all lanes of the wave active.  The
        // shading after it is organised by the operations it needs rather than
        // by material, so that lanes in different situations share one pass of
        // the expensive code (RNG draws, square root, sincos, normalisation,
        // division) instead of each situation running its own divergent block:
        //   * pass A builds a light sample's shadow ray (SampleLights) or a
        //     REFR hit's Fresnel-chosen ray;
        //   * pass B builds a DIFF bounce ray or the next sample's camera ray.
        // A lane that needs both in one iteration (a light sample that yields
        // no shadow ray, then the bounce; a refraction that ends the path,
        // then the camera ray) runs A before B, so per lane the operations and
        // RNG draws are the reference's, in its order.
        ray3 ray;              // the ray queried next
        v3 rad = mk(0.f, 0.f, 0.f), thr = mk(1.f, 1.f, 1.f);
        int depth = 0;
        bool specular = true;
        bool shadow = false;   // ray is the shadow ray of light li (DUAL: a shadow ray (hit, sdir) is pending)
        v3 sdir = mk(0.f, 0.f, 0.f);   // DUAL: the pending shadow ray's direction (origin: hit)
        bool fin = false;      // DUAL: the sample ends once its pending shadow ray is resolved
        // The last hit point IS the next ray's origin: every ray after a hit
        // (bounce, mirror, refraction, shadow) starts there, and a camera
        // ray's origin is written into it when the old hit is dead.  One
        // register triple instead of copying hit into ray.o on four paths.
        v3 &hit = ray.o;
        v3 nl;                 // the last hit's oriented normal (SampleLights' args)
        v3 lsum;               // SampleLights' running result
        float lmax = 0.f;      // shadow ray maxt (len - EPSILON)
        float lw = 0.f;        // that light's weight s (geomfunc.h:159)
        int li = 0;
        int k = active ? 0 : nsamples;      // (refill: a lane without a pixel takes one first)
        bool need_cam = active && nsamples > 0, need_bounce = false;
        BvhWalk walk;          // GEO_BVH: the current query's walk state
#ifdef RT_SPT_TRACE
        walk.tr_leaf = walk.tr_trips = walk.tr_leafruns = 0;
#endif
#ifdef RT_SPT_PROF
        for (int b = 0; b < 3; b++) walk.pf_l[b] = walk.pf_w[b] = 0;
#endif
        bool walking = false;  //   and whether it is suspended mid-walk
        constexpr float nc = 1.f, nt = 1.5f;
        // prio_sched: the three level boundaries as fractions of the samples
        // (8 bits each, in 1/256; host: prio_schedule).  Every wave starts at
        // the top priority and levels down (no group is held at the top: the
        // round-2 rule, measured best for the binary walk, cost configs[4]
        // 2-8 % with the 8-wide one, profiles/r05/c4_heavy_prio_sweep.log).
        int prio_level = 0, prio_next = (nsamples * (prio_sched & 255)) >> 8;
        __builtin_amdgcn_s_setprio(3);
        while (true) {
            if (refill) {
                // ---- refill: lanes whose pixel is done store it, then take
                // the next pixels of the wave's dispatch sequence
                const bool want = k >= nsamples && !exhausted;
                const unsigned long long wm = __builtin_amdgcn_ballot_w64(want);
                if (wm) {
                    if (want && px_ok) {
                        if (nsamples > 0) {
                            colors[3 * (size_t)i] = col.x;
                            colors[3 * (size_t)i + 1] = col.y;
                            colors[3 * (size_t)i + 2] = col.z;
                            pixels[(size_t)y * w + x] =
                                (uint32_t)(to_int(col.x) | (to_int(col.y) << 8) | (to_int(col.z) << 16));
                        }
                        seeds_out[2 * (size_t)i] = s0;
                        seeds_out[2 * (size_t)i + 1] = s1;
                        if (SCHED && group_cost) {      // the pixel's duration: per group the sum, or
                            const unsigned dur = (unsigned)__builtin_amdgcn_s_memrealtime() - pix_t0;
                            if (sflags & 4) atomicMax(&group_cost[pgrp], dur);   //   (cost_max) the longest
                            else atomicAdd(&group_cost[pgrp], dur);
                        }
                    }
                    const unsigned long long need = __builtin_amdgcn_ballot_w64(want);
                    const int ncl = __builtin_popcountll(need);
                    const int rank = __builtin_amdgcn_mbcnt_hi((unsigned)(need >> 32),
                                                               __builtin_amdgcn_mbcnt_lo((unsigned)need, 0u));
                    const bool more = rf_p + ncl > 64;
                    const int f2 = more ? fetch() : nwork;
                    if (want) {
                        const int pos = rf_p + rank;
                        const int mf = pos < 64 ? rf_f : f2, mp = pos < 64 ? pos : pos - 64;
                        px_ok = false;
                        if (mf >= nwork) {
                            exhausted = true;
                        } else {
                            const int it = mf - (n1 << hs) + n1, sl = it >> 2;
                            const int g = group_order ? (sl < nslots ? group_order[sl] : -1) : sl;
                            const int tl = g * 4 + (it & 3);
                            x = (tl % tiles_x) * 8 + (mp & 7);
                            y = row_begin + (tl / tiles_x) * 8 * gstride + (mp >> 3);
                            if ((unsigned)g < (unsigned)((ntiles + 3) >> 2) && tl < ntiles && x < w && y < row_end) {
                                i = (h - y - 1) * w + x;
                                s0 = seeds_in[2 * (size_t)i];
                                s1 = seeds_in[2 * (size_t)i + 1];
                                col = mk(0.f, 0.f, 0.f);
                                if (first_sample > 0)
                                    col = mk(colors[3 * (size_t)i], colors[3 * (size_t)i + 1], colors[3 * (size_t)i + 2]);
                                k = 0;
                                need_cam = nsamples > 0;
                                px_ok = true;
                                pgrp = g;
                                pix_t0 = (unsigned)__builtin_amdgcn_s_memrealtime();
                            }
                        }
                    }
                    if (more) {
                        rf_f = f2;
                        rf_p += ncl - 64;
                    } else {
                        rf_p += ncl;
                    }
                }
            }
            // ---- pass B: DIFF bounce (geomfunc.h:229-269) or camera ray
            // (smallptCPU.cpp:89-105).  Both draw two randoms and normalise
            // one vector.
            if (need_bounce || need_cam) {
                SPT_PROF(PB_BOUNCE);
                const float f1 = get_random_f(s0, s1), f2 = get_random_f(s0, s1);
                const float x1 = __builtin_fmaf(f1, .5f, -1.f), x2 = __builtin_fmaf(f2, .5f, -1.f);
                // bounce: r1 = 2 PI x1, r2 = x2, u = norm(a x w)
                const v3 wv = nl;
                const v3 a = (fabsf(wv.x) > .1f) ? mk(0.f, 1.f, 0.f) : mk(1.f, 0.f, 0.f);
                const v3 cu = vxcross(a, wv);
                // camera: r1 = x1 - .5, r2 = x2 - .5
                const float kcx = (x + __builtin_fmaf(f1, .5f, -1.5f)) * invW - .5f;   // r1 = GetRandom() - .5f
                const float kcy = (y + __builtin_fmaf(f2, .5f, -1.5f)) * invH - .5f;
                const v3 rdir = mk(cam.x.x * kcx + cam.y.x * kcy + cam.dir.x,
                                   cam.x.y * kcx + cam.y.y * kcy + cam.dir.y,
                                   cam.x.z * kcx + cam.y.z * kcy + cam.dir.z);
                const v3 vn = vnorm(need_bounce ? cu : rdir);
                if (need_bounce) {
                    const float r1 = 2.f * PI_F * x1;
                    const float r2s = sqrt_exact(x2);
                    const v3 v = vxcross(wv, vn);
                    float sn1, cs1;
                    rtm::sincosf(r1, sn1, cs1);
                    const v3 u = vsmul(cs1 * r2s, vn);
                    v3 nd = vadd(u, vsmul(sn1 * r2s, v));
                    nd = vadd(nd, vsmul(sqrt_exact(1 - x2), wv));
                    ray.d = nd;                          // origin: hit
                } else {
                    v3 rorig = vsmul(0.1f, rdir);
                    rorig = vadd(rorig, mk(cam.orig.x, cam.orig.y, cam.orig.z));
                    ray.o = rorig;
                    ray.d = vn;
                    // (rad, thr, depth, specular were reset when the previous
                    // sample finished: writing them only on this side made the
                    // compiler copy all six accumulators out and back around
                    // the branch every pass)
                }
                need_bounce = need_cam = false;
            }
            if (k >= nsamples) {
                if (!refill || exhausted) break;
                continue;                       // (a pixel past the frame's edge: claim again)
            }
            // Progress-levelled issue priority.  The SIMD arbitrates VALU issue
            // by priority, then age, so waves that start together finish one
            // after another and the last one runs alone at a fraction of the
            // SIMD's rate.  A wave whose every lane has passed another quarter
            // of its samples drops one priority level, letting the waves
            // behind it catch up: co-resident waves stay level and finish
            // together.  (s_setprio only reorders issue; results unchanged.)
            if (!refill && !wave_any(k < prio_next)) {
                prio_level++;
                prio_next = prio_level < 3 ? (nsamples * ((prio_sched >> (8 * prio_level)) & 255)) >> 8 : nsamples;
                if (prio_level == 1) __builtin_amdgcn_s_setprio(2);
                else if (prio_level == 2) __builtin_amdgcn_s_setprio(1);
                else __builtin_amdgcn_s_setprio(0);
            }

            SPT_PROF(PB_ITER);
#ifdef RT_SPT_TRACE
            tr_iters++;
#endif
            float t = (shadow && !DUAL) ? lmax : 1e20f;
            int first = -1;
            int id;
            bool done = false, lights = false, a_R = false;
            if constexpr (DUAL) {
                // Both rays at once when any lane holds a shadow ray; its
                // result is applied first (the light sample precedes the
                // bounce's hit in the reference's order).
                if (wave_any(shadow)) {
                    float ts = lmax;
                    int ids, firsts = -1;
                    ray3 rs;
                    rs.o = hit;
                    rs.d = sdir;
                    query2_bf<COUNT>(geo, ray, t, id, rs, shadow, ts, ids, firsts);
                    if (shadow) {                               // :154-161, then :229-230
                        SPT_PROF(PB_SHADOW);
                        cnt.isectp++;
                        cnt.tests += firsts >= 0 ? (unsigned)(S.n - firsts) : (unsigned)S.n;
                        if (ids < 0) {
                            const float4 le = S.lrec[2];
                            const v3 ld = vsmul(lw, mk(le.x, le.y, le.z));   // 0 + e * s
                            rad = vadd(rad, vmul(thr, ld));
                        }
                        shadow = false;
                        done = fin;
                    }
                } else {
                    id = query_bf<COUNT>(geo, ray, t, first);
                }
            } else if constexpr (GEO == GEO_BVH) {
                // Resumable walk: a lane whose query needs more than this
                // iteration's step budget sits out the rest of the iteration
                // and continues its walk in the next one.
#ifdef RT_SPT_TRACE
                const unsigned long long tr_w0 = __builtin_amdgcn_s_memtime();
                tr_queries += !walking;
#endif
                if (!walking) bvh_begin<COUNT>(bvh, ray, shadow, t, walk);
                walking = !bvh_walk<COUNT>(bvh, ray, shadow, walk);
#ifdef RT_SPT_TRACE
                tr_walk += (unsigned)(__builtin_amdgcn_s_memtime() - tr_w0);
#endif
                if (walking) continue;
                t = walk.t;
                id = walk.id;
                first = id;                 // any hit: the highest occluder (COUNT)
            } else if constexpr (GEO == GEO_WIDE) {
#ifdef RT_SPT_TRACE
                const unsigned long long tr_w0 = __builtin_amdgcn_s_memtime();
                tr_queries += !walking;
#endif
                if (!walking) wide_begin<COUNT>(bvh, ray, shadow, t, walk);
                if constexpr (CG != 0)
                    walking = coop ? !wide_walk_coop<COUNT, (CG ? CG : 8)>(bvh, wL, wstk, ray, shadow, walk, split)
                                   : !wide_walk<COUNT>(bvh, wL, wstk, ray, shadow, walk, split);
                else
                    walking = !wide_walk<COUNT>(bvh, wL, wstk, ray, shadow, walk, split);
#ifdef RT_SPT_TRACE
                tr_walk += (unsigned)(__builtin_amdgcn_s_memtime() - tr_w0);
#endif
                if (walking) continue;
                SPT_PROF(PB_WSHADE);
                t = walk.t;
                id = walk.id;
                first = id;                 // any hit: the highest occluder (COUNT)
            } else {
                id = query_bf<COUNT>(geo, ray, t, first);
            }
            float dp = 0.f, inv_sign = 1.f;  // REFR (pass A): vdot(normal, ray.d), -1 * sign(dp); and id
            if (DUAL && fin) {
                // the path ended at the last DIFF vertex: no path ray this iteration
            } else if (shadow && !DUAL) {                       // :154-161
                SPT_PROF(PB_SHADOW);
                cnt.isectp++;
                cnt.tests += first >= 0 ? (unsigned)(S.n - first) : (unsigned)S.n;
                if (id < 0) {
                    const float4 le = S.lrec[3 * li + 2];
                    lsum = vadd(lsum, vsmul(lw, mk(le.x, le.y, le.z)));
                }
                li++;
                lights = true;
                shadow = false;
            } else {                                            // one bounce of :182-337
                cnt.isect++;
                cnt.tests += S.n;
                if (id < 0) {
                    done = true;
                } else {
                    SPT_PROF(PB_NEAREST);
                    const float4 og = S.geo[id], oe = S.emi[id], oc = S.col[id];
                    hit = vadd(ray.o, vsmul(t, ray.d)); // ray.o + ray.d * t (hit aliases ray.o)
                    v3 normal = vsub(hit, mk(og.x, og.y, og.z));
                    normal = vnorm(normal);
                    dp = vdot(normal, ray.d);
                    inv_sign = -1.f * (dp > 0 ? 1.f : -1.f);
                    nl = vsmul(inv_sign, normal);
                    const int refl = __float_as_int(oe.w);
                    if (!((oe.x == 0.f) && (oe.x == 0.f) && (oe.z == 0.f))) {
                        if (specular) {
                            v3 e = vsmul(fabsf(dp), mk(oe.x, oe.y, oe.z));
                            e = vmul(thr, e);
                            rad = vadd(rad, e);
                        }
                        done = true;
                    } else if (refl == DIFF) {
                        SPT_PROF(PB_DIFF);
                        specular = false;
                        thr = vmul(thr, mk(oc.x, oc.y, oc.z));
                        lsum = mk(0.f, 0.f, 0.f);
                        li = 0;
                        lights = true;
                    } else if (refl == SPEC) {
                        SPT_PROF(PB_SPEC);
                        specular = true;
                        v3 nd = vsmul(2.f * vdot(normal, ray.d), normal);
                        nd = vsub(ray.d, nd);
                        thr = vmul(thr, mk(oc.x, oc.y, oc.z));
                        ray.d = nd;                             // origin: hit
                    } else {
                        SPT_PROF(PB_REFR);
                        specular = true;
                        a_R = true;                             // ray, hit, nl, dp, inv_sign, id -> pass A
                    }
                    depth++;
                    done = done || (!lights && !a_R && depth > 6);   // :184 at the next bounce
                }
            }

            // ---- pass A: SampleLights (:112-165) from light li on, stopping at
            // the next light that needs a shadow test, and/or the REFR branch
            // (:281-336).  Repeats only while some lane skips a light (several
            // lights).  UniformSampleSphere's two GetRandom() arguments are
            // drawn second-first, as the g++-built oracle does (:138); the
            // Russian-roulette draw of REFR is taken before its Fresnel terms
            // (no other draw of the lane lies between).
            bool a_L = lights && li < S.nlights;
            bool lights_done = lights && !a_L;
            const bool was_R = a_R;
            // One pass for every lane that needs A, then further light-only
            // passes while some lane skipped a light (scenes with several
            // lights).  The body is one lambda instantiated twice so the
            // common single pass is straight-line code (a loop around both
            // made the compiler shuffle all loop-carried state every pass).
            const auto pass_a = [&](const bool with_r) {
                {
                    SPT_PROF(PB_LIGHT);
                    // Loaded by every lane (an R-only lane's light terms are
                    // discarded by the selects below; li is clamped into the
                    // light list) -- a conditional load left five zeroing
                    // moves and a branch in every pass.
                    const int lj = li < S.nlights ? li : 0;
                    const float4 lg = S.lrec[3 * lj];           // centre
                    const float4 lc = S.lrec[3 * lj + 1];       // colour.xyz, rad
                    // REFR terms (:281-296), rebuilt here from the few values
                    // kept since the hit: normal = inv_sign * nl exactly
                    // (inv_sign = +-1), and, rounding being sign-symmetric,
                    // vdot(normal, nl) = inv_sign * |n|^2 and vdot(ray.d, nl) =
                    // inv_sign * dp exactly: into is dp <= 0 (false for NaN, as
                    // the reference's NaN dot) and ddn is dp signed.
                    const v3 normal = vsmul(inv_sign, nl);
                    const bool into = dp <= 0.f;
                    const float nnt = into ? nc / nt : nt / nc;
                    const float ddn = inv_sign * dp;
                    const float cos2t = 1.f - nnt * nnt * (1.f - ddn * ddn);
                    const bool tir = cos2t < 0.f;
                    float x1 = 0.f, x2 = 0.f;
                    if (a_L || (with_r && !tir)) x1 = get_random(s0, s1);   // L: u2; R: the roulette draw
                    if (a_L) x2 = get_random(s0, s1);           // L: u1
                    const float zz = 1.f - 2.f * x2;            // UniformSampleSphere, :61-69
                    const float q = 1.f - zz * zz;
                    const float sq = sqrt_exact((!with_r || a_L) ? ((0.f > q) ? 0.f : q) : (tir ? 1.f : cos2t));
                    const float phi = 2.f * PI_F * x1;
                    float sp_sin, sp_cos;
                    rtm::sincosf(phi, sp_sin, sp_cos);
                    const v3 unit = mk(sq * sp_cos, sq * sp_sin, zz);
                    v3 sp = vsmul(lc.w, unit);
                    sp = vadd(sp, mk(lg.x, lg.y, lg.z));
                    const v3 vl = vsub(sp, hit);                // shadow ray direction
                    const float kk = (into ? 1.f : -1.f) * (ddn * nnt + sq);
                    const v3 vr = vsub(vsmul(nnt, ray.d), vsmul(kk, normal));   // refracted direction
                    const v3 vv = (!with_r || a_L) ? vl : vr;
                    const float dd = vdot(vv, vv);
                    float len, ilen;                            // sqrtf(dd), 1.f / len
                    if (!wave_any(!sqrt_nr_ok(dd))) {
                        len = sqrt_nr(dd);
                        ilen = rcp_nr(len);
                    } else {
                        len = sqrt_rn(dd);
                        ilen = 1.f / len;
                    }
                    const v3 vn = vsmul(ilen, vv);
                    const float dv = vdot(vn, (!with_r || a_L) ? unit : normal);   // L: wo; R: vdot(td, normal)
                    // L: weight (4 PI rad^2) wi wo / len^2; R: RP = Re / P or TP = Tr / (1 - P)
                    const float wo = -dv;
                    const float wi = vdot(vn, nl);
                    const bool lit = a_L && !(dv > 0.f) && wi > 0.f;
                    const float a = nt - nc, b = nt + nc;
                    const float R0 = a * a / (b * b);
                    const float c = 1 - (into ? -ddn : dv);
                    const float Re = R0 + (1 - R0) * c * c * c * c * c;
                    const float Tr = 1.f - Re;
                    const float P = .25f + .5f * Re;
                    const bool refl_pick = x1 < P;
                    const bool l_lane = !with_r || a_L;
                    const float num = l_lane ? (4.f * PI_F * lc.w * lc.w) * wi * wo : (refl_pick ? Re : Tr);
                    const float den = l_lane ? len * len : (refl_pick ? P : 1.f - P);
                    const float quo = num / den;
                    if (!with_r || a_L) {
                        if (lit) {
                            if (DUAL) {
                                sdir = vn;                      // queried next iteration, with the bounce ray
                            } else {
                                ray.d = vn;                     // origin: hit
                            }
                            lmax = len - EPS;
                            lw = quo;
                            shadow = true;
                            a_L = false;
                            if (DUAL) lights_done = true;       // the only light
                        } else {
                            li++;
                            a_L = li < S.nlights;
                            lights_done = !a_L;
                        }
                    } else {
                        const float4 oc = S.col[id];
                        v3 nd = vsmul(2.f * dp, normal);         // vdot(normal, ray.d) = dp
                        nd = vsub(ray.d, nd);
                        if (tir) {                              // origin: hit
                            thr = vmul(thr, mk(oc.x, oc.y, oc.z));
                            ray.d = nd;
                        } else {
                            thr = vsmul(quo, thr);
                            thr = vmul(thr, mk(oc.x, oc.y, oc.z));
                            ray.d = refl_pick ? nd : vn;
                        }
                        a_R = false;
                    }
                }
            };
            // A scene without REFR spheres (sflags bit 0: configs[4]'s 10k
            // spheres are all DIFF) never sets a_R: its lanes take the
            // light-only body, whose operations and draws for an a_L lane are
            // pass_a(true)'s without the Fresnel / refraction terms it would
            // compute and discard (~45 VALU per pass).  Hierarchy kernels only.
            if ((GEO == GEO_BVH || GEO == GEO_WIDE) && (sflags & 1)) {
                if (a_L) pass_a(false);
            } else if (a_L || a_R) {
                pass_a(true);
            }
            // With one light the pass above always leaves a_L false (lit, or
            // li = 1 = nlights); the scalar test keeps the light-only loop --
            // and the copies of the loop-carried state the compiler puts at
            // its header, 12 VALU ops per iteration -- out of such scenes.
            if (S.nlights > 1) {
                while (wave_any(a_L)) {
                    if (a_L) pass_a(false);
                }
            }
            if (was_R) done = depth > 6;
            if (lights_done) {                                  // :229-230, then the bounce
                // (DUAL: Ld is 0 + e * s once the pending shadow ray is
                // resolved, or 0 -- and rad + thr * 0 == rad -- if none.)
                if (!DUAL) rad = vadd(rad, vmul(thr, lsum));
                if (DL) {
                    done = true;                                // :413-414
                } else if (depth > 6) {                         // the bounce's two draws, then :184
                    (void)get_random(s0, s1);
                    (void)get_random(s0, s1);
                    if (DUAL && shadow) fin = true;             // ends after the shadow result
                    else done = true;
                } else {
                    need_bounce = true;
                }
            }
            if (done) {                                         // :110-118 running average
                SPT_PROF(PB_DONE);
                const int current = first_sample + k;
                if (current == 0) {
                    col = rad;
                } else {
                    const float k1 = (float)current;
                    const float k2 = rcp_nr(k1 + 1.f);      // 2 <= k1 + 1 <= 2^31: rcp_nr range
                    col.x = (col.x * k1 + rad.x) * k2;
                    col.y = (col.y * k1 + rad.y) * k2;
                    col.z = (col.z * k1 + rad.z) * k2;
                }
                cnt.samples++;
                if (CALLS && (cnt.isect | cnt.isectp) >= 0x80000000u) {   // (long launches: before 32 bits wrap)
                    atomicAdd(counters, (unsigned long long)cnt.isect);
                    atomicAdd(counters + 1, (unsigned long long)cnt.isectp);
                    cnt.isect = cnt.isectp = 0;
                }
                k++;
                need_cam = k < nsamples;
                fin = false;
                rad = mk(0.f, 0.f, 0.f);                        // the next sample's path state
                thr = mk(1.f, 1.f, 1.f);                        // (smallptCPU.cpp:89-105 via pass B)
                depth = 0;
                specular = true;
            }
        }
        if (GSTORE) {                                   // staged: the group's last wave stores it
            float *gs_col = (float *)GS_BASE();
            uint32_t *gs_seed = (uint32_t *)(GS_BASE() + 3072), *gs_px = (uint32_t *)(GS_BASE() + 5120);
            const int c = (wave & 3) * 8 + (lane & 7), r = lane >> 3;
            if (nsamples > 0) {
                gs_col[r * 96 + 3 * c] = col.x;
                gs_col[r * 96 + 3 * c + 1] = col.y;
                gs_col[r * 96 + 3 * c + 2] = col.z;
                gs_px[r * 32 + c] = (uint32_t)(to_int(col.x) | (to_int(col.y) << 8) | (to_int(col.z) << 16));
            }
            gs_seed[r * 64 + 2 * c] = s0;
            gs_seed[r * 64 + 2 * c + 1] = s1;
        } else if (lead && !refill) {            // (refill: stored as each pixel finished)
            if (nsamples > 0) {
                colors[3 * (size_t)i] = col.x;
                colors[3 * (size_t)i + 1] = col.y;
                colors[3 * (size_t)i + 2] = col.z;
                pixels[(size_t)y * w + x] =
                    (uint32_t)(to_int(col.x) | (to_int(col.y) << 8) | (to_int(col.z) << 16));
            }
            seeds_out[2 * (size_t)i] = s0;
            seeds_out[2 * (size_t)i + 1] = s1;
        }
#ifdef RT_SPT_PROF
        for (int b = 0; b < 3; b++) {
            prof_l[PB_WCALL + b] += walk.pf_l[b];
            prof_w[PB_WCALL + b] += walk.pf_w[b];
        }
#endif
#ifdef RT_SPT_TRACE
        if (GEO == GEO_BVH || GEO == GEO_WIDE) {
            tr_leaf = walk.tr_leaf;
            tr_trips = walk.tr_trips;
            tr_leafruns = walk.tr_leafruns;
        }
#endif
    }
    if (GSTORE) {
        // The group's four waves finish at different times (configs[4]: per-
        // wave work varies 6x); each leaves its 8x8 tile in LDS and the last
        // one stores the whole 32x8 strip, so every 128-B line of the colour,
        // seed and pixel rows is written once, whole.  (Stored per wave, the
        // 96-B colour and 32-B pixel row segments of a tile share lines with
        // the neighbouring tiles' and reach HBM as partial lines when the
        // neighbours finish much later: 71 MB written per frame for 50 MB.)
        const float *gs_col = (const float *)GS_BASE();
        const uint32_t *gs_seed = (const uint32_t *)(GS_BASE() + 3072), *gs_px = (const uint32_t *)(GS_BASE() + 5120);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        int old = 0;
        if (lane == 0) old = atomicAdd((int *)(GS_BASE() + 6144), 1);
        old = __shfl(old, 0, 64);
        if (old == 3) {
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
            // entry (row r, group column c) -> its pixel, or invalid
            const auto pix = [&](int r, int c, int &xx, int &yy) {
                const int tl = grp * 4 + (c >> 3);
                xx = (tl % tiles_x) * 8 + (c & 7);
                yy = row_begin + (tl / tiles_x) * 8 * gstride + r;
                return gvalid && tl < ntiles && xx < w && yy < row_end;
            };
            int xx, yy;
            if (nsamples > 0) {
#pragma unroll 4
                for (int k = 0; k < 12; k++) {
                    const int j = k * 64 + lane, r = j / 96, c3 = j % 96, c = c3 / 3;
                    if (pix(r, c, xx, yy)) colors[3 * ((size_t)(h - yy - 1) * w + xx) + (c3 - 3 * c)] = gs_col[j];
                }
#pragma unroll
                for (int k = 0; k < 4; k++) {
                    const int j = k * 64 + lane, r = j >> 5, c = j & 31;
                    if (pix(r, c, xx, yy)) pixels[(size_t)yy * w + xx] = gs_px[j];
                }
            }
#pragma unroll
            for (int k = 0; k < 8; k++) {
                const int j = k * 64 + lane, r = j >> 6, c2 = j & 63, c = c2 >> 1;
                if (pix(r, c, xx, yy)) seeds_out[2 * ((size_t)(h - yy - 1) * w + xx) + (c2 & 1)] = gs_seed[j];
            }
        }
    }
#undef GS_BASE
    if (SCHED && group_cost && gvalid && lane == 0 && !refill) {  // this tile's duration (100 MHz ticks), summed per group
        const unsigned dur = (unsigned)(__builtin_amdgcn_s_memrealtime() - t_start);
        if (sflags & 4) atomicMax(&group_cost[grp], dur);           // (Shape::cost_max: the group's longest tile)
        else atomicAdd(&group_cost[grp], dur);
    }
#ifdef RT_SPT_TRACE
    {
        const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
        unsigned mx = tr_iters;
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) mx = max(mx, (unsigned)__shfl_xor((int)mx, off, 64));
        const unsigned sum = (unsigned)wave_sum_u64(tr_iters);
        const size_t wv = (size_t)f;                       // one record per work item (tile)
        const unsigned tr_tot = (unsigned)(__builtin_amdgcn_s_memtime() - tr_c0);
        unsigned ph[6] = {tr_walk, tr_leaf, tr_trips, tr_leafruns, tr_queries, tr_tot};
#pragma unroll
        for (int q = 0; q < 6; q++)
#pragma unroll
            for (int off = 32; off > 0; off >>= 1) ph[q] = max(ph[q], (unsigned)__shfl_xor((int)ph[q], off, 64));
        if (lane == 0 && g_spt_trace) {
            g_spt_trace[4 * wv] = make_uint4((unsigned)tr_t0, (unsigned)t1, __builtin_amdgcn_s_getreg(0xF804),
                                             __builtin_amdgcn_s_getreg(0xF814));
            g_spt_trace[4 * wv + 1] = make_uint4(sum, mx, (unsigned)grp, ph[5]);
            g_spt_trace[4 * wv + 2] = make_uint4(ph[0], ph[1], ph[2], ph[3]);
            g_spt_trace[4 * wv + 3] = make_uint4(ph[4], 0u, 0u, 0u);
        }
    }
#endif
    if (CALLS && PERSIST && (split & 4)) {              // a cooperative group counts its pixel once:
        if (!lead) cnt = Counts{0, 0, 0, 0};            //   flushed per work item
        const unsigned long long c[4] = {cnt.isect, cnt.isectp, COUNT ? cnt.tests : 0ull, cnt.samples};
        flush_counters<4>(counters, c);
        cnt = Counts{0, 0, 0, 0};
    }
    if (!PERSIST || refill) break;          // (refill: the wave took pixels until the window ran out)
    f = __builtin_amdgcn_readfirstlane(fetch());
    }   // work items
    if (CALLS) {
        const unsigned long long c[4] = {cnt.isect, cnt.isectp, COUNT ? cnt.tests : 0ull, cnt.samples};
        flush_counters<4>(counters, c);
    }
#ifdef RT_SPT_PROF
#pragma unroll
    for (int b = 0; b < PB_N; b++) {
        const unsigned long long l = wave_sum_u64(prof_l[b]), v = wave_sum_u64(prof_w[b]);
        if (lane == 0) { atomicAdd(&g_spt_prof[2 * b], l); atomicAdd(&g_spt_prof[2 * b + 1], v); }
    }
#endif
}

// toInt pack of rows [row_begin, row_end) from the accumulator: the pixels
// render_kernel writes at the end of a launch (smallptCPU.cpp:120-122), for a
// frame whose colour bands came from other ranks.
__global__ void __launch_bounds__(256) pack_kernel(const float *__restrict__ colors, uint32_t *__restrict__ pixels,
                                                   int w, int h, int row_begin, int row_end)
{
    const size_t n = (size_t)(row_end - row_begin) * w;
    for (size_t p = (size_t)blockIdx.x * blockDim.x + threadIdx.x; p < n; p += (size_t)gridDim.x * blockDim.x) {
        const int y = row_begin + (int)(p / w), x = (int)(p % w);
        const size_t i = (size_t)(h - y - 1) * w + x;
        pixels[(size_t)y * w + x] =
            (uint32_t)(to_int(colors[3 * i]) | (to_int(colors[3 * i + 1]) << 8) | (to_int(colors[3 * i + 2]) << 16));
    }
}

// Tile groups <-> a packed buffer (a multi-GPU frame split by explicit group
// lists, spt_groups_pack_async): group g is the 8x8 tiles 4g .. 4g+3 of the
// frame in row-major tile order; its 768 packed floats are tile by tile, row
// by row, pixel by pixel, (r, g, b) -- the accumulator slots (h-y-1)*w+x.
// Pixels outside the frame (and entries outside [0, ngroups_total)) pack as
// 0 and are skipped when unpacking.  Exact copies.
constexpr int GROUP_FLOATS = 4 * 64 * 3;
template <bool PACK>
__global__ void __launch_bounds__(256) groups_copy_kernel(float *__restrict__ colors, int w, int h,
                                                          const int *__restrict__ groups, int n,
                                                          float *__restrict__ buf)
{
    const int tiles_x = (w + 7) / 8, ntiles = tiles_x * ((h + 7) / 8), total = (ntiles + 3) / 4;
    const size_t ne = (size_t)n * GROUP_FLOATS;
    for (size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x; e < ne; e += (size_t)gridDim.x * blockDim.x) {
        const int k = (int)(e / GROUP_FLOATS), q = (int)(e % GROUP_FLOATS);
        const int g = groups[k];
        const int tile = g * 4 + q / 192, p = (q % 192) / 3, comp = q % 3;
        const int x = (tile % tiles_x) * 8 + (p & 7), y = (tile / tiles_x) * 8 + (p >> 3);
        const bool in = (unsigned)g < (unsigned)total && tile < ntiles && x < w && y < h;
        const size_t i = 3 * ((size_t)(h - 1 - y) * w + x) + comp;
        if (PACK) buf[e] = in ? colors[i] : 0.f;
        else if (in) colors[i] = buf[e];
    }
}

// A caller's group list made a set (spt_scene_render_list_async): one entry
// per listed group survives into `out` -- the one whose claim on the group's
// bit of `claimed` (zeroed) came first -- and every repeat or out-of-range
// entry becomes -1, which render_kernel skips.  Two waves can then never
// render the same pixels (their accumulator and seed slots) in one launch, and
// a group's wave time is added to its cost entry once.  Which copy of a repeat
// survives moves only its dispatch slot, never a result.
__global__ void __launch_bounds__(256) list_dedup_kernel(const int *__restrict__ groups, int n, int total,
                                                         unsigned *__restrict__ claimed, int *__restrict__ out)
{
    for (int k = blockIdx.x * blockDim.x + threadIdx.x; k < n; k += gridDim.x * blockDim.x) {
        const int g = groups[k];
        int v = -1;
        if ((unsigned)g < (unsigned)total) {
            const unsigned bit = 1u << (g & 31);
            if (!(atomicOr(&claimed[g >> 5], bit) & bit)) v = g;
        }
        out[k] = v;
    }
}

}  // namespace smallpt
}  // namespace rt

// ------------------------------------------------------------------ host side
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <algorithm>
#include <mutex>
#include <string>
#include <vector>
#include "rt_runtime.h"
#include "spt_bvh.h"

// A prepared scene (spt_scene_create): device AoS copy for the per-block LDS
// staging, device SoA + light list for scenes above the LDS budget.
// Adaptive dispatch order of a scene's tile groups (scene_render): the first
// launch for a given window / camera / sample count records each group's
// wave time; once that is back on the host, later launches of the same key
// dispatch the groups heaviest first, so the long tiles of a non-uniform
// scene (configs[4]: per-wave work varies 6x) start at once instead of
// setting the frame's tail.  Scheduling only: every pixel's computation is
// unchanged.
struct SptSched {
    int w = 0, h = 0, r0 = 0, r1 = 0, gstride = 0, ns = -1, mode = -1, nslots = 0;
    rt_camera cam = {};
    int state = 0;                    // 0: none, 1: costs recorded (copy in flight), 2: order set
    int cap = 0;
    unsigned *d_cost = nullptr, *h_cost = nullptr;   // h_*: pinned
    int *d_order = nullptr, *h_order = nullptr;
    hipEvent_t ev = nullptr;
    // d_order is never rewritten or freed once a stream capture has used it
    // (the graph holds its address): it is retired instead and freed with
    // the scene, and a fresh buffer takes the next order.
    bool order_captured = false;
    std::vector<int *> retired;
};

struct spt_scene {
    int device = -1;
    int cus = 256;
    int n = 0;
    rt_sphere *d_spheres = nullptr;   // n x 44 B
    float4 *d_soa = nullptr;          // geo | emi | col (n each) | light records (3 per light)
    int nlights = 0;
    void *d_bvh = nullptr;            // nodes | geo | id | always geo | always id | wide nodes (large scenes)
    rt::smallpt::BvhView bvh = {};
    std::vector<rt_sphere> host;
    bool force_global = false;        // RT_SPT_GEO=global: scalar-load path at any size (A/B)
    mutable SptSched sched;           // adaptive group order (hierarchy scenes)
    mutable SptSched sched_cnt;       //   ... of the full-counter launches (their own tile costs)
    // Work counters of the persistent (8-wide hierarchy) launches: a ring,
    // one zeroed quad (rest, routed heavy, cooperative, unused) per launch, so
    // launches in flight on several streams do not share one.
    // An entry a stream capture used is baked into that graph, which may be
    // replayed at any time: it is never handed out again (work_captured).
    // spt_scene_release_captures hands those entries out again once the
    // caller has destroyed the graphs.  work_mu guards the ring's host state
    // (launches of one scene from several host threads).
    static constexpr int NWORK = 64;
    int *d_work = nullptr;
    mutable std::mutex work_mu;
    mutable int work_next = 0;
    mutable unsigned long long work_captured = 0;
    bool no_refr = false;             // no sphere has refl == REFR (render_kernel sflags bit 0)
};

namespace {
// 8-wide hierarchy launches: blocks of WIDE_WPB waves (each holds its own
// LDS copy of the nodes and its waves' stacks), one per CU at the kernel's
// occupancy of 4 waves per SIMD.
constexpr int WIDE_WPB = 16;
constexpr size_t WIDE_LDS_MAX = 144 * 1024;
size_t wide_lds_bytes(int wnodes, int wdepth, int wpb, bool counted = true)
{
    return (size_t)(counted ? 144 : 112) * wnodes + (size_t)wpb * 256 * (wdepth > 1 ? wdepth - 1 : 1);
}

// The launch policy's tuning knobs, in one place.  The defaults are the
// measured best; RT_SPT_TUNE="key=value,..." overrides any of
// them for an A/B run or a test (read at every launch, so a test may change
// it between frames).  Keys:
//   coop=N      cooperative (tier-1) tiles of an ordered 8-wide launch
//               (default: 2 x CUs at <= 5 waves of work per SIMD, 4 x CUs at
//               <= 10, else 0)
//   coop_g=G    lanes per pixel of those tiles, 8, 4 or 2 (default 8 at <= 5
//               waves of work per SIMD, 4 at <= 10, 2 at <= 20)
//   coop_waves=K waves of each block that fetch tier-1 sub-items first (16)
//   routed=N    tier-2 tiles routed one per SIMD (default 4 x blocks when
//               there is no cooperative tier, else 0)
//   walk=B/P/S  wide_walk: trip budget per call, leaf batch threshold and
//               early stop, both in 1/64 of the call's lanes (16/16/32; the
//               stop 16 in windows with a cooperative tier)
//   prio=A/B/C  priority-levelling boundaries in 1/256 of the samples
//               (64/128/192 for the 4-wave block shape, 128/192/224 for 16)
//   wpb=4|16    full-scan block shape (default: by waves of work per SIMD)
//   blocks=N    8-wide persistent grid size (default: one block per CU)
struct SptTune {
    int coop = -1, coop_g = 0, coop_waves = -1, routed = -1;
    int budget = 16, batch = 16, stop = -1;     // (stop -1: by window, see launch)
    int prio[3] = {-1, -1, -1};
    int wpb = 0, blocks = 0;
};
SptTune spt_tune()
{
    SptTune t;
    const char *e = getenv("RT_SPT_TUNE");
    if (!e) return t;
    std::string all(e);
    size_t pos = 0;
    while (pos < all.size()) {
        size_t end = all.find(',', pos);
        if (end == std::string::npos) end = all.size();
        const std::string kv = all.substr(pos, end - pos);
        pos = end + 1;
        const size_t eq = kv.find('=');
        if (eq == std::string::npos) continue;
        const std::string k = kv.substr(0, eq);
        const char *v = kv.c_str() + eq + 1;
        if (k == "coop") t.coop = std::max(atoi(v), 0);
        else if (k == "coop_g") t.coop_g = atoi(v) == 4 ? 4 : (atoi(v) == 2 ? 2 : 8);
        else if (k == "coop_waves") t.coop_waves = std::min(std::max(atoi(v), 0), 16);
        else if (k == "routed") t.routed = std::max(atoi(v), 0);
        else if (k == "walk") sscanf(v, "%d/%d/%d", &t.budget, &t.batch, &t.stop);
        else if (k == "prio") sscanf(v, "%d/%d/%d", &t.prio[0], &t.prio[1], &t.prio[2]);
        else if (k == "wpb") t.wpb = atoi(v) == 16 ? 16 : 4;
        else if (k == "blocks") t.blocks = std::max(atoi(v), 0);
    }
    return t;
}

// Launch shape: one wave per 8x8 tile of rows [r0, r1).  256-thread blocks
// (several per CU, dispatched as CUs free up) unless the window has at most
// four tiles per SIMD (a multi-GPU row band): then 1024-thread blocks with
// more than half the CU's LDS reserved, so a CU holds exactly one and every
// SIMD gets four waves, instead of the dispatcher's uneven 3..5 per SIMD.
struct Shape {
    int tiles_x, ntiles, gstride, wpb, nblocks;
    int work = 0;                     // tiles this launch renders (ntiles, or 4 x a group list's length)
    int nslots = 0;                   // dispatch slots (tile groups of four) the order / cost arrays cover
    const int *order = nullptr;       // adaptive schedule (render_kernel's group_order / group_cost)
    unsigned *cost = nullptr;
    bool tiers = true;                // with order: its first tiles get the heavy-tile treatment
    bool cost_max = false;            // cost: a group's longest tile (atomic max), not the sum
    SptTune tune;
};
// Rows [r0, r1), or (gstride > 1) the 8-row groups r0/8, r0/8 + gstride, ...
// below r1 (r0 a multiple of 8); or (nlist > 0) the nlist tile groups of a
// caller's list over the frame [r0, r1) = [0, h).
Shape launch_shape(const spt_scene &sc, int w, int r0, int r1, int gstride = 1, int nlist = 0)
{
    Shape g;
    g.tune = spt_tune();
    g.tiles_x = (w + 7) / 8;
    g.gstride = gstride;
    const int groups = (r1 - r0 + 7) / 8;
    g.ntiles = g.tiles_x * ((groups + gstride - 1) / gstride);
    const int work = nlist > 0 ? 4 * nlist : g.ntiles;      // tiles this launch renders
    g.work = work;
    // Waves of work per SIMD: up to 4 (an N = 8 band) run as one round of the
    // 16-wave block shape (four waves per SIMD, one block per CU); 6..8 (an
    // N = 4 band: 7.97) as two such rounds -- at occupancy 6 they run as a
    // full round of 6 and a tail of 2 (N = 4 bands 5.25-5.87 ms -> 5.44-5.47
    // ms); otherwise 256-thread blocks at the kernel's occupancy.
    const double wps = (double)work / (4.0 * sc.cus);
    g.wpb = (wps <= 4.0 || (wps > 6.0 && wps <= 8.0)) ? 16 : 4;
    if (g.tune.wpb) g.wpb = g.tune.wpb;
    g.nblocks = (work + g.wpb - 1) / g.wpb;
    g.nslots = nlist > 0 ? nlist : g.nblocks * (g.wpb / 4);
    if (sc.bvh.wnode) {               // persistent waves: one block per CU (fewer for a small window)
        g.wpb = WIDE_WPB;
        g.nblocks = std::min(sc.cus, (work + g.wpb - 1) / g.wpb);
        if (g.tune.blocks) g.nblocks = g.tune.blocks;
        g.nslots = nlist > 0 ? nlist : (g.ntiles + 3) / 4;
    }
    return g;
}

// Priority levelling schedule (render_kernel's prio_sched): levels at 1/4,
// 1/2, 3/4 of the samples for the full-frame shape; for the 16-wave block
// shape (multi-GPU windows of <= 8 waves per SIMD, one or two rounds) at
// 1/2, 3/4, 7/8 -- finer where the co-resident waves drain.
int prio_schedule(const Shape &g)
{
    int a = 64, b = 128, c = 192;
    if (g.wpb == 16) { a = 128; b = 192; c = 224; }
    if (g.tune.prio[0] >= 0) { a = g.tune.prio[0]; b = g.tune.prio[1]; c = g.tune.prio[2]; }
    return (a & 255) | ((b & 255) << 8) | ((c & 255) << 16);
}

// A zeroed work-counter quad of the scene's ring for one persistent launch
// on `s` (nullptr + rt error: none left).
int *work_entry(const spt_scene &sc, hipStream_t s)
{
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    const bool capturing = hipStreamIsCapturing(s, &cs) == hipSuccess && cs != hipStreamCaptureStatusNone;
    std::lock_guard<std::mutex> lk(sc.work_mu);
    for (int tries = 0; tries < spt_scene::NWORK; tries++) {
        const int k = sc.work_next++ % spt_scene::NWORK;
        if ((sc.work_captured >> k) & 1ull) continue;
        if (capturing) sc.work_captured |= 1ull << k;
        int *work = sc.d_work + 4 * k;
        if (hipMemsetAsync(work, 0, 4 * sizeof(int), s) != hipSuccess) return nullptr;   // (check_launch reports it)
        return work;
    }
    rtrt::fail(RT_ERR_INVALID, "spt render: every work-counter entry of the scene is held by a captured graph");
    return nullptr;
}

template <bool DL, bool COUNT, int GEO, bool DUAL = false, bool RAYS = false>
int launch(const Shape &g, hipStream_t s, const spt_scene &sc, const rt_camera &cam, float *colors,
           const uint32_t *sin, uint32_t *sout, uint32_t *pixels, int w, int h, int r0, int r1,
           int first, int ns, unsigned long long *cnt)
{
    constexpr bool LDS = GEO == rt::smallpt::GEO_LDS;
    const int n = sc.n;
    const float4 *gg = sc.d_soa, *ge = gg + n, *gc = ge + n, *gl = gc + n;
    size_t lds = LDS ? (size_t)(3 * n + 3 * std::max(sc.nlights, 1)) * sizeof(float4) : 0;
    if (GEO == rt::smallpt::GEO_BVH) lds = (size_t)(g.wpb / 4) * rt::smallpt::GS_BYTES;
    if (g.wpb == 16 && lds < 81 * 1024) lds = 81 * 1024;   // > half the CU's 160 KiB: one block per CU
    int *work = nullptr;
    int sflags = sc.no_refr ? 1 : 0;
    if (g.cost_max) sflags |= 4;
    if (GEO == rt::smallpt::GEO_WIDE) {
        lds = wide_lds_bytes(sc.bvh.wnodes, sc.bvh.wdepth, g.wpb, COUNT);
        if (!(work = work_entry(sc, s))) return rtrt::check_launch("spt work counters") ? RT_ERR_HIP : RT_ERR_INVALID;
    }
    // Heavy tiles (with a learnt order, GEO_WIDE persistent launches), in
    // dispatch order: n1 cooperative tiles (8 or 4 lanes per pixel,
    // wide_walk_coop), fetched first by hw waves of each block, then n2 tiles
    // routed one per SIMD beside lighter waves, then the rest.  A window of
    // many waves of work per SIMD (a full frame: 31.6) is throughput-bound:
    // routing only.  A window of few (a multi-GPU rank's share: N = 8 is 4.0,
    // N = 4 7.9, N = 2 15.8) is bound by its heaviest tiles' sample chains,
    // which the cooperative walk shortens ~2x at ~3x their issue cost (8
    // lanes per pixel at N = 8, 4 at N = 4, 2 at N = 2).
    // configs[4], 64 spp (profiles/r03/c4_coop_*.log): N = 8 windows
    // 18.0-19.8 -> 11.4-15.1 ms, N = 4 18.7 -> 17 ms; see DESIGN.md.
    const SptTune &tu = g.tune;
    int n1 = 0, n2 = 0, sp = 0, kcg = 0;
    if (GEO == rt::smallpt::GEO_WIDE && g.order && g.tiers) {
        n2 = std::min(4 * g.nblocks, 4 * g.nslots);
        const double wps = (double)g.work / (4.0 * sc.cus);
        int hw = 0, cg = 8;
        if (wps <= 5.0) {
            n1 = 2 * sc.cus;
            hw = 16;
        } else if (wps <= 10.0) {
            // An N = 4 share holds more ~13 ms chains than 512 tiles at
            // eight lanes per pixel cover (c4_phase_n4.log): twice the tiles
            // at four lanes per pixel, fetched by every wave of the block
            // first (one round: 4 sub-items x 1,024 tiles = 16 waves per CU).
            // N = 4 shares 16.3-16.6 -> 13.8 ms; at N = 8 four lanes lose
            // (9.9 -> 13.5 ms), c4_coop_g4_ab.log.
            n1 = 4 * sc.cus;
            hw = 16;
            cg = 4;
        } else if (wps <= 20.0) {
            // An N = 2 share (15.8 waves of work per SIMD): still bound by its
            // heaviest chains, and too full for four- or eight-lane tiers to
            // pay (20.5 -> 19.8-23 ms); two lanes per pixel for the heaviest
            // 1,024 tiles halve their walks at the least duplicated shading:
            // 20.5 -> 19.3-19.5 ms (round 6, c4_coop_g2_ab.log; 768-1,024
            // best, 1,280+ slower; at N = 4 two lanes lose to four).
            n1 = 4 * sc.cus;
            cg = 2;
        }
        if (tu.coop_g) cg = tu.coop_g;
        if (tu.coop >= 0) n1 = tu.coop;
        if (tu.coop_waves >= 0) hw = tu.coop_waves;
        if (n1 > 0) n2 = 0;   // routed tiles beside cooperative ones: N = 4 17 -> 24 ms (c4_coop_tiers_ab.log)
        if (tu.routed >= 0) n2 = tu.routed;
        n1 = std::min(n1, 4 * g.nslots);
        n2 = std::min(n2, 4 * g.nslots - n1);
        if (n1 > 0) sp = (cg == 8 ? 3 : cg == 4 ? 2 : 1) | 4 | (hw << 3);
        kcg = n1 > 0 ? cg : 0;
    }
    const int nheavy = std::min(n1, 0xffff) | (std::min(n2, 0xffff) << 16);
    int split = 0;
    if (GEO == rt::smallpt::GEO_WIDE) {
        // A walk call returns once <= stop/64 of the lanes that started it
        // still walk: 32 on the full frame; 16 in a window with a cooperative
        // tier, where the heaviest waves' chains bound the share (round 6,
        // with the deferred leaf sections: N = 8 9.5 -> 9.2 ms, N = 4 13.2 ->
        // 12.8 ms, profiles/r06/c4_walk_stop_sweep.log).
        const int stop = tu.stop >= 0 ? tu.stop : (n1 > 0 ? 16 : 32);
        split = sp | (std::min(std::max(tu.budget, 1), 255) << 8) | (std::min(std::max(tu.batch, 0), 64) << 16) |
                (std::min(std::max(stop, 0), 64) << 24);
    }
    // (the kernel carries the cooperative walk only when this launch has a
    // cooperative tier, and only the group size it uses)
    auto kern = rt::smallpt::render_kernel<DL, COUNT, GEO, DUAL, RAYS, 0>;
    if constexpr (GEO == rt::smallpt::GEO_WIDE) {
        if (kcg == 8) kern = rt::smallpt::render_kernel<DL, COUNT, GEO, DUAL, RAYS, 8>;
        else if (kcg == 4) kern = rt::smallpt::render_kernel<DL, COUNT, GEO, DUAL, RAYS, 4>;
        else if (kcg == 2) kern = rt::smallpt::render_kernel<DL, COUNT, GEO, DUAL, RAYS, 2>;
    }
    hipLaunchKernelGGL(kern, dim3(g.nblocks), dim3(64 * g.wpb), lds, s,
                       sc.d_spheres, n, cam, colors, sin, sout, pixels, w, h, r0, r1, g.tiles_x, g.ntiles, g.nslots, g.gstride, first,
                       ns, prio_schedule(g), g.order, g.cost, gg, ge, gc, gl, sc.nlights, sc.bvh, cnt, work, split,
                       nheavy, sflags);
    return RT_OK;
}

// Counter modes of a launch: none, all four counters, or calls and samples
// only (SPT_COUNT_RAYS: the uncounted queries).
enum { CNT_NONE = 0, CNT_FULL = 1, CNT_RAYS = 2 };

template <int GEO, bool DL, bool DUAL>
int launch_counted(int cmode, const Shape &grid, hipStream_t s, const spt_scene &sc, const rt_camera &cam,
                   float *colors, const uint32_t *sin, uint32_t *sout, uint32_t *pixels, int w, int h, int r0,
                   int r1, int first, int ns, unsigned long long *cnt)
{
    if (cmode == CNT_FULL)
        return launch<DL, true, GEO, DUAL>(grid, s, sc, cam, colors, sin, sout, pixels, w, h, r0, r1, first, ns, cnt);
    if (cmode == CNT_RAYS)
        return launch<DL, false, GEO, DUAL, true>(grid, s, sc, cam, colors, sin, sout, pixels, w, h, r0, r1, first, ns,
                                                  cnt);
    return launch<DL, false, GEO, DUAL>(grid, s, sc, cam, colors, sin, sout, pixels, w, h, r0, r1, first, ns, cnt);
}

template <int GEO>
int launch_mode(bool dl, int cmode, const Shape &grid, hipStream_t s, const spt_scene &sc, const rt_camera &cam,
                float *colors, const uint32_t *sin, uint32_t *sout, uint32_t *pixels, int w, int h,
                int r0, int r1, int first, int ns, unsigned long long *cnt)
{
    // The two-query iteration for path tracing in single-light scenes, at
    // every launch shape: one iteration per lit DIFF vertex instead of two.
    // Once the one-query kernel's copies were gone (hit aliasing ray.o, path
    // state reset at sample end) it fits 72 VGPRs at occupancy 7 and beats
    // the one-query form both where per-wave ILP is short (N = 8 band) and on
    // the full frame (17.98 -> 17.3 ms).  RT_SPT_DUAL=0 / 1 forces it off / on (A/B).
    // (The hierarchy walks keep the one-query form: their two resumable
    // walks in one loop spill)
    const int dual_env = getenv("RT_SPT_DUAL") ? atoi(getenv("RT_SPT_DUAL")) : -1;
    const bool dual_ok = dual_env != 0;
    if (dl)
        return launch_counted<GEO, true, false>(cmode, grid, s, sc, cam, colors, sin, sout, pixels, w, h, r0, r1,
                                                first, ns, cnt);
    if constexpr (GEO != rt::smallpt::GEO_BVH && GEO != rt::smallpt::GEO_WIDE) {
        if (sc.nlights == 1 && dual_ok)
            return launch_counted<GEO, false, true>(cmode, grid, s, sc, cam, colors, sin, sout, pixels, w, h, r0, r1,
                                                    first, ns, cnt);
    }
    return launch_counted<GEO, false, false>(cmode, grid, s, sc, cam, colors, sin, sout, pixels, w, h, r0, r1, first,
                                             ns, cnt);
}

// ---- hierarchy build (host, spt_bvh.h) for scenes of >= sptbvh::MIN_SPHERES spheres
// Builds the hierarchy into sc->d_bvh / sc->bvh (nothing for small scenes):
// the binary tree's eight octant layouts and, when a block's LDS can hold it
// (two blocks of WIDE_WPB waves per CU), the 8-wide layout -- with the
// smallest leaf size in {8, 12, 16} whose tree fits.
int build_scene_bvh(spt_scene *sc, const rt_sphere *spheres)
{
    const int n = sc->n;
    if (n < sptbvh::MIN_SPHERES || getenv("RT_SPT_NO_BVH")) return RT_OK;
    std::vector<int> always;
    sptbvh::BvhBuild b;
    sptbvh::partition_and_build(spheres, n, always, b);
    const int nn = (int)b.nodes.size(), nb = (int)b.idx.size(), na = (int)always.size();
    // Eight layouts (one per direction octant), each with layout-local links.
    std::vector<sptbvh::f4> nodes;
    nodes.reserve(2 * (size_t)nn * 8);
    for (int oct = 0; oct < 8; oct++) {
        std::vector<sptbvh::f4> lay;
        lay.reserve(2 * (size_t)nn);
        if (nn) b.emit(0, oct, lay);
        nodes.insert(nodes.end(), lay.begin(), lay.end());
    }
    sptbvh::WideBuild wb;
    bool wide = false;
    const char *we = getenv("RT_SPT_WIDE");             // 0: the binary walk only (A/B, tests)
    if (nn && !(we && atoi(we) == 0)) {
        for (int lm : {8, 12, 16}) {    // (leaves of <= 5 or 6: slower, profiles/r03/c4_leaf_size_ab.log)
            wb.leaf_max = lm;
            wb.build(b);
            if (wide_lds_bytes(wb.nnodes, wb.depth, WIDE_WPB) <= WIDE_LDS_MAX) { wide = true; break; }
        }
    }
    std::vector<float4> geo(nb + na);
    std::vector<int> ids(nb + na);
    for (int j = 0; j < nb + na; j++) {
        const int i = j < nb ? b.idx[j] : always[j - nb];
        const rt_sphere &q = spheres[i];
        geo[j] = make_float4(q.p.x, q.p.y, q.p.z, q.rad * q.rad);     // geomfunc.h:42 product
        ids[j] = i;
    }
    const size_t nb_bytes = sizeof(float4) * nodes.size(), g_bytes = sizeof(float4) * geo.size(),
                 i_bytes = sizeof(int) * ids.size(), w_bytes = wide ? 4 * wb.words.size() : 0,
                 m_bytes = wide ? 4 * wb.maxid.size() : 0;
    const size_t w_off = (nb_bytes + g_bytes + i_bytes + 15) & ~(size_t)15;
    hipError_t e = hipMalloc(&sc->d_bvh, w_off + w_bytes + m_bytes + 16);
    char *base = (char *)sc->d_bvh;
    if (e == hipSuccess) e = hipMemcpy(base, nodes.data(), nb_bytes, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(base + nb_bytes, geo.data(), g_bytes, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(base + nb_bytes + g_bytes, ids.data(), i_bytes, hipMemcpyHostToDevice);
    if (e == hipSuccess && wide) e = hipMemcpy(base + w_off, wb.words.data(), w_bytes, hipMemcpyHostToDevice);
    if (e == hipSuccess && wide)
        e = hipMemcpy(base + w_off + w_bytes, wb.maxid.data(), m_bytes, hipMemcpyHostToDevice);
    if (e == hipSuccess && wide) e = hipMalloc(&sc->d_work, 4 * sizeof(int) * spt_scene::NWORK);
    if (e != hipSuccess) return rtrt::fail_hip(e, "spt_scene_create hierarchy upload");
    rt::smallpt::BvhView &v = sc->bvh;
    v.node = (const float4 *)base;
    v.geo = (const float4 *)(base + nb_bytes);
    v.id = (const int *)(base + nb_bytes + g_bytes);
    v.ageo = v.geo + nb;
    v.aid = v.id + nb;
    v.nalways = na;
    v.nnodes = nn;
    v.wnode = wide ? (const uint4 *)(base + w_off) : nullptr;
    v.wmax = wide ? (const uint4 *)(base + w_off + w_bytes) : nullptr;
    v.wnodes = wide ? wb.nnodes : 0;
    v.wdepth = wide ? wb.depth : 0;
    return RT_OK;
}

int check_render_args(const rt_camera *camera, float *d_colors, const uint32_t *d_seeds_in,
                      uint32_t *d_seeds_out, uint32_t *d_pixels, int w, int h, int row_begin, int row_end,
                      int first_sample, int nsamples, int mode)
{
    if (!camera || !d_colors || !d_seeds_in || !d_seeds_out || !d_pixels)
        return rtrt::fail(RT_ERR_INVALID, "spt render: null pointer");
    if (w < 1 || h < 1 || first_sample < 0 || nsamples < 0)
        return rtrt::fail(RT_ERR_INVALID, "spt render: bad sizes");
    if (row_begin < 0 || row_end > h || row_begin > row_end)
        return rtrt::fail(RT_ERR_INVALID, "spt render: bad row range");
    const int base = mode & ~(SPT_COUNT_RAYS | SPT_COST_MAX);
    if (base != SPT_PATH_TRACING && base != SPT_DIRECT_LIGHTING)
        return rtrt::fail(RT_ERR_INVALID, "spt render: bad mode");
    return RT_OK;
}

}  // namespace

extern "C" int spt_scene_create(const rt_sphere *spheres, unsigned nspheres, spt_scene **out)
{
    if (!spheres || !out || nspheres < 1 || nspheres > (1u << 24))
        return rtrt::fail(RT_ERR_INVALID, "spt_scene_create: bad arguments");
    rtrt::DeviceState *st;
    int rc = rtrt::state(&st);
    if (rc) return rc;
    spt_scene *sc = new spt_scene();
    sc->device = st->device;
    if (st->cus > 0) sc->cus = st->cus;
    sc->n = (int)nspheres;
    sc->host.assign(spheres, spheres + nspheres);
    const char *geo_env = getenv("RT_SPT_GEO");
    sc->force_global = geo_env && !strcmp(geo_env, "global");
    const int n = sc->n;
    std::vector<float4> soa((size_t)3 * n);
    std::vector<int> lights;
    for (int i = 0; i < n; i++) {
        const rt_sphere &q = spheres[i];
        soa[i] = make_float4(q.p.x, q.p.y, q.p.z, q.rad * q.rad);
        int refl = q.refl;
        float frefl;
        memcpy(&frefl, &refl, 4);
        soa[n + i] = make_float4(q.e.x, q.e.y, q.e.z, frefl);
        soa[2 * (size_t)n + i] = make_float4(q.c.x, q.c.y, q.c.z, q.rad);
        if (!((q.e.x == 0.f) && (q.e.x == 0.f) && (q.e.z == 0.f))) lights.push_back(i);  // vec.h:44
    }
    sc->nlights = (int)lights.size();
    // render_kernel's branch order (geomfunc.h:223-281): an emitter (the
    // viszero test of vec.h:44, x tested twice) ends the path, then refl ==
    // DIFF, refl == SPEC, and EVERY other refl value takes the REFR branch
    // (:281 `else`) -- refl 2, but also 3 or -1.  Only a scene whose every
    // non-emitter is DIFF or SPEC may skip the refraction terms.
    sc->no_refr = std::all_of(spheres, spheres + nspheres, [](const rt_sphere &q) {
        const bool emitter = !((q.e.x == 0.f) && (q.e.x == 0.f) && (q.e.z == 0.f));
        return emitter || q.refl == 0 || q.refl == 1;
    });
    if (lights.empty())                    // one zero record (render_kernel loads light 0 unconditionally)
        soa.insert(soa.end(), 3, make_float4(0.f, 0.f, 0.f, 0.f));
    for (int i : lights) {                 // light records: geo, col, emi of each light, ascending
        const float4 g = soa[i], c = soa[2 * (size_t)n + i], e = soa[(size_t)n + i];
        soa.push_back(g);
        soa.push_back(c);
        soa.push_back(e);
    }
    hipError_t e = hipMalloc(&sc->d_spheres, sizeof(rt_sphere) * n);
    if (e == hipSuccess) e = hipMalloc(&sc->d_soa, sizeof(float4) * soa.size());
    if (e == hipSuccess) e = hipMemcpy(sc->d_spheres, spheres, sizeof(rt_sphere) * n, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(sc->d_soa, soa.data(), sizeof(float4) * soa.size(), hipMemcpyHostToDevice);
    if (e != hipSuccess) {
        if (sc->d_spheres) (void)hipFree(sc->d_spheres);
        if (sc->d_soa) (void)hipFree(sc->d_soa);
        delete sc;
        return rtrt::fail_hip(e, "spt_scene_create upload");
    }
    if ((rc = build_scene_bvh(sc, spheres))) {
        spt_scene_destroy(sc);
        return rc;
    }
    *out = sc;
    return RT_OK;
}

extern "C" int spt_scene_destroy(spt_scene *sc)
{
    if (!sc) return RT_OK;
    (void)hipSetDevice(sc->device);
    (void)hipDeviceSynchronize();
    if (sc->d_spheres) (void)hipFree(sc->d_spheres);
    if (sc->d_soa) (void)hipFree(sc->d_soa);
    if (sc->d_bvh) (void)hipFree(sc->d_bvh);
    if (sc->d_work) (void)hipFree(sc->d_work);
    for (SptSched *qp : {&sc->sched, &sc->sched_cnt}) {
        SptSched &q = *qp;
        if (q.d_cost) (void)hipFree(q.d_cost);
        if (q.d_order) (void)hipFree(q.d_order);
        for (int *p : q.retired) (void)hipFree(p);
        if (q.h_cost) (void)hipHostFree(q.h_cost);
        if (q.h_order) (void)hipHostFree(q.h_order);
        if (q.ev) (void)hipEventDestroy(q.ev);
    }
    delete sc;
    return RT_OK;
}

extern "C" int spt_scene_release_captures(const spt_scene *sc)
{
    if (!sc) return rtrt::fail(RT_ERR_INVALID, "spt_scene_release_captures: null scene");
    std::lock_guard<std::mutex> lk(sc->work_mu);
    sc->work_captured = 0;
    return RT_OK;
}

namespace {
// Adaptive order (SptSched) for one launch: sets g.order / g.cost; returns
// true if the caller must queue the cost read-back after the launch.
bool sched_before(const spt_scene &sc, Shape &g, hipStream_t s, int w, int h, int r0, int r1, int gstride,
                  int ns, int mode, const rt_camera &cam, bool full_count)
{
    const char *e = getenv("RT_SPT_SCHED");
    if (!sc.bvh.node || (e && atoi(e) == 0)) return false;   // the full-scan kernels have no order/cost code
    // Full-counter launches learn and use an order of their own: their
    // shadow walks seek the highest-index occluder (twice the uncounted
    // walk's work, unevenly over the tiles), so their tile costs would order
    // the uncounted launches wrongly (configs[4]: 28.0 ms with such an order,
    // 25.4 ms with the uncounted kernel's own) -- and the uncounted order is
    // not theirs either (counted 44.7 ms with it, 52.9 ms with none).
    SptSched &q = full_count ? sc.sched_cnt : sc.sched;
    const int nslots = g.nslots;
    if (!(q.w == w && q.h == h && q.r0 == r0 && q.r1 == r1 && q.gstride == gstride && q.ns == ns &&
          q.mode == mode && q.nslots == nslots && memcmp(&q.cam, &cam, sizeof(cam)) == 0)) {
        q.w = w; q.h = h; q.r0 = r0; q.r1 = r1; q.gstride = gstride; q.ns = ns; q.mode = mode;
        q.nslots = nslots; q.cam = cam;
        q.state = 0;
    }
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(s, &cs) != hipSuccess || cs != hipStreamCaptureStatusNone) {
        if (q.state == 2) {                            // a device pointer, kept alive and unchanged from now on
            g.order = q.d_order;
            q.order_captured = true;
        }
        return false;
    }
    if (nslots > q.cap) {                               // grow (the old buffers may still be read)
        if (q.ev && hipEventSynchronize(q.ev) != hipSuccess) return false;
        if (hipStreamSynchronize(s) != hipSuccess) return false;
        if (q.d_cost) (void)hipFree(q.d_cost);
        if (q.d_order && q.order_captured) q.retired.push_back(q.d_order);
        else if (q.d_order) (void)hipFree(q.d_order);
        q.order_captured = false;
        if (q.h_cost) (void)hipHostFree(q.h_cost);
        if (q.h_order) (void)hipHostFree(q.h_order);
        q.d_cost = q.h_cost = nullptr;
        q.d_order = q.h_order = nullptr;
        q.cap = 0;
        if (hipMalloc(&q.d_cost, sizeof(unsigned) * nslots) != hipSuccess ||
            hipMalloc(&q.d_order, sizeof(int) * nslots) != hipSuccess ||
            hipHostMalloc(&q.h_cost, sizeof(unsigned) * nslots) != hipSuccess ||
            hipHostMalloc(&q.h_order, sizeof(int) * nslots) != hipSuccess)
            return false;                               // plain launches (the frees above are safe)
        if (!q.ev && hipEventCreateWithFlags(&q.ev, hipEventDisableTiming) != hipSuccess) return false;
        q.cap = nslots;
        q.state = 0;
    }
    if (q.state == 1 && hipEventQuery(q.ev) == hipSuccess) {
        // heaviest first; ties (and the groups past the window: no tiles, 0)
        // in slot order
        std::vector<int> idx(nslots);
        for (int i = 0; i < nslots; i++) idx[i] = i;
        std::stable_sort(idx.begin(), idx.end(), [&](int a, int b) { return q.h_cost[a] > q.h_cost[b]; });
        memcpy(q.h_order, idx.data(), sizeof(int) * nslots);
        if (q.order_captured) {                        // a graph reads the old order: keep it, take a new buffer
            int *fresh = nullptr;
            if (hipMalloc(&fresh, sizeof(int) * q.cap) != hipSuccess) return false;
            q.retired.push_back(q.d_order);
            q.d_order = fresh;
            q.order_captured = false;
        }
        if (hipMemcpyAsync(q.d_order, q.h_order, sizeof(int) * nslots, hipMemcpyHostToDevice, s) != hipSuccess)
            return false;
        q.state = 2;
    }
    if (q.state == 2) {
        g.order = q.d_order;
        return false;
    }
    if (q.state == 0) {
        if (hipMemsetAsync(q.d_cost, 0, sizeof(unsigned) * nslots, s) != hipSuccess) return false;
        g.cost = q.d_cost;
        // The order key is a group's longest tile (its slowest pixel chain),
        // not the sum of its four: the heavy-tile treatment (cooperative or
        // routed tiles) goes to the first groups in order, and a group with
        // one very long tile outranks four middling ones (configs[4] N = 4
        // interleaved windows 17.1 -> 16.3 ms; the full frame level).
        g.cost_max = true;
        return true;
    }
    return false;                                       // state 1, read-back in flight: plain launch
}

void sched_after(const spt_scene &sc, hipStream_t s, bool full_count)
{
    SptSched &q = full_count ? sc.sched_cnt : sc.sched;
    if (hipMemcpyAsync(q.h_cost, q.d_cost, sizeof(unsigned) * q.nslots, hipMemcpyDeviceToHost, s) == hipSuccess &&
        hipEventRecord(q.ev, s) == hipSuccess)
        q.state = 1;
}

// One launch of rows [row_begin, row_end) (every gstride-th 8-row group), or
// (d_list) of the caller's nlist tile groups over the whole frame.
int scene_render(const spt_scene *sc, const rt_camera *camera, float *d_colors, const uint32_t *d_seeds_in,
                 uint32_t *d_seeds_out, uint32_t *d_pixels, int w, int h, int row_begin, int row_end, int gstride,
                 int first_sample, int nsamples, int mode, uint64_t *d_counters, void *stream,
                 const int *d_list = nullptr, int nlist = 0, unsigned *d_cost = nullptr)
{
    if (row_begin >= row_end || (d_list && nlist < 1)) return RT_OK;
    Shape grid = launch_shape(*sc, w, row_begin, row_end, gstride, d_list ? nlist : 0);
    hipStream_t s = (hipStream_t)stream;
    const int base = mode & ~(SPT_COUNT_RAYS | SPT_COST_MAX);
    bool record = false;
    if (d_list) {
        // The caller's order, heaviest first: its first groups get the
        // heavy-tile treatment (cooperative or routed tiles)
        // as with a learnt order -- unless the launch records costs
        // (d_cost): the list is then taken as unordered and every tile runs
        // a lane per pixel, so the recorded costs compare like with like.
        grid.order = d_list;
        grid.cost = sc->bvh.node ? d_cost : nullptr;
        grid.cost_max = (mode & SPT_COST_MAX) != 0;
        grid.tiers = d_cost == nullptr;
    } else {
        record = sched_before(*sc, grid, s, w, h, row_begin, row_end, gstride, nsamples, base, *camera,
                              d_counters && !(mode & SPT_COUNT_RAYS));
    }
    unsigned long long *cnt = (unsigned long long *)d_counters;
    const bool dl = base == SPT_DIRECT_LIGHTING;
    const int cmode = !cnt ? CNT_NONE : (mode & SPT_COUNT_RAYS) ? CNT_RAYS : CNT_FULL;
    int rc;
    if (sc->bvh.wnode)
        rc = launch_mode<rt::smallpt::GEO_WIDE>(dl, cmode, grid, s, *sc, *camera, d_colors, d_seeds_in, d_seeds_out,
                                                d_pixels, w, h, row_begin, row_end, first_sample, nsamples, cnt);
    else if (sc->bvh.node)
        rc = launch_mode<rt::smallpt::GEO_BVH>(dl, cmode, grid, s, *sc, *camera, d_colors, d_seeds_in, d_seeds_out,
                                               d_pixels, w, h, row_begin, row_end, first_sample, nsamples, cnt);
    else if ((size_t)(3 * sc->n + 3 * std::max(sc->nlights, 1)) * sizeof(float4) <=
                 (size_t)rt::smallpt::MAX_LDS_BYTES &&
             !sc->force_global)
        rc = launch_mode<rt::smallpt::GEO_LDS>(dl, cmode, grid, s, *sc, *camera, d_colors, d_seeds_in, d_seeds_out,
                                               d_pixels, w, h, row_begin, row_end, first_sample, nsamples, cnt);
    else
        rc = launch_mode<rt::smallpt::GEO_GLOBAL>(dl, cmode, grid, s, *sc, *camera, d_colors, d_seeds_in,
                                                  d_seeds_out, d_pixels, w, h, row_begin, row_end, first_sample,
                                                  nsamples, cnt);
    if (rc == RT_OK) rc = rtrt::check_launch("spt render_kernel");
    if (rc == RT_OK && record) sched_after(*sc, s, cmode == CNT_FULL);
    return rc;
}
}  // namespace

extern "C" int spt_scene_render_async(const spt_scene *sc, const rt_camera *camera, float *d_colors,
                                      const uint32_t *d_seeds_in, uint32_t *d_seeds_out, uint32_t *d_pixels,
                                      int w, int h, int row_begin, int row_end, int first_sample,
                                      int nsamples, int mode, uint64_t *d_counters, void *stream)
{
    if (!sc) return rtrt::fail(RT_ERR_INVALID, "spt_scene_render_async: null scene");
    int rc = check_render_args(camera, d_colors, d_seeds_in, d_seeds_out, d_pixels, w, h, row_begin,
                               row_end, first_sample, nsamples, mode);
    if (rc) return rc;
    return scene_render(sc, camera, d_colors, d_seeds_in, d_seeds_out, d_pixels, w, h, row_begin, row_end, 1,
                        first_sample, nsamples, mode, d_counters, stream);
}

extern "C" int spt_scene_render_groups_async(const spt_scene *sc, const rt_camera *camera, float *d_colors,
                                             const uint32_t *d_seeds_in, uint32_t *d_seeds_out, uint32_t *d_pixels,
                                             int w, int h, int group, int ngroups, int first_sample, int nsamples,
                                             int mode, uint64_t *d_counters, void *stream)
{
    if (!sc) return rtrt::fail(RT_ERR_INVALID, "spt_scene_render_groups_async: null scene");
    if (ngroups < 1 || group < 0 || group >= ngroups)
        return rtrt::fail(RT_ERR_INVALID, "spt_scene_render_groups_async: need 0 <= group < ngroups");
    int rc = check_render_args(camera, d_colors, d_seeds_in, d_seeds_out, d_pixels, w, h, 0, h, first_sample,
                               nsamples, mode);
    if (rc) return rc;
    return scene_render(sc, camera, d_colors, d_seeds_in, d_seeds_out, d_pixels, w, h, 8 * group, h, ngroups,
                        first_sample, nsamples, mode, d_counters, stream);
}

extern "C" int spt_group_count(int w, int h)
{
    if (w < 1 || h < 1) return rtrt::fail(RT_ERR_INVALID, "spt_group_count: bad size");
    const long long n = ((long long)((w + 7) / 8) * ((h + 7) / 8) + 3) / 4;
    if (n > (1LL << 28)) return rtrt::fail(RT_ERR_INVALID, "spt_group_count: frame too large");
    return (int)n;
}

extern "C" int spt_scene_render_list_async(const spt_scene *sc, const rt_camera *camera, float *d_colors,
                                           const uint32_t *d_seeds_in, uint32_t *d_seeds_out, uint32_t *d_pixels,
                                           int w, int h, const int *d_groups, int ngroups, int first_sample,
                                           int nsamples, int mode, uint64_t *d_counters, unsigned *d_group_cost,
                                           void *stream)
{
    if (!sc) return rtrt::fail(RT_ERR_INVALID, "spt_scene_render_list_async: null scene");
    const int total = spt_group_count(w, h);
    if (total < 0) return total;
    if (ngroups < 0 || ngroups > total || (ngroups > 0 && !d_groups))
        return rtrt::fail(RT_ERR_INVALID, "spt_scene_render_list_async: need 0 <= ngroups <= spt_group_count(w, h)");
    const bool is_set = (mode & SPT_LIST_SET) != 0;
    mode &= ~SPT_LIST_SET;
    int rc = check_render_args(camera, d_colors, d_seeds_in, d_seeds_out, d_pixels, w, h, 0, h, first_sample,
                               nsamples, mode);
    if (rc || ngroups == 0) return rc;
    if (is_set)                           // (the caller's promise: no dedup pass)
        return scene_render(sc, camera, d_colors, d_seeds_in, d_seeds_out, d_pixels, w, h, 0, h, 1, first_sample,
                            nsamples, mode, d_counters, stream, d_groups, ngroups, d_group_cost);
    // The list as a set (list_dedup_kernel): repeated entries render once.
    // Stream-ordered scratch (graph-capturable): ngroups entries + the claim bits.
    hipStream_t s = (hipStream_t)stream;
    const size_t bits = sizeof(unsigned) * (size_t)((total + 31) / 32);
    char *scratch = nullptr;
    hipError_t e = hipMallocAsync((void **)&scratch, sizeof(int) * (size_t)ngroups + bits, s);
    if (e == hipSuccess) e = hipMemsetAsync(scratch + sizeof(int) * (size_t)ngroups, 0, bits, s);
    if (e != hipSuccess) return rtrt::fail_hip(e, "spt_scene_render_list_async scratch");
    int *d_set = (int *)scratch;
    const unsigned blocks = (unsigned)std::min((ngroups + 255) / 256, 1024);
    hipLaunchKernelGGL(rt::smallpt::list_dedup_kernel, dim3(blocks), dim3(256), 0, s, d_groups, ngroups, total,
                       (unsigned *)(scratch + sizeof(int) * (size_t)ngroups), d_set);
    rc = rtrt::check_launch("spt list_dedup_kernel");
    if (rc == RT_OK)
        rc = scene_render(sc, camera, d_colors, d_seeds_in, d_seeds_out, d_pixels, w, h, 0, h, 1, first_sample,
                          nsamples, mode, d_counters, stream, d_set, ngroups, d_group_cost);
    e = hipFreeAsync(scratch, s);
    if (rc == RT_OK && e != hipSuccess) rc = rtrt::fail_hip(e, "spt_scene_render_list_async scratch free");
    return rc;
}

namespace {
int groups_copy(bool pack, float *d_colors, int w, int h, const int *d_groups, int n, float *d_buf, void *stream)
{
    const int total = spt_group_count(w, h);
    if (total < 0) return total;
    if (!d_colors || !d_buf || n < 0 || n > total || (n > 0 && !d_groups))
        return rtrt::fail(RT_ERR_INVALID, "spt_groups_pack/unpack: bad arguments");
    if (n == 0) return RT_OK;
    const size_t ne = (size_t)n * rt::smallpt::GROUP_FLOATS;
    const unsigned blocks = (unsigned)std::min<size_t>((ne + 255) / 256, 8192);
    if (pack)
        hipLaunchKernelGGL(rt::smallpt::groups_copy_kernel<true>, dim3(blocks), dim3(256), 0, (hipStream_t)stream,
                           d_colors, w, h, d_groups, n, d_buf);
    else
        hipLaunchKernelGGL(rt::smallpt::groups_copy_kernel<false>, dim3(blocks), dim3(256), 0, (hipStream_t)stream,
                           d_colors, w, h, d_groups, n, d_buf);
    return rtrt::check_launch("spt groups_copy_kernel");
}
}  // namespace

extern "C" int spt_groups_pack_async(const float *d_colors, int w, int h, const int *d_groups, int ngroups,
                                     float *d_out, void *stream)
{
    return groups_copy(true, (float *)d_colors, w, h, d_groups, ngroups, d_out, stream);
}

extern "C" int spt_groups_unpack_async(float *d_colors, int w, int h, const int *d_groups, int ngroups,
                                       const float *d_in, void *stream)
{
    return groups_copy(false, d_colors, w, h, d_groups, ngroups, (float *)d_in, stream);
}

namespace {
// One prepared scene per device for the entry points that take a bare sphere
// array (spt_render, spt_render_async), reused while the array is unchanged
// (compared byte for byte): a progressive loop calling them once per pass no
// longer re-uploads the scene, rebuilds its hierarchy (>= 256 spheres) and
// synchronises the device to free it on every call.
struct SceneCache {
    std::vector<rt_sphere> host;
    std::string hooks;                // the preparation's test hooks (RT_SPT_NO_BVH, RT_SPT_GEO, RT_SPT_WIDE[_LEAF])
    spt_scene *sc = nullptr;
};
SceneCache g_scene_cache[64];

}  // namespace

namespace rtrt {
std::string scene_prep_hooks()
{
    std::string h;
    for (const char *k : {"RT_SPT_NO_BVH", "RT_SPT_GEO", "RT_SPT_WIDE"}) {
        const char *v = getenv(k);
        h += v ? v : "-";
        h += "|";
    }
    return h;
}
}  // namespace rtrt

namespace {
// Caller holds the device state's lock.
int cached_scene(const rtrt::DeviceState &st, const rt_sphere *spheres, unsigned n, spt_scene **out)
{
    SceneCache &c = g_scene_cache[st.device];
    const std::string hooks = rtrt::scene_prep_hooks();
    if (c.sc && c.host.size() == n && c.hooks == hooks &&
        memcmp(c.host.data(), spheres, sizeof(rt_sphere) * n) == 0) {
        *out = c.sc;
        return RT_OK;
    }
    if (c.sc) {
        spt_scene_destroy(c.sc);          // waits for the frames that use it
        c.sc = nullptr;
        c.host.clear();
    }
    int rc = spt_scene_create(spheres, n, &c.sc);
    if (rc) {
        c.sc = nullptr;
        return rc;
    }
    c.host.assign(spheres, spheres + n);
    c.hooks = hooks;
    *out = c.sc;
    return RT_OK;
}
}  // namespace

namespace rtrt {
// Under each device state's lock, the one cached_scene's callers hold: a
// render on another thread never sees a destroyed cached scene.
void release_cached_scenes()
{
    for (int d = 0; d < 64; d++) {
        SceneCache &c = g_scene_cache[d];
        DeviceState *st = nullptr;
        if (c.sc) {
            DeviceScope scope;
            if (scope.select(d) == RT_OK && state(&st) == RT_OK) {
                std::lock_guard<std::recursive_mutex> lk(st->mu);
                if (c.sc) spt_scene_destroy(c.sc);
                c.sc = nullptr;
                c.host.clear();
                continue;
            }
        }
        if (c.sc) spt_scene_destroy(c.sc);
        c.sc = nullptr;
        c.host.clear();
    }
}
}  // namespace rtrt

// Device-pointer-only entry: reads the sphere array back (one sync of
// `stream`) to find or prepare the cached scene, then renders asynchronously.
extern "C" int spt_render_async(const rt_sphere *d_spheres, unsigned nspheres, const rt_camera *camera,
                                float *d_colors, const uint32_t *d_seeds_in, uint32_t *d_seeds_out,
                                uint32_t *d_pixels, int w, int h, int row_begin, int row_end,
                                int first_sample, int nsamples, int mode, uint64_t *d_counters,
                                void *stream)
{
    if (!d_spheres || nspheres < 1 || nspheres > (1u << 24))
        return rtrt::fail(RT_ERR_INVALID, "spt_render_async: bad scene");
    int rc = check_render_args(camera, d_colors, d_seeds_in, d_seeds_out, d_pixels, w, h, row_begin,
                               row_end, first_sample, nsamples, mode);
    if (rc) return rc;
    rtrt::DeviceState *st;
    if ((rc = rtrt::state(&st))) return rc;
    std::lock_guard<std::recursive_mutex> lk(st->mu);
    std::vector<rt_sphere> host(nspheres);
    hipError_t e = hipMemcpyAsync(host.data(), d_spheres, sizeof(rt_sphere) * nspheres, hipMemcpyDeviceToHost,
                                  (hipStream_t)stream);
    if (e == hipSuccess) e = hipStreamSynchronize((hipStream_t)stream);
    if (e != hipSuccess) return rtrt::fail_hip(e, "spt_render_async scene read");
    spt_scene *sc;
    if ((rc = cached_scene(*st, host.data(), nspheres, &sc))) return rc;
    return spt_scene_render_async(sc, camera, d_colors, d_seeds_in, d_seeds_out, d_pixels, w, h, row_begin,
                                  row_end, first_sample, nsamples, mode, d_counters, stream);
}

extern "C" int spt_pack_pixels_async(const float *d_colors, uint32_t *d_pixels, int w, int h, int row_begin,
                                     int row_end, void *stream)
{
    if (!d_colors || !d_pixels || w < 1 || h < 1 || row_begin < 0 || row_end > h || row_begin > row_end)
        return rtrt::fail(RT_ERR_INVALID, "spt_pack_pixels_async: bad arguments");
    const size_t n = (size_t)(row_end - row_begin) * w;
    if (n == 0) return RT_OK;
    const unsigned blocks = (unsigned)std::min<size_t>((n + 255) / 256, 8192);
    hipLaunchKernelGGL(rt::smallpt::pack_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, d_colors, d_pixels,
                       w, h, row_begin, row_end);
    return rtrt::check_launch("spt pack_kernel");
}

#ifdef RT_SPT_PROF
// Tools-only: reads and clears the block profile (18 counters).
extern "C" int spt_prof_read(unsigned long long *out)
{
    hipError_t e = hipMemcpyFromSymbol(out, HIP_SYMBOL(rt::smallpt::g_spt_prof), sizeof(rt::smallpt::g_spt_prof));
    static const unsigned long long zero[2 * rt::smallpt::PB_N] = {};
    if (e == hipSuccess) e = hipMemcpyToSymbol(HIP_SYMBOL(rt::smallpt::g_spt_prof), zero, sizeof(zero));
    return e == hipSuccess ? RT_OK : rtrt::fail_hip(e, "spt_prof_read");
}
#endif

#ifdef RT_SPT_TRACE
// Tools-only: sets the wave-timeline buffer (uint4 per wave of the grid; null: off).
extern "C" int spt_trace_set(void *buf)
{
    uint4 *p = (uint4 *)buf;
    hipError_t e = hipMemcpyToSymbol(HIP_SYMBOL(rt::smallpt::g_spt_trace), &p, sizeof(p));
    return e == hipSuccess ? RT_OK : rtrt::fail_hip(e, "spt_trace_set");
}

// Tools-only: renders only tile group g (-1: all) in later launches.
extern "C" int spt_trace_only_group(int g)
{
    hipError_t e = hipMemcpyToSymbol(HIP_SYMBOL(rt::smallpt::g_spt_only_group), &g, sizeof(g));
    return e == hipSuccess ? RT_OK : rtrt::fail_hip(e, "spt_trace_only_group");
}
#endif

extern "C" int spt_render(const rt_sphere *spheres, unsigned nspheres, const rt_camera *camera,
                          float *colors, uint32_t *seeds, uint32_t *pixels, int w, int h,
                          int first_sample, int nsamples, int mode, uint64_t *counters)
{
    if (!spheres || !camera || !colors || !seeds || !pixels || w < 1 || h < 1 || nspheres < 1)
        return rtrt::fail(RT_ERR_INVALID, "spt_render: bad arguments");
    rtrt::DeviceState *st;
    int rc = rtrt::state(&st);
    if (rc) return rc;
    std::lock_guard<std::recursive_mutex> lk(st->mu);
    const size_t npx = (size_t)w * h;
    void *d_col, *d_seed, *d_px, *d_cnt;
    if ((rc = rtrt::scratch(*st, 1, 3 * sizeof(float) * npx, &d_col))) return rc;
    if ((rc = rtrt::scratch(*st, 2, 2 * sizeof(uint32_t) * npx, &d_seed))) return rc;
    if ((rc = rtrt::scratch(*st, 3, sizeof(uint32_t) * npx, &d_px))) return rc;
    if ((rc = rtrt::scratch(*st, 4, 4 * sizeof(uint64_t), &d_cnt))) return rc;
    spt_scene *sc;
    if ((rc = cached_scene(*st, spheres, nspheres, &sc))) return rc;
    hipStream_t s = st->stream;
    hipError_t e = hipMemcpyAsync(d_seed, seeds, 2 * sizeof(uint32_t) * npx, hipMemcpyHostToDevice, s);
    if (e == hipSuccess && first_sample > 0)
        e = hipMemcpyAsync(d_col, colors, 3 * sizeof(float) * npx, hipMemcpyHostToDevice, s);
    if (e == hipSuccess && counters) e = hipMemsetAsync(d_cnt, 0, 4 * sizeof(uint64_t), s);
    if (e != hipSuccess) return rtrt::fail_hip(e, "spt_render H2D");
    rc = spt_scene_render_async(sc, camera, (float *)d_col, (uint32_t *)d_seed, (uint32_t *)d_seed,
                                (uint32_t *)d_px, w, h, 0, h, first_sample, nsamples, mode,
                                counters ? (uint64_t *)d_cnt : nullptr, s);
    if (rc) return rc;
    e = hipMemcpyAsync(seeds, d_seed, 2 * sizeof(uint32_t) * npx, hipMemcpyDeviceToHost, s);
    if (e == hipSuccess && nsamples > 0) {
        e = hipMemcpyAsync(colors, d_col, 3 * sizeof(float) * npx, hipMemcpyDeviceToHost, s);
        if (e == hipSuccess) e = hipMemcpyAsync(pixels, d_px, sizeof(uint32_t) * npx, hipMemcpyDeviceToHost, s);
    }
    if (e == hipSuccess && counters)
        e = hipMemcpyAsync(counters, d_cnt, 4 * sizeof(uint64_t), hipMemcpyDeviceToHost, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    if (e != hipSuccess) return rtrt::fail_hip(e, "spt_render D2H");
    return RT_OK;
}
