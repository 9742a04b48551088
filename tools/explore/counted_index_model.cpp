// tools/explore/counted_index_model.cpp -- CPU model (tools only): work per
// counted shadow query (IntersectP's early-exit position = the highest-index
// occluder) of (a) the current counted walk over the spatial 8-wide tree
// (tests/native/spt_bvh_check.cpp's restatement, max-index pruning) against
// (b) an index-ordered binary hierarchy: nodes cover contiguous index
// ranges, the walk visits the higher range first and tests a leaf's spheres
// in descending index, so its first occluder IS the answer.  Boxes exact
// (float), grown by a relative margin; counts only (not an exactness check).
//   g++ -O2 -std=c++17 -ffp-contract=off -shared -fPIC -I se-195-project-ray-tracer_amd/csrc \
//       -o /tmp/libcim.so tools/explore/counted_index_model.cpp
#include <math.h>
#include <algorithm>
#include <vector>
#include "spt_bvh.h"

namespace {
constexpr float EPS = 0.01f;
float hit(const rt_sphere &s, const float *o, const float *d)
{
    const float opx = s.p.x - o[0], opy = s.p.y - o[1], opz = s.p.z - o[2];
    const float b = opx * d[0] + opy * d[1] + opz * d[2];
    float det = b * b - (opx * opx + opy * opy + opz * opz) + s.rad * s.rad;
    if (det < 0.f) return INFINITY;
    det = sqrtf(det);
    float t = b - det;
    if (t > EPS) return t;
    t = b + det;
    return t > EPS ? t : INFINITY;
}
struct Node { float lo[3], hi[3]; int a, b, left, right; };   // index range [a, b); leaf: left < 0
struct IdxTree {
    const rt_sphere *sp;
    std::vector<Node> nodes;
    int leaf;
    int build(int a, int b)
    {
        Node n;
        for (int k = 0; k < 3; k++) { n.lo[k] = INFINITY; n.hi[k] = -INFINITY; }
        for (int i = a; i < b; i++) {
            const float c[3] = {sp[i].p.x, sp[i].p.y, sp[i].p.z};
            for (int k = 0; k < 3; k++) {
                n.lo[k] = std::min(n.lo[k], c[k] - sp[i].rad);
                n.hi[k] = std::max(n.hi[k], c[k] + sp[i].rad);
            }
        }
        n.a = a; n.b = b; n.left = n.right = -1;
        const int id = (int)nodes.size();
        nodes.push_back(n);
        if (b - a > leaf) {
            const int m = (a + b) / 2;
            const int l = build(a, m), r = build(m, b);
            nodes[id].left = l;
            nodes[id].right = r;
        }
        return id;
    }
};
bool box_hit(const Node &n, const float *o, const float *inv, float maxt, float rel)
{
    float tn = 0.f, tf = maxt;
    for (int k = 0; k < 3; k++) {
        const float g = rel * (n.hi[k] - n.lo[k] + fabsf(o[k]) + 1.f);
        const float t1 = (n.lo[k] - g - o[k]) * inv[k], t2 = (n.hi[k] + g - o[k]) * inv[k];
        tn = std::max(tn, std::min(t1, t2));
        tf = std::min(tf, std::max(t1, t2));
    }
    return tn <= tf;
}
// highest-index occluder, descending; counts nodes and sphere tests
int idx_anyhit(const IdxTree &T, int nd, const float *o, const float *d, const float *inv, float maxt,
               long long &nodes, long long &tests)
{
    const Node &n = T.nodes[nd];
    nodes++;
    if (!box_hit(n, o, inv, maxt, 1e-3f)) return -1;
    if (n.left < 0) {
        for (int i = n.b - 1; i >= n.a; i--) {
            tests++;
            if (hit(T.sp[i], o, d) < maxt) return i;
        }
        return -1;
    }
    const int r = idx_anyhit(T, n.right, o, d, inv, maxt, nodes, tests);
    if (r >= 0) return r;
    return idx_anyhit(T, n.left, o, d, inv, maxt, nodes, tests);
}
}  // namespace

extern "C" {
// rays (o, d) x nr with maxt; out: [0] mismatches vs the full scan, [1] nodes, [2] sphere tests of (b)
long long cim_run(const rt_sphere *sp, int n, const float *rays, const float *maxt, long long nr, int leaf,
                  int nskip_low, long long *out)
{
    IdxTree T;
    T.sp = sp;
    T.leaf = leaf;
    // spheres [0, nskip_low) (the light and ground: the "always" ones) are
    // tested last, below the tree, as their indices are the lowest
    T.build(nskip_low, n);
    long long bad = 0, nodes = 0, tests = 0;
    for (long long r = 0; r < nr; r++) {
        const float *o = rays + 6 * r, *d = o + 3;
        float inv[3];
        for (int k = 0; k < 3; k++) inv[k] = 1.f / (fabsf(d[k]) < 1e-30f ? copysignf(1e-30f, d[k]) : d[k]);
        int id = idx_anyhit(T, 0, o, d, inv, maxt[r], nodes, tests);
        if (id < 0) {
            for (int i = nskip_low - 1; i >= 0; i--) {
                tests++;
                if (hit(sp[i], o, d) < maxt[r]) { id = i; break; }
            }
        }
        int ref = -1;
        for (int i = n - 1; i >= 0; i--)
            if (hit(sp[i], o, d) < maxt[r]) { ref = i; break; }
        if (ref != id) bad++;
    }
    out[0] = bad; out[1] = nodes; out[2] = tests;
    return bad;
}
}
