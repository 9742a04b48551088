// spt_bvh.h -- host-side builders of smallpt's exact-culling sphere
// hierarchies (scenes of >= 256 spheres; the device walks are in smallpt.hip).
// Host-only C++ (no HIP types): smallpt.hip uploads what these build, and
// tests/native/libspt_bvh_check.so runs the same builders on the CPU to check
// their invariants against a scalar restatement of the device walk.
//
// The reference tests every sphere for every ray (smallptgpu-v1.6/
// geomfunc.h:71-110).  A hierarchy only skips spheres whose float
// SphereIntersect distance provably cannot be taken; smallpt.hip's "Skipping
// rule" comment gives the margin argument.  Two layouts are built:
//   * BvhBuild: binned-SAH binary tree (64 bins), leaves of <= 4 spheres, eight
//     depth-first layouts (one per ray-direction octant, near child first)
//     with escape links -- walked stacklessly from global memory;
//   * WideBuild: the same tree collapsed to 8 children per node, child boxes
//     quantised to 8 bits per plane in the node's frame (rounded outward),
//     children placed in slots so that visiting slot p ^ octant for p = 0..7
//     is roughly front-to-back -- small enough to live in LDS (configs[4]:
//     ~60 KB), walked with a short per-lane stack of (node, child mask).
#ifndef SPT_BVH_H
#define SPT_BVH_H

#include <math.h>
#include <stdint.h>
#include <string.h>
#include <algorithm>
#include <vector>
#include "../../include/rt_hip.h"

namespace sptbvh {

struct f4 { float x, y, z, w; };

constexpr float ALPHA_R = 1.f / 64.f;   // margin per unit of a box's half diagonal (smallpt.hip)
constexpr int LEAF = 4;                  // spheres per leaf
constexpr int MIN_SPHERES = 256;         // scenes below this are scanned in full
constexpr int MAX_ALWAYS = 16;           // spheres tested outside the hierarchy (radius > 64 x median)
#ifndef SPT_SAH_BINS
#define SPT_SAH_BINS 64   // binned-SAH bins per axis (16: configs[4] heavy-tile rays visit ~20 % more nodes)
#endif

struct HostNode {
    float lo[3], hi[3];
    int left = -1, right = -1;   // children (inner) ...
    int first = 0, count = 0;    // ... or the leaf's sphere range
    int axis = 0;                // split axis (inner)
    float margin = 0.f;          // ALPHA_R * R + BETA
};

// Binned-SAH binary tree over sphere boxes (host, once per scene).
struct BvhBuild {
    const rt_sphere *sp = nullptr;
    std::vector<int> idx;
    std::vector<HostNode> nodes;

    void box(int i, float *lo, float *hi) const
    {
        const rt_sphere &q = sp[i];
        const float c[3] = {q.p.x, q.p.y, q.p.z};
        for (int k = 0; k < 3; k++) { lo[k] = c[k] - q.rad; hi[k] = c[k] + q.rad; }
    }
    float centre(int i, int k) const { return k == 0 ? sp[i].p.x : (k == 1 ? sp[i].p.y : sp[i].p.z); }
    static float area(const float *lo, const float *hi)
    {
        const float x = hi[0] - lo[0], y = hi[1] - lo[1], z = hi[2] - lo[2];
        return x * y + y * z + z * x;
    }

    int build(int lo, int hi)
    {
        const int me = (int)nodes.size();
        nodes.emplace_back();
        HostNode nd;
        float clo[3] = {1e30f, 1e30f, 1e30f}, chi[3] = {-1e30f, -1e30f, -1e30f};
        for (int k = 0; k < 3; k++) { nd.lo[k] = 1e30f; nd.hi[k] = -1e30f; }
        for (int j = lo; j < hi; j++) {
            float a[3], b[3];
            box(idx[j], a, b);
            for (int k = 0; k < 3; k++) {
                nd.lo[k] = std::min(nd.lo[k], a[k]);
                nd.hi[k] = std::max(nd.hi[k], b[k]);
                clo[k] = std::min(clo[k], centre(idx[j], k));
                chi[k] = std::max(chi[k], centre(idx[j], k));
            }
        }
        // Margin term ALPHA * R + BETA (R = half diagonal); BETA also covers
        // the float rounding of the box corners and tiny absolute scales.
        double d2 = 0, mag = 0;
        for (int k = 0; k < 3; k++) {
            d2 += (double)(nd.hi[k] - nd.lo[k]) * (nd.hi[k] - nd.lo[k]);
            mag = std::max(mag, (double)std::max(fabsf(nd.lo[k]), fabsf(nd.hi[k])));
        }
        nd.margin = (float)(ALPHA_R * 0.5 * sqrt(d2) + 1e-3 + 1e-5 * mag);
        const int n = hi - lo;
        if (n <= LEAF) {
            nd.first = lo;
            nd.count = n;
            nodes[me] = nd;
            return me;
        }
        // SAH over SPT_SAH_BINS centroid bins per axis.
        constexpr int NB = SPT_SAH_BINS;
        int best_ax = -1, best_b = 0;
        float best_cost = 1e30f;
        for (int ax = 0; ax < 3; ax++) {
            const float ext = chi[ax] - clo[ax];
            if (!(ext > 0.f)) continue;
            int cnt[NB] = {};
            float blo[NB][3], bhi[NB][3];
            for (int q = 0; q < NB; q++)
                for (int k = 0; k < 3; k++) { blo[q][k] = 1e30f; bhi[q][k] = -1e30f; }
            for (int j = lo; j < hi; j++) {
                int q = (int)((centre(idx[j], ax) - clo[ax]) / ext * NB);
                q = std::min(std::max(q, 0), NB - 1);
                float a[3], b[3];
                box(idx[j], a, b);
                cnt[q]++;
                for (int k = 0; k < 3; k++) { blo[q][k] = std::min(blo[q][k], a[k]); bhi[q][k] = std::max(bhi[q][k], b[k]); }
            }
            float rlo[NB][3], rhi[NB][3];
            int rc[NB];
            float alo[3] = {1e30f, 1e30f, 1e30f}, ahi[3] = {-1e30f, -1e30f, -1e30f};
            int ac = 0;
            for (int q = NB - 1; q >= 1; q--) {
                for (int k = 0; k < 3; k++) { alo[k] = std::min(alo[k], blo[q][k]); ahi[k] = std::max(ahi[k], bhi[q][k]); }
                ac += cnt[q];
                for (int k = 0; k < 3; k++) { rlo[q][k] = alo[k]; rhi[q][k] = ahi[k]; }
                rc[q] = ac;
            }
            float llo[3] = {1e30f, 1e30f, 1e30f}, lhi[3] = {-1e30f, -1e30f, -1e30f};
            int lc = 0;
            for (int q = 0; q < NB - 1; q++) {
                for (int k = 0; k < 3; k++) { llo[k] = std::min(llo[k], blo[q][k]); lhi[k] = std::max(lhi[k], bhi[q][k]); }
                lc += cnt[q];
                if (lc == 0 || rc[q + 1] == 0) continue;
                const float cost = area(llo, lhi) * lc + area(rlo[q + 1], rhi[q + 1]) * rc[q + 1];
                if (cost < best_cost) { best_cost = cost; best_ax = ax; best_b = q + 1; }
            }
        }
        int mid;
        if (best_ax >= 0) {
            const int ax = best_ax;
            const float ext = chi[ax] - clo[ax];
            auto it = std::partition(idx.begin() + lo, idx.begin() + hi, [&](int i) {
                int q = (int)((centre(i, ax) - clo[ax]) / ext * NB);
                q = std::min(std::max(q, 0), NB - 1);
                return q < best_b;
            });
            mid = (int)(it - idx.begin());
            nd.axis = ax;
        } else {
            mid = lo + n / 2;   // all centres equal: any split
        }
        if (mid == lo || mid == hi) mid = lo + n / 2;
        nd.left = build(lo, mid);
        nd.right = build(mid, hi);
        nodes[me] = nd;
        return me;
    }

    // Depth-first layout for ray-direction octant `oct` (bit k set: d_k < 0):
    // at each inner node the child on the near side of its split axis comes
    // first; link = escape index (inner) or ~(first | count << 24) (leaf).
    void emit(int node, int oct, std::vector<f4> &out) const
    {
        const HostNode &h = nodes[node];
        const size_t me = out.size() / 2;
        out.push_back(f4{0.5f * (h.lo[0] + h.hi[0]), 0.5f * (h.lo[1] + h.hi[1]), 0.5f * (h.lo[2] + h.hi[2]), 0.f});
        out.push_back(f4{0.5f * (h.hi[0] - h.lo[0]), 0.5f * (h.hi[1] - h.lo[1]), 0.5f * (h.hi[2] - h.lo[2]), h.margin});
        int link;
        if (h.left < 0) {
            link = ~(h.first | (h.count << 24));
        } else {
            const HostNode &L = nodes[h.left], &R = nodes[h.right];
            const bool l_low = L.lo[h.axis] + L.hi[h.axis] <= R.lo[h.axis] + R.hi[h.axis];
            const bool neg = (oct >> h.axis) & 1;
            const int c0 = (l_low != neg) ? h.left : h.right;
            emit(c0, oct, out);
            emit(c0 == h.left ? h.right : h.left, oct, out);
            link = (int)(out.size() / 2);                   // escape: the node after this subtree
        }
        float f;
        memcpy(&f, &link, 4);
        out[2 * me].w = f;
    }
};

// Splits a scene into the "always" spheres (radius > 64 x the median: the
// ground of configs[4]) and the rest, and builds the binary tree over the rest.
inline void partition_and_build(const rt_sphere *spheres, int n, std::vector<int> &always, BvhBuild &b)
{
    std::vector<float> rads(n);
    for (int i = 0; i < n; i++) rads[i] = spheres[i].rad;
    std::nth_element(rads.begin(), rads.begin() + n / 2, rads.end());
    const float med = rads[n / 2];
    std::vector<int> rest;
    always.clear();
    for (int i = 0; i < n; i++) {
        if (spheres[i].rad > 64.f * med && (int)always.size() < MAX_ALWAYS) always.push_back(i);
        else rest.push_back(i);
    }
    b.sp = spheres;
    b.idx = rest;
    b.nodes.clear();
    if (!rest.empty()) b.build(0, (int)rest.size());
}

// ---------------------------------------------------------------------------
// 8-wide layout.  One node = 28 words (112 B, seven 16-B reads):
//   w0..2  p: the quantisation origin (the node box's low corner), float
//   w3     biased exponents e_x | e_y << 8 | e_z << 16 (scale 2^(e - 127) per
//          axis) | valid-slot mask << 24
//   w4     D0: the node box's diagonal length (|o - p| + D0 bounds the distance
//          from a ray origin o to any point of the box), float
//   w5     K: max over the children of their ALPHA_R * R + BETA margin term
//   w6..7  0
//   w8..15 child word per slot: >= 0 a wide node, < 0 a leaf ~(first | count << 24)
//   w16..27 child boxes, one byte per slot, four slots per word: words
//          16 + 6h .. 21 + 6h hold qlo_x, qlo_y, qlo_z, qhi_x, qhi_y, qhi_z of
//          slots 4h .. 4h + 3 (slot s = byte s & 3); the child box is
//          [p + qlo 2^e, p + qhi 2^e] per axis,
//          which contains the binary tree's box for that child (rounded
//          outward, checked in long double).
// Slot order: slot s holds the child most "behind" the direction octant s
// (sign bit k of s set: d_k < 0), chosen greedily; a ray of octant o visits
// slot p ^ o at position p.
constexpr int WIDE = 8, WIDE_WORDS = 28;

struct WideBuild {
    std::vector<uint32_t> words;
    int nnodes = 0, depth = 0;          // depth: levels of wide nodes (the stack needs depth - 1 entries)
    int leaf_max = LEAF;                // binary subtrees of <= leaf_max spheres become one leaf child
    // Per node and slot the highest reference index under that child (8
    // words per node, 0 for empty slots): the counted any-hit walk, which
    // must find the highest occluder (IntersectP's early-exit position),
    // skips children that cannot hold a higher one.
    std::vector<uint32_t> maxid;
    std::vector<int> cnt, mx;           // spheres / highest reference index under each binary node
    int count(const BvhBuild &b, int r)
    {
        const HostNode &h = b.nodes[r];
        if (h.left < 0) {
            int m = -1;
            for (int j = 0; j < h.count; j++) m = std::max(m, b.idx[h.first + j]);
            mx[r] = m;
            return cnt[r] = h.count;
        }
        const int c = count(b, h.left) + count(b, h.right);
        mx[r] = std::max(mx[h.left], mx[h.right]);
        return cnt[r] = c;
    }
    bool is_leaf(const BvhBuild &b, int r) const { return b.nodes[r].left < 0 || cnt[r] <= leaf_max; }
    int first(const BvhBuild &b, int r) const { return b.nodes[r].left < 0 ? b.nodes[r].first : first(b, b.nodes[r].left); }

    static uint32_t fbits(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }

    // Children of binary node r after collapsing: up to 8 binary nodes.
    void collapse(const BvhBuild &b, int r, std::vector<int> &kids) const
    {
        kids.clear();
        const HostNode &h = b.nodes[r];
        if (is_leaf(b, r)) { kids.push_back(r); return; }   // a leaf root: one leaf child
        kids.push_back(h.left);
        kids.push_back(h.right);
        while ((int)kids.size() < WIDE) {
            int best = -1;
            float ba = -1.f;
            for (int i = 0; i < (int)kids.size(); i++) {
                const HostNode &c = b.nodes[kids[i]];
                if (is_leaf(b, kids[i])) continue;
                const float a = BvhBuild::area(c.lo, c.hi);
                if (a > ba) { ba = a; best = i; }
            }
            if (best < 0) break;
            const HostNode &c = b.nodes[kids[best]];
            kids[best] = c.left;
            kids.push_back(c.right);
        }
    }

    int emit(const BvhBuild &b, int r, int level)
    {
        depth = std::max(depth, level + 1);
        const int me = nnodes++;
        words.resize((size_t)nnodes * WIDE_WORDS, 0u);
        maxid.resize((size_t)nnodes * WIDE, 0u);
        std::vector<int> kids;
        collapse(b, r, kids);
        const int nk = (int)kids.size();
        // node box, centroid
        float lo[3] = {1e30f, 1e30f, 1e30f}, hi[3] = {-1e30f, -1e30f, -1e30f};
        float K = 0.f;
        for (int c : kids)
            for (int k = 0; k < 3; k++) {
                lo[k] = std::min(lo[k], b.nodes[c].lo[k]);
                hi[k] = std::max(hi[k], b.nodes[c].hi[k]);
            }
        for (int c : kids) K = std::max(K, b.nodes[c].margin);
        // greedy slot assignment: cost(child, slot) = dot(centroid - C, dir(slot))
        double C[3];
        for (int k = 0; k < 3; k++) C[k] = 0.5 * ((double)lo[k] + hi[k]);
        int slot_of[WIDE], child_in[WIDE];
        for (int s = 0; s < WIDE; s++) { slot_of[s] = -1; child_in[s] = -1; }
        std::vector<std::pair<double, int>> cost;
        for (int i = 0; i < nk; i++) {
            const HostNode &c = b.nodes[kids[i]];
            for (int s = 0; s < WIDE; s++) {
                double d = 0;
                for (int k = 0; k < 3; k++)
                    d += (0.5 * ((double)c.lo[k] + c.hi[k]) - C[k]) * (((s >> k) & 1) ? -1.0 : 1.0);
                cost.push_back({d, i * WIDE + s});
            }
        }
        std::stable_sort(cost.begin(), cost.end(),
                         [](const std::pair<double, int> &a, const std::pair<double, int> &c) { return a.first < c.first; });
        for (auto &e : cost) {
            const int i = e.second / WIDE, s = e.second % WIDE;
            if (slot_of[i] < 0 && child_in[s] < 0) { slot_of[i] = s; child_in[s] = i; }
        }
        // quantisation frame
        int eb[3];
        for (int k = 0; k < 3; k++) {
            const double ext = (double)hi[k] - (double)lo[k];
            int e = -126;
            while (e < 127 && ldexp(255.0, e) < ext) e++;
            eb[k] = e;
        }
        uint32_t valid = 0;
        uint8_t q[6][WIDE];
        memset(q, 0, sizeof(q));
        for (int s = 0; s < WIDE; s++) { q[0][s] = q[1][s] = q[2][s] = 255; }   // empty slots: inverted (masked anyway)
        for (int s = 0; s < WIDE; s++) {
            const int i = child_in[s];
            if (i < 0) continue;
            valid |= 1u << s;
            const HostNode &c = b.nodes[kids[i]];
            for (int k = 0; k < 3; k++) {
                const long double sc = ldexpl(1.0L, eb[k]);
                long double ql = floorl(((long double)c.lo[k] - (long double)lo[k]) / sc);
                long double qh = ceill(((long double)c.hi[k] - (long double)lo[k]) / sc);
                ql = std::max(0.0L, std::min(255.0L, ql));
                qh = std::max(0.0L, std::min(255.0L, qh));
                while (ql > 0 && (long double)lo[k] + ql * sc > (long double)c.lo[k]) ql -= 1;
                while (qh < 255 && (long double)lo[k] + qh * sc < (long double)c.hi[k]) qh += 1;
                q[k][s] = (uint8_t)ql;
                q[3 + k][s] = (uint8_t)qh;
            }
        }
        double d2 = 0;
        for (int k = 0; k < 3; k++) d2 += ((double)hi[k] - lo[k]) * ((double)hi[k] - lo[k]);
        const float D0 = (float)(sqrt(d2) * (1.0 + 1e-6));
        int child[WIDE] = {};
        for (int s = 0; s < WIDE; s++) {
            const int i = child_in[s];
            if (i < 0) continue;
            const HostNode &c = b.nodes[kids[i]];
            child[s] = is_leaf(b, kids[i]) ? ~(first(b, kids[i]) | (cnt[kids[i]] << 24)) : emit(b, kids[i], level + 1);
            (void)c;
        }
        uint32_t *w = &words[(size_t)me * WIDE_WORDS];
        w[0] = fbits(lo[0]); w[1] = fbits(lo[1]); w[2] = fbits(lo[2]);
        w[3] = (uint32_t)(eb[0] + 127) | ((uint32_t)(eb[1] + 127) << 8) | ((uint32_t)(eb[2] + 127) << 16) | (valid << 24);
        w[4] = fbits(D0);
        w[5] = fbits(K);
        for (int s = 0; s < WIDE; s++) w[8 + s] = (uint32_t)child[s];
        for (int a = 0; a < 6; a++)
            for (int s = 0; s < WIDE; s++) w[16 + 6 * (s >> 2) + a] |= (uint32_t)q[a][s] << (8 * (s & 3));
        for (int s = 0; s < WIDE; s++)
            if (child_in[s] >= 0) maxid[(size_t)me * WIDE + s] = (uint32_t)mx[kids[child_in[s]]];
        return me;
    }

    void build(const BvhBuild &b)
    {
        words.clear();
        maxid.clear();
        nnodes = depth = 0;
        cnt.assign(b.nodes.size(), 0);
        mx.assign(b.nodes.size(), -1);
        if (!b.nodes.empty()) {
            count(b, 0);
            emit(b, 0, 0);
        }
    }
};

}  // namespace sptbvh

#endif
