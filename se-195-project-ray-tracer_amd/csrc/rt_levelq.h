// rt_levelq.h -- segmented work queues of the level-synchronous ray-tree passes
// (whitted.hip: raytracer3.0.06's Engine_Render; queue.hip: Raytracer3.2.03's
// raytracer_non_kernel).
//
// A level's queue is split into NSEG segments with their own counters (a
// producing wave appends to segment wave_id mod NSEG, so thousands of waves
// finishing a step together do not queue on one atomic address); a segment's
// items are laid out in PAGE-slot pages, page c of segment s at
// base + (c * NSEG + s) * PAGE.  The levels of one pass share one record pool:
// level L+1 starts right after level L's last page (next_base), so the pool
// holds the levels' actual item counts, not a per-level worst case.
// Consumers enumerate the pages of a level from a wave-level prefix of the
// segments' lengths (seg_view / seg_chunk): whole waves only.
#ifndef RT_LEVELQ_H
#define RT_LEVELQ_H

#include "rt_common.h"

namespace rt {
namespace lq {

constexpr int NSEG = 64;
constexpr int PAGE = 64;              // slots per page (one segment's)
constexpr int PAGE_ROW = NSEG * PAGE; // one page of every segment
constexpr int CSTRIDE = 32;           // ints between counters: one 128-B line each
                                      // (same-line atomics serialise in the L2)

// Pool slot of item j of segment s of the level based at `base`.
__device__ __forceinline__ int seg_slot(int base, int s, int j)
{
    return base + ((j >> 6) * NSEG + s) * PAGE + (j & (PAGE - 1));
}

// Per-segment item limit of a level based at `base` (the pages left in a pool
// of `pool` slots).
__device__ __forceinline__ int seg_limit(int pool, int base)
{
    return (pool - base) / PAGE_ROW * PAGE;
}

// Wave-aggregated queue allocation: every active lane asks for `want` (0..2)
// items; one atomic per wave.  Returns the lane's first item index.
__device__ __forceinline__ int wave_alloc(int *counter, int want)
{
    const unsigned long long m1 = __builtin_amdgcn_ballot_w64((want & 1) != 0);
    const unsigned long long m2 = __builtin_amdgcn_ballot_w64((want & 2) != 0);
    const int lane = __lane_id();
    const unsigned long long lt = (1ull << lane) - 1ull;
    const int pre = __popcll(m1 & lt) + 2 * __popcll(m2 & lt);
    const int tot = __popcll(m1) + 2 * __popcll(m2);
    const int first = __builtin_ctzll(__builtin_amdgcn_read_exec());
    int base = 0;
    if (lane == first && tot) base = atomicAdd(counter, tot);
    base = __shfl(base, first, 64);
    return base + pre;
}

// Consumer view of a level's segmented queue: lane s holds segment s's length
// (segs[s * CSTRIDE], capped at `limit`) and the inclusive prefix of its page
// counts.
struct SegView { int incl, n, base; };

__device__ __forceinline__ SegView seg_view(const int *segs, int base, int limit)
{
    const int lane = __lane_id();
    SegView v;
    v.base = base;
    v.n = min(segs[lane * CSTRIDE], limit);
    int x = (v.n + PAGE - 1) / PAGE;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const int y = __shfl_up(x, off, 64);
        if (lane >= off) x += y;
    }
    v.incl = x;
    return v;
}

// The pool base after the level: past the last page of its fullest segment.
__device__ __forceinline__ int next_base(const SegView &v)
{
    int p = (v.n + PAGE - 1) / PAGE;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) p = max(p, __shfl_xor(p, off, 64));
    return v.base + p * PAGE_ROW;
}

// Page k (wave-uniform) of the queue: first slot and number of valid items;
// false once k is past the last page.
__device__ __forceinline__ bool seg_chunk(const SegView &v, int k, int &base, int &nvalid)
{
    if (k >= __shfl(v.incl, 63, 64)) return false;
    const int s = __popcll(__builtin_amdgcn_ballot_w64(v.incl <= k));
    const int incl = __shfl(v.incl, s, 64), n = __shfl(v.n, s, 64);
    const int c = k - (incl - ((n + PAGE - 1) / PAGE));
    base = seg_slot(v.base, s, c * PAGE);
    nvalid = min(PAGE, n - c * PAGE);
    return true;
}

}  // namespace lq
}  // namespace rt

#endif
