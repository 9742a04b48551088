// spt_band.h -- the row-band layout of a smallpt frame tiled over N devices
// (spt_multi.hip; include/rt_hip.h spt_multi_bands), host-only arithmetic
// shared with the CPU check tests/native/band_check.cpp.
//
// Band k owns the flipped colour / seed slot rows [s0, s1) (pixel rows
// [h - s1, h - s0), smallptCPU.cpp:86's slot (h-y-1)*w+x).  Every band is
// B = ceil(h / N) rows in the all-gather's padded buffer (N * B colour rows);
// band k's real rows are the part of [k B, (k + 1) B) below h, so a ragged h
// leaves the last band short and may leave trailing bands empty (h = 9,
// N = 8: B = 2, bands 5..7 empty) -- their all-gather chunks are padding,
// and the repack reads rows [0, h) only.
#ifndef SPT_BAND_H
#define SPT_BAND_H

#include <stddef.h>

namespace sptband {

inline int rows_per_band(int h, int n) { return (h + n - 1) / n; }

// Band k's flipped slot rows [*s0, *s1).
inline void span(int h, int n, int k, int *s0, int *s1)
{
    const int B = rows_per_band(h, n);
    const long long a = (long long)k * B, b = (long long)(k + 1) * B;
    *s0 = (int)(a < h ? a : h);
    *s1 = (int)(b < h ? b : h);
}

// Floats one rank sends in the in-place all-gather, and where rank k's chunk
// starts in the padded colour buffer (3 floats per pixel).
inline size_t gather_count(int w, int h, int n) { return 3 * (size_t)w * rows_per_band(h, n); }
inline size_t send_offset(int w, int h, int n, int k) { return (size_t)k * gather_count(w, h, n); }
// Colour floats of the padded buffer (N * B rows).
inline size_t padded_floats(int w, int h, int n) { return (size_t)n * gather_count(w, h, n); }

// The pixel-row windows a band's device repacks after the gather -- every
// row it did not render: win[0] = [win[0][0], win[0][1]) below its own pixel
// rows [h - s1, h - s0), win[1] above them (either may be empty).
inline void repack_windows(int h, int s0, int s1, int win[2][2])
{
    win[0][0] = 0;
    win[0][1] = h - s1;
    win[1][0] = h - s0;
    win[1][1] = h;
}

}  // namespace sptband

#endif
