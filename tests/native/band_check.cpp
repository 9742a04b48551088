// CPU check of the multi-GPU row-band layout (csrc/spt_band.h, used by
// spt_multi.hip): for h = 1..300 and N = 1..min(h, 64) bands,
//  * the bands partition the flipped slot rows [0, h), in order;
//  * every non-empty band starts at k B, so rank k's all-gather chunk
//    (send_offset) is exactly where its real rows sit in the full buffer;
//  * every chunk lies inside the padded buffer, and only rows >= h of it are
//    padding (a chunk holds padding only past its band's real rows);
//  * the repack windows each device runs after the gather (repack_windows,
//    the helper spt_multi.hip calls) and the pixel rows its band renders
//    (the flip of its slot rows, derived independently) cover every pixel
//    row exactly once.
// Prints the number of (h, N) cases checked, or the first failure.
#include <stdio.h>
#include <vector>
#include "spt_band.h"

int main()
{
    long cases = 0;
    for (int h = 1; h <= 300; h++)
        for (int n = 1; n <= h && n <= 64; n++) {
            const int w = 1 + (h * 7 + n) % 13;
            const int B = sptband::rows_per_band(h, n);
            if ((long long)B * n < h || (long long)(B - 1) * n >= h) { printf("FAIL B h=%d n=%d\n", h, n); return 1; }
            int next = 0;
            for (int k = 0; k < n; k++) {
                int s0, s1;
                sptband::span(h, n, k, &s0, &s1);
                if (s0 != next || s1 < s0 || s1 > h) { printf("FAIL span h=%d n=%d k=%d\n", h, n, k); return 1; }
                next = s1;
                const size_t off = sptband::send_offset(w, h, n, k), cnt = sptband::gather_count(w, h, n);
                if (off + cnt > sptband::padded_floats(w, h, n)) { printf("FAIL pad h=%d n=%d k=%d\n", h, n, k); return 1; }
                if (s1 > s0 && off != 3 * (size_t)w * s0) { printf("FAIL offset h=%d n=%d k=%d\n", h, n, k); return 1; }
                // chunk rows [off / 3w, off / 3w + B): real rows exactly [s0, s1), the rest >= h
                const int c0 = (int)(off / (3 * (size_t)w));
                for (int r = c0; r < c0 + B; r++) {
                    const bool real = r >= s0 && r < s1;
                    if (real != (r < h)) { printf("FAIL chunk h=%d n=%d k=%d r=%d\n", h, n, k, r); return 1; }
                }
                // repack (the windows spt_multi.hip takes from repack_windows)
                // plus the pixel rows the band renders itself -- smallptCPU.cpp:86's
                // flip of its slot rows [s0, s1), derived here pixel by pixel --
                // cover every pixel row exactly once
                std::vector<int> seen(h, 0);
                int win[2][2];
                sptband::repack_windows(h, s0, s1, win);
                for (const auto &wn : win) {
                    if (wn[0] < 0 || wn[1] > h) { printf("FAIL window h=%d n=%d k=%d\n", h, n, k); return 1; }
                    for (int y = wn[0]; y < wn[1]; y++) seen[y]++;
                }
                for (int slot_row = s0; slot_row < s1; slot_row++) seen[h - 1 - slot_row]++;
                for (int y = 0; y < h; y++)
                    if (seen[y] != 1) { printf("FAIL repack h=%d n=%d k=%d y=%d\n", h, n, k, y); return 1; }
            }
            if (next != h) { printf("FAIL cover h=%d n=%d\n", h, n); return 1; }
            cases++;
        }
    printf("%ld\n", cases);
    return 0;
}
