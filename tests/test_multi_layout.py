"""CPU check of the multi-GPU row-band arithmetic (csrc/spt_band.h) that
spt_multi.hip's bands, its in-place ncclAllGather offsets and its repack
windows use: tests/native/band_check.cpp over every h <= 300 and N <= 64
bands, ragged h and N > h/2 (trailing empty bands) included."""
import os
import subprocess

NATIVE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "native")


def test_band_layout_arithmetic():
    subprocess.run(["make", "-s", "-C", NATIVE, "band_check"], check=True)
    out = subprocess.run([os.path.join(NATIVE, "band_check")], capture_output=True, text=True)
    assert out.returncode == 0, out.stdout + out.stderr
    assert int(out.stdout.split()[-1]) == sum(min(h, 64) for h in range(1, 301))


def test_band_layout_examples():
    """h = 9, N = 8: B = 2, bands 0..3 two rows, band 4 one, bands 5..7
    empty (their all-gather chunks are padding); 1080 / 8 = 135 rows each."""
    import re
    src = open(os.path.join(os.path.dirname(NATIVE), "..", "se-195-project-ray-tracer_amd", "csrc",
                            "spt_band.h")).read()
    assert re.search(r"rows_per_band\(int h, int n\) \{ return \(h \+ n - 1\) / n; \}", src)

    def span(h, n, k):
        B = (h + n - 1) // n
        return min(h, k * B), min(h, (k + 1) * B)
    assert [span(9, 8, k) for k in range(8)] == [(0, 2), (2, 4), (4, 6), (6, 8), (8, 9), (9, 9), (9, 9), (9, 9)]
    assert [span(1080, 8, k)[1] - span(1080, 8, k)[0] for k in range(8)] == [135] * 8
