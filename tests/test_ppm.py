"""PPM output formats of the reference apps (rtamd.ppm) against loop-for-loop
restatements of the C writers (displayfunc.cpp keyFunc 'p';
testapp.cpp:180-199 DrawWindow + :50-54 GetPixelColor)."""
import numpy as np

import rtamd


def _smallpt_c(pixels, w, h):
    out = ["P3\n%d %d\n%d\n" % (w, h, 255)]
    for y in range(h - 1, -1, -1):
        for x in range(w):
            v = int(pixels[y * w + x])
            out.append("%d %d %d " % (v & 0xff, (v >> 8) & 0xff, (v >> 16) & 0xff))
    return "".join(out).encode()


def _whitted_c(frame):
    h, w = frame.shape
    out = ["P3\n%d %d\n255\n" % (w, h)]
    i = 0
    flat = frame.ravel()
    for r in range(h):
        for c in range(w):
            p = int(flat[i])
            out.append("%d %d %d " % ((p & 0x00ff0000) >> 16, (p & 0x0000ff00) >> 8, p & 0xff))
            i += 1
            if c % 5 == 0:
                out.append("\n")
        out.append("\n")
    return "".join(out).encode()


def test_smallpt_ppm_matches_keyfunc_writer():
    rng = np.random.default_rng(3)
    w, h = 13, 7
    px = rng.integers(0, 2**24, size=w * h, dtype=np.uint32)
    assert rtamd.ppm.smallpt_ppm(px, w, h) == _smallpt_c(px, w, h)


def test_whitted_ppm_matches_drawwindow_writer():
    rng = np.random.default_rng(4)
    f = rng.integers(0, 2**24, size=(6, 11), dtype=np.uint32)
    assert rtamd.ppm.whitted_ppm(f) == _whitted_c(f)
    hdr = rtamd.ppm.whitted_ppm(np.zeros((600, 800), np.uint32))[:15]
    assert hdr == b"P3\n800 600\n255\n"      # the reference's hard-coded header at its size
