"""PPM writers of the two reference apps, byte for byte, for frames rendered
through this package (host-side formatting; the reference apps keep their own).

* smallpt_ppm: the 'p' key handler of smallptgpu-v1.6/displayfunc.cpp
  (keyFunc, case 'p'): "P3\\n<W> <H>\\n255\\n", rows bottom-up, each pixel
  "<R> <G> <B> " from the RGBA8 word's bytes 0,1,2, no line breaks.
* whitted_ppm: DrawWindow of raytracer3.0.06.no_rec.samp/testapp.cpp:180-199:
  header "P3\\n800 600\\n255\\n" (the reference hard-codes 800x600; here the
  frame's size, identical at 800x600), rows top-down, GetPixelColor
  (testapp.cpp:50-54: R = bits 16-23, G = 8-15, B = 0-7), "<R> <G> <B> ", a
  newline after every column c with c % 5 == 0 and after every row.
"""
import numpy as np


def _triples(r, g, b):
    return np.char.add(np.char.add(np.char.add(np.char.add(r.astype(str), " "), np.char.add(g.astype(str), " ")),
                                   b.astype(str)), " ")


def smallpt_ppm(pixels, w, h):
    """bytes of image.ppm for smallpt's pixels (uint32 [h*w], row y at y*w)."""
    px = np.asarray(pixels, dtype=np.uint32).reshape(h, w)[::-1]
    t = _triples(px & 0xff, (px >> 8) & 0xff, (px >> 16) & 0xff)
    return ("P3\n%d %d\n%d\n" % (w, h, 255)).encode() + "".join(t.ravel().tolist()).encode()


def whitted_ppm(frame):
    """bytes of output<N>.ppm for a Whitted XRGB frame (uint32 [h, w])."""
    f = np.asarray(frame, dtype=np.uint32)
    h, w = f.shape
    t = _triples((f >> 16) & 0xff, (f >> 8) & 0xff, f & 0xff)
    brk = np.where(np.arange(w) % 5 == 0, "\n", "")
    rows = ["".join(np.char.add(t[r], brk).tolist()) + "\n" for r in range(h)]
    return ("P3\n%d %d\n255\n" % (w, h)).encode() + "".join(rows).encode()


def write(path, data):
    with open(path, "wb") as f:
        f.write(data)
