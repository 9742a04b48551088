"""Generates tests/golden/known_answers.json (committed fixture).

Sources, in order of authority:
  * SURVEY.md §8(c)/§6 [probe] figures measured on the reference itself:
    Whitted ray / test counts, TIR count, spot pixels, the smallpt camera basis.
  * oracle/_ref/libref_smallpt.so -- the reference's own smallpt radiance
    core (geomfunc.h/simplernd.h/vec.h/scene.h compiled unmodified): FNV-1a-64
    hashes of colours / pixels / seeds after k samples.
  * oracle/liboracle.so (C restatement) for the Whitted frames: raytracer.cpp
    needs <windows.h> and is not built (DESIGN.md "Parity pins"); the hashes
    are recorded so the GPU path is checked at full size without the oracle.

Run from the repo root in the build container (needs /root/reference-built
oracle/_ref):  python tests/golden/make_golden.py
"""
import ctypes as C
import json
import os
import sys
import time
from concurrent.futures import ThreadPoolExecutor

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
import oracle_lib as O  # noqa: E402

SURVEY = {
    "whitted_counts": {  # [traced, shadow, Primitive_Intersect calls] SURVEY.md §6
        "640x480": [4353070, 17375668, 230765796],
        "1920x1080": [31325673, 125055504, 1683118331],
    },
    "whitted_tir_events_640x480": 1874,            # SURVEY.md §7 (all TIR events)
    "whitted_pixel_400_300": {"640x480": 0xccaaaa, "800x600": 0xf1f1f1, "1920x1080": 0xffc4c4},
    "smallpt_camera_1024x768": {"dir": [0.0, -0.0425715372, -0.999093413],
                                "x": [1.04719758, 0.0, 0.0],
                                "y": [0.0, 0.784686148, -0.0334356092]},
}


def ref_smallpt(w, h, spp, mode=0, threads=8):
    """Reference-built smallpt (oracle/_ref) over row bands on host threads."""
    _, S = O.ref_libs()
    sph = (O.Sphere * 9)()
    n = S.ref_cornell(sph, 9)
    cam = O.cornell_camera(w, h)
    col = np.zeros(3 * w * h, np.float32)
    seeds = O.seeds(w, h)
    px = np.zeros(w * h, np.uint32)
    bands = np.linspace(0, h, threads * 4 + 1).astype(int)

    def run(k):
        S.ref_smallpt_render(sph, n, C.byref(cam), col.ctypes.data, seeds.ctypes.data, px.ctypes.data,
                             w, h, int(bands[k]), int(bands[k + 1]), 0, spp, mode)

    with ThreadPoolExecutor(threads) as ex:
        list(ex.map(run, range(len(bands) - 1)))
    return {"colors": O.fnv1a64(col), "pixels": O.fnv1a64(px), "seeds": O.fnv1a64(seeds),
            "source": "oracle/_ref (reference geomfunc.h core)"}


def main():
    out = {"survey": SURVEY, "whitted": {}, "smallpt": {}}
    for w, h in [(640, 480), (800, 600), (1920, 1080)]:
        f, c = O.whitted_render(w, h, nthreads=8)
        out["whitted"]["%dx%d" % (w, h)] = {"xrgb": O.fnv1a64(f), "counters": c,
                                            "source": "oracle (restatement; pinned by survey counts)"}
    cases = [(640, 480, 1, 0), (640, 480, 4, 0), (320, 240, 2, 1), (1024, 768, 64, 0),
             (1920, 1080, 64, 0), (1920, 1080, 256, 0)]
    for w, h, spp, mode in cases:
        t0 = time.time()
        key = "%dx%d_%dspp%s" % (w, h, spp, "_dl" if mode else "")
        out["smallpt"][key] = ref_smallpt(w, h, spp, mode)
        print(key, out["smallpt"][key], "%.1fs" % (time.time() - t0), flush=True)
    with open(os.path.join(HERE, "known_answers.json"), "w") as fh:
        json.dump(out, fh, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
