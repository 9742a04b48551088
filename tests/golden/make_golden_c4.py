"""Adds BASELINE configs[4] to tests/golden/known_answers.json (committed fixture).

configs[4] = the scene_build_complex 10k-sphere scene (rtamd.scenes.complex10k:
complex.scn's light + ground, then the first 9,998 HyperSphere spheres at
maxDepth 6, complex.scn's camera) at 1920x1080, 64 spp from the initial state
(currentSample 0, AllocateBuffers' glibc rand() seeds).  Rendered by
oracle/_ref/libref_smallpt.so -- the reference's own geomfunc.h core
(full-scan Intersect / IntersectP, geomfunc.h:71-110), compiled unmodified --
one row per work item over host threads.  ~3.3e12 sphere tests: tens of
minutes on the build container's 8 cores.  Rows are checkpointed to an .npz
under /tmp so an interrupted run resumes.

Run from the repo root in the build container:
    python tests/golden/make_golden_c4.py [--threads 8] [--spp 64]
"""
import argparse
import ctypes as C
import json
import os
import sys
import threading
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "se-195-project-ray-tracer_amd"))
import oracle_lib as O  # noqa: E402
import rtamd.scenes as S  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--threads", type=int, default=8)
    ap.add_argument("--spp", type=int, default=64)
    ap.add_argument("--w", type=int, default=1920)
    ap.add_argument("--h", type=int, default=1080)
    ap.add_argument("--rows", type=int, default=0, help="only the first ROWS rows (timing probe)")
    a = ap.parse_args()
    w, h, spp = a.w, a.h, a.spp
    _, R = O.ref_libs()
    spheres, n, cam = S.complex10k()
    S.update_camera(cam, w, h)
    sph = C.cast(spheres, C.POINTER(O.Sphere))
    ocam = O.Camera.from_buffer_copy(bytes(cam))
    key = "%dx%d_%dspp_complex10k" % (w, h, spp)
    ck = "/tmp/golden_c4_%s.npz" % key
    col = np.zeros(3 * w * h, np.float32)
    seeds = S.seeds(w, h)
    px = np.zeros(w * h, np.uint32)
    done = np.zeros(h, bool)
    if os.path.exists(ck) and not a.rows:
        z = np.load(ck)
        col[:], seeds[:], px[:], done[:] = z["col"], z["seeds"], z["px"], z["done"]
    todo = [y for y in range(a.rows or h) if not done[y]]
    lock = threading.Lock()
    t0 = time.time()
    nd = [0]

    def worker():
        while True:
            with lock:
                if not todo:
                    return
                y = todo.pop(0)
            R.ref_smallpt_render(sph, n, C.byref(ocam), col.ctypes.data, seeds.ctypes.data, px.ctypes.data,
                                 w, h, y, y + 1, 0, spp, 0)
            with lock:
                done[y] = True
                nd[0] += 1
                if nd[0] % 16 == 0:
                    print("%d rows %.0fs" % (done.sum(), time.time() - t0), flush=True)
                    if not a.rows:
                        np.savez(ck, col=col, seeds=seeds, px=px, done=done)

    th = [threading.Thread(target=worker) for _ in range(a.threads)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    print("%d rows in %.1fs" % (len(done.nonzero()[0]), time.time() - t0), flush=True)
    if a.rows:
        return
    path = os.path.join(HERE, "known_answers.json")
    ka = json.load(open(path))
    ka["smallpt"][key] = {"colors": O.fnv1a64(col), "pixels": O.fnv1a64(px), "seeds": O.fnv1a64(seeds),
                          "source": "oracle/_ref (reference geomfunc.h core, full scan), make_golden_c4.py"}
    with open(path, "w") as fh:
        json.dump(ka, fh, indent=1, sort_keys=True)
    print(key, ka["smallpt"][key])


if __name__ == "__main__":
    main()
