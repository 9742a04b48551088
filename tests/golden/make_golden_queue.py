"""Adds the Raytracer3.2.03 queue-tracer known answers to
tests/golden/known_answers.json (committed fixture), key "queue3203".

Sources:
  * the reference's own committed output
    /root/reference/Raytracer3.2.03/raytracer/OpenCL Raytracer/test.bmp
    (800 x 600, written by raytracer.c:787 from raytracer_non_kernel's frame):
    its size and SHA-256;
  * oracle/_ref/libref_queue.so -- raytracer_non_OpenCL.c + scene.c +
    bitmap.c compiled unmodified (oracle/Makefile): FNV-1a-64 of the uchar4
    frame at 640x480, 800x600, 1920x1080 from the reference's own scene, and
    the BMP its own write_bmp_file produces at 800x600 (must equal test.bmp);
  * oracle/liboracle.so (the restatement, bit-equal to the above): the work
    counters, which the reference does not count.

Run from the repo root in the build container: python tests/golden/make_golden_queue.py
"""
import ctypes as C
import hashlib
import json
import os
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
import oracle_lib as O  # noqa: E402

REF_BMP = "/root/reference/Raytracer3.2.03/raytracer/OpenCL Raytracer/test.bmp"


def main():
    Q = O.ref_queue_lib()
    assert Q is not None, "build oracle/_ref first (make -C oracle)"
    P = (O.QPrimitive * 64)()
    n = Q.ref_q_scene(P, 64)
    ref = open(REF_BMP, "rb").read()
    out = {"test_bmp": {"bytes": len(ref), "sha256": hashlib.sha256(ref).hexdigest(),
                        "source": "Raytracer3.2.03/raytracer/OpenCL Raytracer/test.bmp"}}
    for w, h in [(640, 480), (800, 600), (1920, 1080)]:
        px = O.ref_queue_render(Q, w, h, P, n)
        _, cnt = O.queue_render(w, h, nthreads=os.cpu_count())
        out["%dx%d" % (w, h)] = {"frame_fnv": O.fnv1a64(px), "counters": cnt}
        if (w, h) == (800, 600):
            with tempfile.TemporaryDirectory() as d:
                path = os.path.join(d, "ours.bmp")
                Q.ref_q_write_bmp(px.ctypes.data, w, h, path.encode())
                mine = open(path, "rb").read()
            assert mine == ref, "the reference build does not reproduce test.bmp"
            out["800x600"]["bmp_sha256"] = hashlib.sha256(mine).hexdigest()
        print(w, h, out["%dx%d" % (w, h)], flush=True)
    path = os.path.join(HERE, "known_answers.json")
    d = json.load(open(path))
    d["queue3203"] = out
    with open(path, "w") as f:
        json.dump(d, f, indent=1, sort_keys=True)
        f.write("\n")


if __name__ == "__main__":
    main()
