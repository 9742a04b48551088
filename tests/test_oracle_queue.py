"""The Raytracer3.2.03 queue tracer's oracle and its pins (CPU only).

* oracle/_ref/libref_queue.so is the reference's own raytracer_non_OpenCL.c,
  scene.c and bitmap.c compiled in place; with raytracer.c's main() sequence
  restated it writes the reference's committed test.bmp byte for byte.
* The C restatement (oracle/queue_oracle.c) equals that build bit for bit on
  the reference scene and on random closed-room scenes.
* Without /root/reference (the GPU box) the restatement is checked against
  the committed known answers (tests/golden/make_golden_queue.py).
"""
import hashlib
import json
import os

import numpy as np
import pytest

import oracle_lib as O

HERE = os.path.dirname(os.path.abspath(__file__))
KA = json.load(open(os.path.join(HERE, "golden", "known_answers.json")))["queue3203"]
REF_BMP = "/root/reference/Raytracer3.2.03/raytracer/OpenCL Raytracer/test.bmp"


def _ref():
    Q = O.ref_queue_lib()
    if Q is None:
        pytest.skip("oracle/_ref not built (no /root/reference here)")
    return Q


def test_reference_build_reproduces_test_bmp(tmp_path):
    Q = _ref()
    if not os.path.exists(REF_BMP):
        pytest.skip("reference tree absent")
    P = (O.QPrimitive * 64)()
    n = Q.ref_q_scene(P, 64)
    assert n == 17
    px = O.ref_queue_render(Q, 800, 600, P, n)
    path = str(tmp_path / "test.bmp")
    assert Q.ref_q_write_bmp(px.ctypes.data, 800, 600, path.encode()) == 1
    mine = open(path, "rb").read()
    ref = open(REF_BMP, "rb").read()
    assert mine == ref
    assert hashlib.sha256(ref).hexdigest() == KA["test_bmp"]["sha256"]


def test_oracle_frame_matches_known_answers():
    for key in ("640x480", "800x600"):
        w, h = map(int, key.split("x"))
        px, cnt = O.queue_render(w, h, nthreads=os.cpu_count())
        assert O.fnv1a64(px) == KA[key]["frame_fnv"], key
        assert cnt == KA[key]["counters"], key


def test_oracle_bmp_is_the_reference_test_bmp():
    import rtamd.bmp
    px, _ = O.queue_render(800, 600, nthreads=os.cpu_count())
    data = rtamd.bmp.bmp_bytes(px)
    assert len(data) == KA["test_bmp"]["bytes"] == 1440054
    assert hashlib.sha256(data).hexdigest() == KA["test_bmp"]["sha256"]


def test_scene_matches_reference_scene_fields():
    """Every field the computation reads equals the reference's create_scene
    + copy (the others are uninitialised stack in the reference)."""
    Q = _ref()
    import rtamd
    R = (O.QPrimitive * 64)()
    n = Q.ref_q_scene(R, 64)
    P, m = rtamd.scenes.queue_scene()
    assert n == m == 17
    for i in range(n):
        a, b = R[i], P[i]
        assert a.type == b.type and a.is_light == b.is_light, i
        for f in ("m_refl", "m_diff", "m_refr", "m_refr_index", "m_spec"):
            assert getattr(a, f) == getattr(b, f), (i, f)
        assert (a.m_color.x, a.m_color.y, a.m_color.z) == (b.m_color.x, b.m_color.y, b.m_color.z), i
        if a.type == 1:
            for f in ("radius", "sq_radius", "r_radius"):
                assert getattr(a, f) == getattr(b, f), (i, f)
            assert (a.center.x, a.center.y, a.center.z) == (b.center.x, b.center.y, b.center.z), i
        else:
            assert a.depth == b.depth, i
            assert (a.normal.x, a.normal.y, a.normal.z) == (b.normal.x, b.normal.y, b.normal.z), i


def test_oracle_equals_reference_build_reference_scene():
    Q = _ref()
    R = (O.QPrimitive * 64)()
    n = Q.ref_q_scene(R, 64)               # with the reference's uninitialised fields
    P, m = O.queue_scene()
    for w, h in [(800, 600), (161, 97), (1, 1), (7, 3)]:
        ref = O.ref_queue_render(Q, w, h, R, n)
        ours, cnt = O.queue_render(w, h, P, m, nthreads=os.cpu_count())
        assert (ref == ours).all(), (w, h)
        assert cnt[3] == 0


@pytest.mark.parametrize("seed", range(12))
def test_oracle_equals_reference_build_random_scenes(seed):
    Q = _ref()
    P, n = random_scene(seed)
    ref = O.ref_queue_render(Q, 80, 60, P, n)
    ours, cnt = O.queue_render(80, 60, P, n, nthreads=os.cpu_count())
    assert cnt[3] == 0          # no undefined behaviour in the reference
    assert (ref == ours).all()


def random_scene(seed, w=80, h=60):
    """A random closed-room scene in which no ray of a w x h frame reaches the
    reference's undefined behaviour (re-drawn until the oracle counts none)."""
    rng = np.random.default_rng(1000 + seed)
    while True:
        P, n = O.queue_random_scene(rng, nspheres=int(rng.integers(2, 40)), nlights=int(rng.integers(1, 5)),
                                    nplanes_extra=int(rng.integers(0, 3)))
        if O.queue_render(w, h, P, n, nthreads=os.cpu_count())[1][3] == 0:
            return P, n
