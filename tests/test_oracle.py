"""Pins the oracle (oracle/*.c, the CPU restatement) before it is trusted:
  * against the reference's own sources compiled in oracle/_ref
    (smallpt radiance core; Whitted scene.cpp),
  * against the [probe] figures SURVEY.md records for the reference itself
    (Whitted ray/test/TIR counts, spot pixels, smallpt camera basis),
  * against the committed golden hashes (tests/golden/known_answers.json)."""
import ctypes as C
import json
import os

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = json.load(open(os.path.join(HERE, "golden", "known_answers.json")))


def _ref(oracle):
    libs = oracle.ref_libs()
    if libs is None:
        pytest.skip("oracle/_ref not built (needs /root/reference at build time)")
    return libs


def test_whitted_counts_match_reference_probe(oracle):
    for key, want in GOLD["survey"]["whitted_counts"].items():
        w, h = map(int, key.split("x"))
        f, c = oracle.whitted_render(w, h, nthreads=8)
        assert c[:3] == want, key
        assert int(f[300, 400]) == GOLD["survey"]["whitted_pixel_400_300"][key]


def test_whitted_tir_events_match_reference_probe(oracle):
    # The oracle counts TIR events with a traced child (nodes < 31); the probe
    # counted all of them.  Both are checked through the golden counters.
    f, c = oracle.whitted_render(640, 480, nthreads=8)
    assert c == GOLD["whitted"]["640x480"]["counters"]


@pytest.mark.parametrize("key", ["640x480", "800x600"])
def test_whitted_golden_frames(oracle, key):
    w, h = map(int, key.split("x"))
    f, c = oracle.whitted_render(w, h, nthreads=8)
    assert oracle.fnv1a64(f) == GOLD["whitted"][key]["xrgb"]
    assert c == GOLD["whitted"][key]["counters"]


def test_whitted_scene_matches_reference_scene_cpp(oracle):
    W, _ = _ref(oracle)
    prims, n = oracle.whitted_scene()
    rp = (oracle.Primitive * 50)()
    m = W.ref_whitted_scene(rp, 50)
    assert m == n == 17
    for a, b in zip(prims[:n], rp[:m]):   # plane_cell is uninitialised in the reference
        for f, _t in oracle.Primitive._fields_:
            if f != "plane_cell":
                assert bytes(getattr(a, f)) == bytes(getattr(b, f)) if hasattr(getattr(a, f), "_fields_") \
                    else getattr(a, f) == getattr(b, f), f


def test_whitted_intersect_normal_match_reference(oracle):
    W, _ = _ref(oracle)
    L = oracle.lib()
    prims, n = oracle.whitted_scene()
    rng = np.random.default_rng(7)
    for _ in range(4000):
        o = rng.uniform(-8, 8, 3).astype(np.float32)
        d = rng.normal(size=3).astype(np.float32)
        d /= np.float32(np.linalg.norm(d))
        ray = np.concatenate([o, d]).astype(np.float32)
        for p in range(n):
            d1, d2 = C.c_float(1e6), C.c_float(1e6)
            r1 = L.orw_primitive_intersect(C.byref(prims[p]), ray.ctypes.data, C.byref(d1))
            r2 = W.ref_primitive_intersect(C.byref(prims[p]), ray.ctypes.data, C.byref(d2))
            assert (r1, d1.value) == (r2, d2.value)
            n1, n2 = np.zeros(3, np.float32), np.zeros(3, np.float32)
            L.orw_primitive_normal(C.byref(prims[p]), o.ctypes.data, n1.ctypes.data)
            W.ref_primitive_normal(C.byref(prims[p]), o.ctypes.data, n2.ctypes.data)
            assert (n1.view(np.uint32) == n2.view(np.uint32)).all()


def test_cornell_matches_reference_scene_h(oracle):
    _, S = _ref(oracle)
    a, n = oracle.cornell()
    b = (oracle.Sphere * 9)()
    assert S.ref_cornell(b, 9) == n
    assert bytes(a) == bytes(b)


def test_get_random_matches_reference(oracle):
    _, S = _ref(oracle)
    rng = np.random.default_rng(3)
    for s in rng.integers(2, 2**32, size=(2000, 2), dtype=np.uint64):
        a0, a1 = C.c_uint32(int(s[0])), C.c_uint32(int(s[1]))
        b0, b1 = C.c_uint32(int(s[0])), C.c_uint32(int(s[1]))
        x = oracle.lib().ors_get_random(C.byref(a0), C.byref(a1))
        y = S.ref_get_random(C.byref(b0), C.byref(b1))
        assert (x, a0.value, a1.value) == (y, b0.value, b1.value)


@pytest.mark.parametrize("w,h,steps,mode", [(640, 480, [1], 0), (640, 480, [1, 3], 0), (200, 150, [3], 1)])
def test_smallpt_oracle_matches_reference_core(oracle, w, h, steps, mode):
    _, S = _ref(oracle)
    sph, n = oracle.cornell()
    cam = oracle.cornell_camera(w, h)
    c1, c2 = np.zeros(3 * w * h, np.float32), np.zeros(3 * w * h, np.float32)
    s1 = oracle.seeds(w, h)
    s2 = s1.copy()
    p1, p2 = np.zeros(w * h, np.uint32), np.zeros(w * h, np.uint32)
    first = 0
    for k in steps:
        oracle.smallpt_render(sph, n, cam, c1, s1, p1, w, h, first, k, dl=mode, nthreads=8)
        S.ref_smallpt_render(sph, n, C.byref(cam), c2.ctypes.data, s2.ctypes.data, p2.ctypes.data,
                             w, h, 0, h, first, k, mode)
        first += k
    assert (c1.view(np.uint32) == c2.view(np.uint32)).all()
    assert (s1 == s2).all() and (p1 == p2).all()


@pytest.mark.parametrize("key", ["640x480_1spp", "640x480_4spp", "320x240_2spp_dl"])
def test_smallpt_golden(oracle, key):
    res, spp, *dl = key.split("_")
    w, h = map(int, res.split("x"))
    spp = int(spp[:-3])
    sph, n = oracle.cornell()
    cam = oracle.cornell_camera(w, h)
    col = np.zeros(3 * w * h, np.float32)
    seeds = oracle.seeds(w, h)
    px = np.zeros(w * h, np.uint32)
    oracle.smallpt_render(sph, n, cam, col, seeds, px, w, h, 0, spp, dl=1 if dl else 0, nthreads=8)
    g = GOLD["smallpt"][key]
    assert (oracle.fnv1a64(col), oracle.fnv1a64(px), oracle.fnv1a64(seeds)) == (g["colors"], g["pixels"], g["seeds"])


def test_camera_matches_reference_probe(oracle):
    cam = oracle.cornell_camera(1024, 768)
    want = GOLD["survey"]["smallpt_camera_1024x768"]
    for f in ("dir", "x", "y"):
        v = getattr(cam, f)
        assert np.allclose([v.x, v.y, v.z], want[f], rtol=0, atol=5e-9), f


def test_seeds_are_glibc_rand_stream(oracle):
    s = oracle.seeds(4, 4, 1)
    assert list(s[:4]) == [1804289383, 846930886, 1681692777, 1714636915]
