"""Product-side scene inputs (rtamd.scenes) equal the oracle's / the
reference's data files."""
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
SCN = os.path.join(HERE, "golden", "scenes")


def test_whitted_scene_equals_oracle(oracle):
    import rtamd
    a, n = rtamd.scenes.whitted_scene()
    b, m = oracle.whitted_scene()
    assert n == m == 17 and bytes(a) == bytes(b)[:96 * 17]


def test_cornell_equals_oracle_and_scn_file(oracle):
    import rtamd
    a, n = rtamd.scenes.cornell()
    b, m = oracle.cornell()
    assert bytes(a) == bytes(b)
    c, k, cam = rtamd.scenes.read_scene(os.path.join(SCN, "cornell.scn"))
    assert k == n and bytes(c) == bytes(a)      # scene.h == scenes/cornell.scn
    ref = rtamd.scenes.cornell_camera(640, 480)
    assert bytes(cam)[:24] == bytes(ref)[:24]


def test_cameras_equal_oracle(oracle):
    import rtamd
    for w, h in [(640, 480), (1024, 768), (1920, 1080), (33, 17)]:
        assert bytes(rtamd.scenes.cornell_camera(w, h)) == bytes(oracle.cornell_camera(w, h))


def test_seeds_equal_oracle(oracle):
    import rtamd
    assert (rtamd.scenes.seeds(64, 48) == oracle.seeds(64, 48)).all()


def test_hypersphere_generator_matches_complex_scn(oracle):
    import rtamd
    arr, n, cam = rtamd.scenes.read_scene(os.path.join(SCN, "complex.scn"))
    gen = rtamd.scenes.hypersphere(4.0)
    assert n == 783 and len(gen) == 781
    for s, g in zip(arr[2:], gen):
        assert (s.rad, s.p.x, s.p.y, s.p.z) == tuple(np.float32([g[0], *g[1]]))
        assert (s.c.x, s.c.y, s.c.z, s.refl) == (*np.float32(g[3]), g[4])
    buf, total = oracle.hypersphere(4.0, 1000)
    assert total == 781
    for s, g in zip(buf[:total], arr[2:]):
        assert bytes(s) == bytes(g)


def test_complex10k_config(oracle):
    import rtamd
    arr, n, cam = rtamd.scenes.complex10k()
    assert n == 10000
    assert len(rtamd.scenes.hypersphere(6.0)) == 19531
    buf, total = oracle.hypersphere(6.0, 9998)
    assert total == 19531 and bytes(buf) == bytes(arr)[2 * 44:]
