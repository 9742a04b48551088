"""CPU checks of the 8-wide hierarchy (csrc/spt_bvh.h WideBuild) through a
scalar restatement of smallpt.hip's wide walk (tests/native/spt_bvh_check.cpp):
for every ray, the walk's nearest hit (distance bits and sphere index, ties to
the highest index) or any-hit occluder (the highest index, as the counted
kernel reports IntersectP's position) equals the reference's full scan
(smallptgpu-v1.6/geomfunc.h:71-110), and the stack never exceeds the depth
the kernel reserves.  The GPU tests compare the kernels themselves."""
import ctypes as C
import os
import subprocess

import numpy as np
import pytest

NATIVE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "native")


@pytest.fixture(scope="module")
def chk():
    subprocess.run(["make", "-s", "-C", NATIVE, "libspt_bvh_check.so"], check=True)
    L = C.CDLL(os.path.join(NATIVE, "libspt_bvh_check.so"))
    P = C.c_void_p
    L.spt_bvh_wide_check.restype = C.c_longlong
    L.spt_bvh_wide_check.argtypes = [P, C.c_int, P, P, C.c_longlong, P, P, P, P, P]
    L.spt_bvh_wide_stats.argtypes = [P, C.c_int, P]
    L.spt_bvh_set_leaf_max.argtypes = [C.c_int]
    return L


@pytest.fixture(scope="module")
def rt():
    """The host layer's scene data only (no device needed)."""
    import rtamd
    return rtamd


def _rays(rng, centres, origin, nr, spread):
    o = centres[rng.integers(0, len(centres), nr)] + rng.normal(0, spread, (nr, 3))
    o[: nr // 8] = origin
    d = rng.normal(0, 1, (nr, 3))
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    d[: nr // 16, 1] = 0.0                          # axis-parallel components (the 1e-30 clamp)
    d[: nr // 16] /= np.linalg.norm(d[: nr // 16], axis=1, keepdims=True)
    return np.ascontiguousarray(np.concatenate([o, d], 1).astype(np.float32))


def _check(chk, S, n, rays, leaf_max):
    chk.spt_bvh_set_leaf_max(leaf_max)
    nr = len(rays)
    tw, ts = np.zeros(nr, np.float32), np.zeros(nr, np.float32)
    iw, is_ = np.zeros(nr, np.int32), np.zeros(nr, np.int32)
    v = C.c_longlong()
    bad = chk.spt_bvh_wide_check(C.addressof(S), n, rays.ctypes.data, None, nr, tw.ctypes.data, iw.ctypes.data,
                                 ts.ctypes.data, is_.ctypes.data, C.addressof(v))
    assert bad == 0 and (iw >= -1).all()
    maxt = np.where(is_ >= 0, ts * np.float32(1.5), np.float32(50.0)).astype(np.float32)
    bad = chk.spt_bvh_wide_check(C.addressof(S), n, rays.ctypes.data, maxt.ctypes.data, nr, tw.ctypes.data,
                                 iw.ctypes.data, ts.ctypes.data, is_.ctypes.data, None)
    assert bad == 0 and (iw >= -1).all()
    return v.value / nr


@pytest.mark.parametrize("leaf_max", [4, 8, 16])
def test_wide_walk_equals_full_scan_configs4(chk, rt, leaf_max):
    S, n, cam = rt.scenes.complex10k()
    sp = np.ctypeslib.as_array(C.cast(S, C.POINTER(C.c_float)), shape=(n * 11,)).reshape(n, 11)
    rays = _rays(np.random.default_rng(leaf_max), sp[2:, 1:4], (20.0, 80.0, 150.0), 6000, 5.0)
    visits = _check(chk, S, n, rays, leaf_max)
    assert visits < 12                                # ~7 wide nodes per ray (~15 binary ones)
    out = (C.c_longlong * 5)()
    chk.spt_bvh_wide_stats(C.addressof(S), n, out)
    if leaf_max == 8:                                 # the layout the kernel stages in LDS
        assert out[4] <= 64 * 1024 and out[2] <= 8


@pytest.mark.parametrize("seed,far", [(1, 0), (2, 0), (3, 3000), (4, 20000)])
def test_wide_walk_equals_full_scan_random_clouds(chk, rt, seed, far):
    """Tiny, overlapping and far spheres, a huge ground sphere; origins in
    and around the cloud, or far away (the widest absolute margins)."""
    rng = np.random.default_rng(seed)
    n = 3000
    S = (rt.Sphere * n)()
    rt.scenes._sphere(S[0], 1e4, (0.0, -1e4 - 20.0, 0.0), (0, 0, 0), (0.7, 0.7, 0.7), 0)
    rt.scenes._sphere(S[1], 3.0, (0.0, 40.0, 0.0), (20, 20, 20), (0, 0, 0), 0)
    cen = rng.uniform(-30, 30, (n, 3))
    for i in range(2, n):
        rt.scenes._sphere(S[i], 10.0 ** rng.uniform(-2.5, 0.5), tuple(cen[i]), (0, 0, 0), (0.5, 0.5, 0.5), 0)
    origin = (0.3 * far, 0.2 * far, far) if far else (1.0, 2.0, 25.0)
    rays = _rays(rng, cen[2:], origin, 4000, 3.0)
    if far:                                           # far origins aimed at the cloud
        k = len(rays) // 2
        tgt = cen[rng.integers(2, n, k)] + rng.normal(0, 1, (k, 3))
        d = tgt - np.array(origin)
        rays[:k, :3] = origin
        rays[:k, 3:] = d / np.linalg.norm(d, axis=1, keepdims=True)
    for lm in (4, 8):
        _check(chk, S, n, rays, lm)
