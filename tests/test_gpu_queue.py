"""GPU parity of the Raytracer3.2.03 queue tracer (rtq_render*) against the
oracle and the reference's own output (test.bmp's SHA-256).  Bar: bit-exact
frames and identical work counters."""
import ctypes as C
import hashlib
import json
import os

import numpy as np
import pytest

import oracle_lib as O
from test_oracle_queue import KA, random_scene

pytestmark = pytest.mark.gpu
NT = min(16, os.cpu_count() or 1)


def test_reference_frame_is_test_bmp(rt):
    import rtamd.bmp
    px, cnt = rt.queue_render(800, 600, counters=True)
    data = rtamd.bmp.bmp_bytes(px)
    assert hashlib.sha256(data).hexdigest() == KA["test_bmp"]["sha256"]
    assert O.fnv1a64(px) == KA["800x600"]["frame_fnv"]
    assert cnt == KA["800x600"]["counters"]


@pytest.mark.parametrize("size", ["640x480", "1920x1080"])
def test_known_answer_frames(rt, size):
    w, h = map(int, size.split("x"))
    px, cnt = rt.queue_render(w, h, counters=True)
    assert O.fnv1a64(px) == KA[size]["frame_fnv"]
    assert cnt == KA[size]["counters"]
    px2 = rt.queue_render(w, h)                       # the uncounted kernels
    assert (px2 == px).all()


@pytest.mark.parametrize("w,h", [(1, 1), (7, 3), (161, 97), (333, 17), (64, 200)])
def test_ragged_sizes(rt, w, h):
    ref, rc = O.queue_render(w, h, nthreads=NT)
    px, cnt = rt.queue_render(w, h, counters=True)
    assert (px == ref).all()
    assert cnt == rc


@pytest.mark.parametrize("seed", range(10))
def test_random_scenes(rt, seed):
    P, n = random_scene(seed, 96, 72)
    ref, rc = O.queue_render(96, 72, P, n, nthreads=NT)
    px, cnt = rt.queue_render(96, 72, P, n, counters=True)
    assert (px == ref).all()
    assert cnt == rc
    assert (rt.queue_render(96, 72, P, n) == ref).all()


def test_max_primitives(rt):
    """MAXP = 64 primitives (the scene image is built a lane per primitive,
    list positions by ballot prefix): lights, spheres and planes shuffled."""
    rng = np.random.default_rng(77)
    while True:
        P, n = O.queue_random_scene(rng, nspheres=52, nlights=4, nplanes_extra=2)
        ref, rc = O.queue_render(64, 48, P, n, nthreads=NT)
        if rc[3] == 0:
            break
    assert n == 64
    px, cnt = rt.queue_render(64, 48, P, n, counters=True)
    assert (px == ref).all()
    assert cnt == rc


def test_single_primitive_scene(rt):
    """One primitive, the reference scene's first wall (open scene: the
    primitives[-1] read is defined and counted identically)."""
    P, n = O.queue_scene()
    ref, rc = O.queue_render(80, 60, P, 1, nthreads=NT)
    px, cnt = rt.queue_render(80, 60, P, 1, counters=True)
    assert (px == ref).all()
    assert cnt == rc


def test_undefined_behaviour_is_counted_and_defined(rt):
    """An open scene (rays escape): the reference reads primitives[-1]; both
    the oracle and the library define it as 'no children' and count it."""
    P, n = O.queue_scene()
    # drop the back, front and top walls: rays leave the room
    keep = [i for i in range(n) if i not in (10, 11, 12)]
    Q = (O.QPrimitive * 64)()
    for k, i in enumerate(keep):
        Q[k] = P[i]
    ref, rc = O.queue_render(120, 90, Q, len(keep), nthreads=NT)
    px, cnt = rt.queue_render(120, 90, Q, len(keep), counters=True)
    assert rc[3] > 0
    assert (px == ref).all() and cnt == rc


@pytest.mark.parametrize("cap", ["4096", "70000"])
def test_pool_overflow_reevaluates_exactly(rt, cap, monkeypatch):
    """A record pool too small for the trees: the trees whose nodes did not
    fit are re-evaluated by final_kernel, with the same frame and counters."""
    monkeypatch.setenv("RT_QUEUE_POOL_CAP", cap)
    ref = KA["800x600"]
    px, cnt = rt.queue_render(800, 600, counters=True)
    assert O.fnv1a64(px) == ref["frame_fnv"]
    assert cnt == ref["counters"]
    P, n = random_scene(3, 96, 72)
    r2, c2 = O.queue_render(96, 72, P, n, nthreads=NT)
    px, cnt = rt.queue_render(96, 72, P, n, counters=True)
    assert (px == r2).all() and cnt == c2


def test_pool_grows_after_overflow(rt, monkeypatch):
    """A first pool far too small (RT_POOL_FRAC): the overflowed frame is
    exact and flags the overflow to the host; the following frames of that
    size get a pool 1.25x larger each time (the arena grows), all exact."""
    monkeypatch.setenv("RT_POOL_FRAC", "0.2")
    w, h = 352, 288                     # a size no other test uses: a fresh pool entry
    ref, rc = O.queue_render(w, h, nthreads=NT)
    rt.lib().rt_release()
    sizes = []
    for _ in range(6):
        px, cnt = rt.queue_render(w, h, counters=True)
        assert (px == ref).all() and cnt == rc
        sizes.append(rt.lib().rt_cached_bytes())
    assert sizes[-1] > sizes[0], sizes


def test_exact_path_everywhere(rt, monkeypatch):
    """RT_QUEUE_EXACT_ALL=1: every specular term is treated as uncertified, so
    nearly every pixel is finished by fix_kernel with glibc's pow restated
    (rtm::pow_d) -- the same frame and counters."""
    monkeypatch.setenv("RT_QUEUE_EXACT_ALL", "1")
    px, cnt = rt.queue_render(800, 600, counters=True)
    assert O.fnv1a64(px) == KA["800x600"]["frame_fnv"]
    assert cnt == KA["800x600"]["counters"]
    P, n = random_scene(5, 96, 72)
    ref, rc = O.queue_render(96, 72, P, n, nthreads=NT)
    px, cnt = rt.queue_render(96, 72, P, n, counters=True)
    assert (px == ref).all() and cnt == rc


@pytest.mark.parametrize("slabs", ["2", "5"])
def test_slabs(rt, slabs, monkeypatch):
    monkeypatch.setenv("RT_QUEUE_SLABS", slabs)
    px, cnt = rt.queue_render(800, 600, counters=True)
    assert O.fnv1a64(px) == KA["800x600"]["frame_fnv"]
    assert cnt == KA["800x600"]["counters"]


def test_async_row_window_on_stream(rt):
    """rtq_render_async: device buffers, a row window, a non-default stream;
    rows outside the window untouched."""
    import torch
    P, n = rt.scenes.queue_scene()
    w, h = 200, 150
    ref, _ = O.queue_render(w, h, nthreads=NT)
    d_prims = torch.frombuffer(bytearray(bytes(P)[:96 * n]), dtype=torch.uint8).cuda()
    frame = torch.full((h, w), 0x7f7f7f7f, dtype=torch.int32, device="cuda")
    cnt = torch.zeros(4, dtype=torch.int64, device="cuda")
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        rt.check(rt.lib().rtq_render_async(d_prims.data_ptr(), n, frame.data_ptr(), w, h, 37, 121,
                                           cnt.data_ptr(), C.c_void_p(s.cuda_stream)))
    s.synchronize()
    got = frame.cpu().numpy().view(np.uint8).reshape(h, w, 4)
    assert (got[37:121] == ref[37:121]).all()
    assert (got[:37] == 0x7f).all() and (got[121:] == 0x7f).all()
    band, bc = O.queue_render(w, h, row_begin=37, row_end=121, nthreads=NT)
    assert cnt.cpu().tolist() == bc


def test_bad_arguments(rt):
    P, n = rt.scenes.queue_scene()
    px = np.zeros((4, 4, 4), np.uint8)
    assert rt.lib().rtq_render(C.addressof(P), 0, px.ctypes.data, 4, 4, None) == rt._lib.RT_ERR_INVALID
    assert rt.lib().rtq_render(C.addressof(P), 65, px.ctypes.data, 4, 4, None) == rt._lib.RT_ERR_INVALID
    assert rt.lib().rtq_render_async(C.addressof(P), n, px.ctypes.data, 4, 4, 3, 2, None, None) == \
        rt._lib.RT_ERR_INVALID


def test_sphere_loop_exact_redo(rt):
    """The queue tracer's lean sphere loops (queue.hip nearest_n, the shadow
    loop of shade_hit) redo a loop exactly when a discriminant leaves sqrt_nr's
    range: a sphere of infinite radius (never hit) forces that redo in every
    loop, for the root pass's two-ray form too; frame and counters stay the
    oracle's."""
    P, n = O.queue_scene()
    p = P[n]
    p.type = 1
    p.center = O.F4(1.0, -2.0, 25.0, 0.0)
    p.radius, p.sq_radius, p.r_radius = float("inf"), float("inf"), 0.0
    p.m_color = O.F4(0.5, 0.5, 0.5, 0.0)
    p.m_diff, p.m_spec = 1.0, 0.0
    ref, rc = O.queue_render(160, 120, P, n + 1, nthreads=NT)
    px, cnt = rt.queue_render(160, 120, P, n + 1, counters=True)
    assert (px == ref).all()
    assert cnt == rc
