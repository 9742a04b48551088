"""GPU parity: Whitted kernel (whitted.hip) vs the oracle restatement of
Engine_Render (raytracer3.0.06.no_rec.samp/raytracer.cpp:301-530).
Bar: bit-exact uint32 frames, identical ray / test / TIR counts."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("w,h", [(640, 480), (800, 600), (1920, 1080)])
def test_full_frame_bit_exact(rt, oracle, w, h):
    ref, rc = oracle.whitted_render(w, h, nthreads=8)
    got, gc = rt.whitted_render(w, h, counters=True)
    diff = np.argwhere(got != ref)
    assert diff.size == 0, "pixels differ at %s (got %x want %x)" % (
        diff[:5].tolist(), got[tuple(diff[0])], ref[tuple(diff[0])])
    assert gc == rc, (gc, rc)


def test_row_window_and_untouched_rows(rt, oracle):
    w, h = 320, 240
    ref, _ = oracle.whitted_render(w, h, row_begin=37, row_end=131)
    frame = np.full((h, w), 0xDEADBEEF, dtype=np.uint32)
    rt.whitted_render(w, h, row_begin=37, row_end=131, frame=frame)
    assert (frame[37:131] == ref[37:131]).all()
    assert (frame[:37] == 0xDEADBEEF).all() and (frame[131:] == 0xDEADBEEF).all()


def test_bad_rows_rejected(rt):
    with pytest.raises(rt.RTError):
        rt.whitted_render(64, 64, row_begin=10, row_end=40)


@pytest.mark.parametrize("w,h", [(97, 131), (33, 91)])
def test_ragged_sizes(rt, oracle, w, h):
    ref, rc = oracle.whitted_render(w, h, row_begin=20, row_end=h)
    got, gc = rt.whitted_render(w, h, row_begin=20, row_end=h, counters=True)
    assert (got == ref).all() and gc == rc


def test_golden_hashes(rt, oracle):
    import json
    import os
    gold = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "known_answers.json")))
    for key, g in gold["whitted"].items():
        w, h = map(int, key.split("x"))
        f, c = rt.whitted_render(w, h, counters=True)
        assert oracle.fnv1a64(f) == g["xrgb"] and c == g["counters"], key


@pytest.mark.parametrize("cap", [1, 1000, 20000])
def test_queue_overflow_falls_back_exactly(rt, oracle, cap, monkeypatch):
    # Child queues smaller than the tree count: nodes that do not fit are
    # evaluated by the sequential fixup pass; frame and counts stay exact.
    monkeypatch.setenv("RT_WHITTED_QUEUE_CAP", str(cap))
    w, h = 320, 240
    ref, rc = oracle.whitted_render(w, h, nthreads=8)
    got, gc = rt.whitted_render(w, h, counters=True)
    assert (got == ref).all() and gc == rc


def test_tir_trees_counted_once(rt, oracle):
    # 640x480 holds 1,874 total-internal-reflection events over all nodes
    # (SURVEY §8(a) W5), 1,056 of them at nodes < 31 (the ones with a traced,
    # stale-ray refraction child, which the counter reports): their trees go
    # through the fixup pass and every count must still match.
    _, rc = oracle.whitted_render(640, 480, nthreads=8)
    _, gc = rt.whitted_render(640, 480, counters=True)
    assert rc[3] == 1056 and gc == rc


@pytest.mark.parametrize("w,h", [(640, 480), (800, 600), (1920, 1080), (97, 131)])
def test_opencl_semantics_bit_exact(rt, oracle, w, h):
    """rtw_render_ocl (raytrace_kernel of openCLcode.cl) vs the oracle's
    restatement of the same kernel: bit-exact frame and counters."""
    ref, rc = oracle.whitted_render_ocl(w, h, nthreads=8)
    got, gc = rt.whitted_render_ocl(w, h, counters=True)
    assert (got == ref).all() and gc == rc


def test_opencl_semantics_differs_from_cpu_path(rt):
    a = rt.whitted_render_ocl(640, 480)
    b = rt.whitted_render(640, 480)
    assert (a[20:410] != b[20:410]).any() and (a[:20] == 0).all()


@pytest.mark.parametrize("seed", [21, 22, 23, 24, 25, 26, 27])
def test_random_scenes_vs_oracle(rt, oracle, seed):
    """Random primitive sets (spheres and planes, refractive / reflective /
    diffuse / specular materials, sphere and plane lights) at ragged sizes,
    both the CPU-path and the OpenCL-kernel semantics: bit-exact frames and
    counters (deep glass trees, TIR, overlapping primitives included)."""
    from rtamd.scenes import PLANE, SPHERE, _prim
    rng = np.random.default_rng(seed)
    n = 64 if seed == 27 else int(rng.integers(4, 48))     # 27: MAXP, a lane per primitive in the scene build
    P = (rt.Primitive * n)()
    for i in range(n):
        light = i < 2 or rng.random() < 0.08
        if rng.random() < 0.75:
            c = (rng.uniform(-8, 8), rng.uniform(-6, 7), rng.uniform(8, 40))
            _prim(P[i], SPHERE, *c, float(rng.uniform(0.2, 4.0)), *rng.uniform(0.05, 1.8, 3),
                  float(rng.choice([0.0, 0.0, rng.uniform(0.1, 1.9)])),
                  float(rng.choice([0.0, 0.0, rng.uniform(0.3, 1.5)])),
                  float(rng.uniform(1.0, 2.6)), float(rng.uniform(0, 1.2)), float(rng.uniform(0, 1.8)), light)
        else:
            nrm = rng.standard_normal(3)
            _prim(P[i], PLANE, *nrm, float(rng.uniform(2, 12)), *rng.uniform(0.05, 2.5, 3),
                  float(rng.choice([0.0, rng.uniform(0.1, 0.9)])), 0.0, 1.0,
                  float(rng.uniform(0, 1.2)), float(rng.uniform(0, 1.5)), light and rng.random() < 0.3)
    w, h = int(rng.integers(60, 200)), int(rng.integers(100, 160))
    ref, rc = oracle.whitted_render(w, h, nthreads=8, prims=P, n=n)
    got, gc = rt.whitted_render(w, h, prims=P, nprims=n, counters=True)
    assert (got == ref).all() and gc == rc
    ref, rc = oracle.whitted_render_ocl(w, h, nthreads=8, prims=P, n=n)
    got, gc = rt.whitted_render_ocl(w, h, prims=P, nprims=n, counters=True)
    assert (got == ref).all() and gc == rc


@pytest.mark.parametrize("streams", ["1", "2"])
@pytest.mark.parametrize("slabs", [2, 3, 7])
def test_interleaved_slabs_bit_exact(rt, oracle, slabs, streams, monkeypatch):
    """The level pass over several interleaved row slabs (what frames above
    SLAB_TREES trees use) gives the same frame and counts; also with queues
    small enough to send trees to the fixup pass.  With two streams, slabs
    alternate between them and slabs 0, 2, ... reuse the first arena."""
    monkeypatch.setenv("RT_WHITTED_SLABS", str(slabs))
    monkeypatch.setenv("RT_WHITTED_STREAMS", streams)
    w, h = 320, 240
    ref, rc = oracle.whitted_render(w, h, nthreads=8)
    got, gc = rt.whitted_render(w, h, counters=True)
    assert (got == ref).all() and gc == rc
    monkeypatch.setenv("RT_WHITTED_QUEUE_CAP", "3000")
    got, gc = rt.whitted_render(w, h, counters=True)
    assert (got == ref).all() and gc == rc
    ref, rc = oracle.whitted_render_ocl(w, h, nthreads=8)
    got, gc = rt.whitted_render_ocl(w, h, counters=True)
    assert (got == ref).all() and gc == rc


@pytest.mark.parametrize("split", ["5,3", "2,1", "1,3", "7,6"])
def test_unequal_two_stream_slabs_bit_exact(rt, oracle, split, monkeypatch):
    """Two slabs on two streams that take unequal shares of the 16-row groups
    (RT_WHITTED_SPLIT=p,q: the first slab p of every p + q groups, the
    second q) give the same frame and counts, at a ragged height too."""
    monkeypatch.setenv("RT_WHITTED_STREAMS", "2")
    monkeypatch.setenv("RT_WHITTED_SPLIT", split)
    for w, h in ((320, 240), (200, 170)):
        ref, rc = oracle.whitted_render(w, h, nthreads=8)
        got, gc = rt.whitted_render(w, h, counters=True)
        assert (got == ref).all() and gc == rc


def test_slab_tree_word_limit(rt, monkeypatch):
    """A queued item carries tree | node << 25, so a slab holds at most 2^25
    trees: a 3840x2400 frame (~80 M trees) forced into one slab
    (RT_WHITTED_SLABS=1) is split into enough slabs by the library and
    renders the same frame and counts as the default slab plan."""
    w, h = 3840, 2400
    ref, rc = rt.whitted_render(w, h, counters=True)
    monkeypatch.setenv("RT_WHITTED_SLABS", "1")
    got, gc = rt.whitted_render(w, h, counters=True)
    assert (got == ref).all() and gc == rc


@pytest.mark.parametrize("w,h,r0,r1", [(1920, 1080, 20, 1010), (1920, 1080, 20, 1080), (3840, 2400, 20, 2330)])
def test_device_memory_bounded(rt, w, h, r0, r1):
    """The level pass's device memory for the reference window of a 1920x1080
    frame, a full-height one and a 3840x2400 one stays within one
    single-stream arena's size: with two streams live at once, each slab
    holds at most SLAB_TREES / 2 trees."""
    rt.lib().rt_release()
    rt.whitted_render(w, h, row_begin=r0, row_end=r1)
    assert rt.lib().rt_cached_bytes() < 1.55e9, rt.lib().rt_cached_bytes()


def test_async_frames_on_other_streams_are_ordered(rt, oracle):
    """Device-resident frames of different sizes issued back to back on two
    non-blocking streams without host synchronisation: the shared arena and
    view tables are reused only after the previous frame."""
    import ctypes as C
    import torch
    prims, n = rt.scenes.whitted_scene()
    dev = torch.device("cuda", 0)
    d_prims = torch.frombuffer(bytearray(bytes(prims)[:96 * n]), dtype=torch.uint8).to(dev)
    s1, s2 = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    sizes = [(1920, 1080, s1), (640, 480, s2), (800, 600, s1), (1920, 1080, s2)]
    frames = [torch.zeros(h * w, dtype=torch.int32, device=dev) for w, h, _ in sizes]
    torch.cuda.synchronize(dev)
    for (w, h, s), f in zip(sizes, frames):
        rt.check(rt.lib().rtw_render_async(d_prims.data_ptr(), n, f.data_ptr(), w, h, 20, h - 70, None,
                                           C.c_void_p(s.cuda_stream)))
    torch.cuda.synchronize(dev)
    for (w, h, _), f in zip(sizes, frames):
        ref, _ = oracle.whitted_render(w, h, nthreads=8)
        got = f.cpu().numpy().view(np.uint32).reshape(h, w)
        assert (got == ref).all(), (w, h)


def test_pool_grows_after_overflow(rt, oracle, monkeypatch):
    """A frame whose nodes overflow the record pool is finished exactly by
    fixup_kernel and raises the host-mapped overflow flag; the next frames of
    that size get a pool 1.25x larger each time until it fits (the arena
    grows).  Every frame bit-exact, counts included."""
    monkeypatch.setenv("RT_POOL_FRAC", "0.25")
    w, h = 352, 288                     # a size no other test uses: a fresh pool entry
    ref, rc = oracle.whitted_render(w, h, nthreads=8)
    rt.lib().rt_release()
    sizes = []
    for _ in range(6):
        got, gc = rt.whitted_render(w, h, counters=True)
        assert (got == ref).all() and gc == rc
        sizes.append(rt.lib().rt_cached_bytes())
    assert sizes[-1] > sizes[0], sizes


def test_sphere_loop_exact_redo(rt, oracle):
    """trace()'s sphere loops use sqrt_nr for every lane and redo the whole
    loop with the exact per-sphere test when some lane's discriminant is
    outside its range (whitted.hip nearest_n, shade_hit).  A non-light sphere of
    infinite radius makes every discriminant +inf -- never a hit, but a redo
    in every nearest and occluder loop: frame and counters stay the
    oracle's."""
    from rtamd.scenes import SPHERE, _prim, whitted_scene
    S, n = whitted_scene()
    P = (rt.Primitive * (n + 2))()
    for i in range(n):
        P[i] = S[i]
    _prim(P[n], SPHERE, 1.0, -2.0, 25.0, float("inf"), 0.5, 0.5, 0.5, 0.0, 0.0, 1.0, 1.0, 0.0, False)
    _prim(P[n + 1], SPHERE, -1.0, 1.0, 20.0, 1e-15, 0.5, 0.5, 0.5, 0.3, 0.0, 1.0, 1.0, 0.5, False)
    w, h = 200, 150
    ref, rc = oracle.whitted_render(w, h, nthreads=8, prims=P, n=n + 2)
    got, gc = rt.whitted_render(w, h, prims=P, nprims=n + 2, counters=True)
    assert (got == ref).all() and gc == rc


@pytest.mark.parametrize("light", [False, True])
def test_single_primitive_scene(rt, oracle, light):
    """One primitive (the scene image's lists then hold one or no entry: a
    light sphere has no occluders, a plain one no lights)."""
    from rtamd.scenes import SPHERE, _prim
    P = (rt.Primitive * 1)()
    _prim(P[0], SPHERE, 0.5, 0.0, 12.0, 2.0, 0.7, 0.6, 0.5, 0.4, 0.0, 1.0, 0.8, 0.6, light)
    ref, rc = oracle.whitted_render(96, 128, nthreads=8, prims=P, n=1)
    got, gc = rt.whitted_render(96, 128, prims=P, nprims=1, counters=True)
    assert (got == ref).all() and gc == rc
