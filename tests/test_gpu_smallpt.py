"""GPU parity: smallpt kernel (smallpt.hip) vs the oracle restatement of
UpdateRenderingCPU + RadiancePathTracing (smallptgpu-v1.6/smallptCPU.cpp:77-132,
geomfunc.h:167-338).  Bar (north star): HDR accumulator within 1e-4 per
channel; the kernel is in fact expected bit-exact, which is asserted too, and
the integer pixels and RNG state must match exactly."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu
TOL = 1e-4


def _oracle_frame(oracle, w, h, steps, mode=0, spheres=None, cam=None):
    S, n = oracle.cornell() if spheres is None else spheres
    cam = oracle.cornell_camera(w, h) if cam is None else cam
    col = np.zeros(3 * w * h, np.float32)
    seeds = oracle.seeds(w, h)
    px = np.zeros(w * h, np.uint32)
    first = 0
    cnt = [0, 0, 0, 0]
    for k in steps:
        c = oracle.smallpt_render(S, n, cam, col, seeds, px, w, h, first, k, dl=mode, nthreads=8)
        cnt = [a + b for a, b in zip(cnt, c)]
        first += k
    return col, seeds, px, cnt


def _check(got, ref):
    gcol, gseeds, gpx, gcnt = got
    rcol, rseeds, rpx, rcnt = ref
    err = np.abs(gcol.astype(np.float64) - rcol.astype(np.float64))
    assert err.max() <= TOL, "max |dHDR| %g" % err.max()
    assert (gcol.view(np.uint32) == rcol.view(np.uint32)).all(), "HDR not bit-exact (%d slots)" % (
        (gcol != rcol).sum())
    assert (gseeds == rseeds).all()
    assert (gpx == rpx).all()
    assert gcnt == rcnt, (gcnt, rcnt)


@pytest.mark.parametrize("w,h,steps", [(640, 480, [1]), (640, 480, [1, 3]), (160, 120, [8, 8])])
def test_path_tracing(rt, oracle, w, h, steps):
    f = rt.SmallptFrame(w, h)
    for k in steps:
        f.render(k)
    _check((f.colors, f.seeds, f.pixels, f.counters), _oracle_frame(oracle, w, h, steps))


def test_direct_lighting(rt, oracle):
    w, h = 320, 240
    f = rt.SmallptFrame(w, h, mode=rt.SPT_DIRECT_LIGHTING)
    f.render(2)
    _check((f.colors, f.seeds, f.pixels, f.counters), _oracle_frame(oracle, w, h, [2], mode=1))


def test_batching_is_exact(rt):
    a = rt.SmallptFrame(96, 64)
    b = rt.SmallptFrame(96, 64)
    for _ in range(4):
        a.render(1)
    b.render(4)
    assert (a.colors == b.colors).all() and (a.seeds == b.seeds).all() and (a.pixels == b.pixels).all()


# Full BASELINE sizes, checked against golden hashes of the reference-built
# core (tests/golden/known_answers.json, oracle/_ref): configs[2] and the bench
# / configs[3] frames.
@pytest.mark.parametrize("key", ["1024x768_64spp", "1920x1080_64spp", "1920x1080_256spp"])
def test_full_size_golden(rt, oracle, key):
    import json
    import os
    gold = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "known_answers.json")))
    g = gold["smallpt"][key]
    res, spp = key.split("_")
    w, h = map(int, res.split("x"))
    f = rt.SmallptFrame(w, h)
    spp = int(spp[:-3])
    f.render(spp // 2)            # two launches: also exercises the first_sample > 0 path,
    f.render(spp - spp // 2, counters=False)   # and the uncounted kernel bench.py times
    got = (oracle.fnv1a64(f.colors), oracle.fnv1a64(f.pixels), oracle.fnv1a64(f.seeds))
    assert got == (g["colors"], g["pixels"], g["seeds"])


def _scene_arrays(rt, rows):
    arr = (rt.Sphere * len(rows))()
    for s, r in zip(arr, rows):
        rt.scenes._sphere(s, *r)
    return arr, len(rows)


def test_generic_lds_path(rt, oracle):
    """A 10-sphere scene (not the compile-time-specialised size 9) runs the
    LDS loop path; must match the oracle bit for bit."""
    rows = list(rt.scenes._CORNELL) + [(4.0, (20.0, 10.0, 100.0), (0, 0, 0), (.5, .9, .2), 1)]
    spheres, n = _scene_arrays(rt, rows)
    w, h = 128, 96
    f = rt.SmallptFrame(w, h, spheres=spheres, nspheres=n)
    f.render(3)
    ref = _oracle_frame(oracle, w, h, [3], spheres=(spheres, n))
    _check((f.colors, f.seeds, f.pixels, f.counters), ref)


def test_large_scene_hierarchy_vs_oracle(rt, oracle):
    """configs[4] scene (10k spheres, >= 256: the exact-culling hierarchy
    path) against the oracle's full scan, small frame."""
    spheres, n, cam = rt.scenes.complex10k()
    w, h = 48, 32
    rt.scenes.update_camera(cam, w, h)
    f = rt.SmallptFrame(w, h, spheres=spheres, nspheres=n, camera=cam)
    f.render(1)
    ref = _oracle_frame(oracle, w, h, [1], spheres=(spheres, n), cam=cam)
    _check((f.colors, f.seeds, f.pixels, f.counters), ref)


@pytest.mark.parametrize("nonstd", [3, -1])
def test_nonstandard_refl_takes_refr_branch(rt, oracle, nonstd):
    """geomfunc.h:281: every refl that is neither DIFF (0) nor SPEC (1) takes
    the REFR branch.  A hierarchy scene (configs[4]'s spheres, all DIFF, so
    normally run with the light-only pass A) with some spheres set to a
    non-standard refl must still refract there, as the oracle does."""
    spheres, n, cam = rt.scenes.complex10k()
    for i in range(2, n, 5):                 # (0: the light, 1: the ground)
        spheres[i].refl = nonstd
    w, h = 48, 32
    rt.scenes.update_camera(cam, w, h)
    f = rt.SmallptFrame(w, h, spheres=spheres, nspheres=n, camera=cam)
    f.render(2)
    ref = _oracle_frame(oracle, w, h, [2], spheres=(spheres, n), cam=cam)
    _check((f.colors, f.seeds, f.pixels, f.counters), ref)


@pytest.mark.parametrize("env", [{"RT_SPT_NO_BVH": "1"}, {"RT_SPT_GEO": "global"}])
def test_large_scene_global_path(rt, oracle, env, monkeypatch):
    """The global-SoA full-scan kernel (GEO_GLOBAL: scenes above the LDS
    budget without the hierarchy, or forced for any scene) vs the oracle:
    the 10k configs[4] scene with the hierarchy disabled, and Cornell."""
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    if "RT_SPT_NO_BVH" in env:
        spheres, n, cam = rt.scenes.complex10k()
        w, h = 32, 24
        rt.scenes.update_camera(cam, w, h)
    else:
        (spheres, n), w, h = rt.scenes.cornell(), 96, 64
        cam = rt.scenes.cornell_camera(w, h)
    f = rt.SmallptFrame(w, h, spheres=spheres, nspheres=n, camera=cam)
    f.render(2)
    ref = _oracle_frame(oracle, w, h, [2], spheres=(spheres, n), cam=cam)
    _check((f.colors, f.seeds, f.pixels, f.counters), ref)


# The two hierarchy walks: the 8-wide LDS-resident tree (default for scenes
# whose tree fits a block's LDS) and the binary octant-layout tree in global
# memory (RT_SPT_WIDE=0; the path for larger trees).
WALKS = [pytest.param({}, id="wide"), pytest.param({"RT_SPT_WIDE": "0"}, id="binary")]


@pytest.mark.parametrize("walk", WALKS)
@pytest.mark.parametrize("counted", [True, False])
def test_configs4_full_size_golden(rt, oracle, counted, walk, monkeypatch):
    """BASELINE configs[4] at full size -- the 10k-sphere scene_build_complex
    scene, 1920x1080, 64 spp from the initial state -- through the hierarchy
    kernel (with and without the work counters), against the golden hashes of
    the reference's own full-scan core (tests/golden/make_golden_c4.py,
    oracle/_ref: geomfunc.h:71-110 Intersect / IntersectP)."""
    import json
    import os
    for k, v in walk.items():
        monkeypatch.setenv(k, v)
    gold = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "known_answers.json")))
    g = gold["smallpt"]["1920x1080_64spp_complex10k"]
    spheres, n, cam = rt.scenes.complex10k()
    w, h = 1920, 1080
    rt.scenes.update_camera(cam, w, h)
    for frame in range(3):          # (the 1st launch of the key learns its order, later ones use it)
        f = rt.SmallptFrame(w, h, spheres=spheres, nspheres=n, camera=cam)
        f.render(64, counters=counted)
        got = (oracle.fnv1a64(f.colors), oracle.fnv1a64(f.pixels), oracle.fnv1a64(f.seeds))
        assert got == (g["colors"], g["pixels"], g["seeds"]), frame
        if counted:
            assert f.counters[3] == w * h * 64


@pytest.mark.parametrize("tune", ["coop=512", "coop=4096", "coop=1024,coop_g=4", "coop=1024,coop_g=2"])
@pytest.mark.parametrize("counted", [False, True])
def test_configs4_cooperative_walk_golden(rt, oracle, counted, tune, monkeypatch):
    """The heaviest tiles walk the 8-wide hierarchy eight, four or two lanes
    per pixel (wide_walk_coop<G>) once a learnt order exists: the 1st frame
    of a key records the tile costs, the next ones dispatch the heaviest tiles
    cooperatively (forced here on the full frame, which by default only
    routes them: 512 and 4096 eight-lane tiles, 1024 four-lane and 1024
    two-lane ones).  Every frame must equal the reference core's golden
    hashes (configs[4], 1920x1080, 64 spp), counted (and the counters exact)
    and uncounted."""
    import json
    import os
    monkeypatch.setenv("RT_SPT_TUNE", tune)
    gold = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "known_answers.json")))
    g = gold["smallpt"]["1920x1080_64spp_complex10k"]
    spheres, n, cam = rt.scenes.complex10k()
    w, h = 1920, 1080
    rt.scenes.update_camera(cam, w, h)
    first = None
    for i in range(3):
        f = rt.SmallptFrame(w, h, spheres=spheres, nspheres=n, camera=cam)
        # (full-counter launches learn an order of their own: after the
        # uncounted 1st frame, the 2nd records the counted tile costs and the
        # 3rd runs the counted order, cooperative tiles included)
        f.render(64, counters=counted and i > 0)
        got = (oracle.fnv1a64(f.colors), oracle.fnv1a64(f.pixels), oracle.fnv1a64(f.seeds))
        assert got == (g["colors"], g["pixels"], g["seeds"])
        if counted and i > 0:            # the 1st frame (no order yet) walks a lane per pixel
            assert f.counters[3] == w * h * 64
            first = first or list(f.counters)
            assert list(f.counters) == first


@pytest.mark.parametrize("nranks", [2, 4, 8])
def test_configs4_rank_shares_golden(rt, oracle, nranks):
    """BASELINE configs[4] split as the multi-GPU bench splits it: every
    nranks-th 8-row group per rank (spt_scene_render_groups_async), each
    share with a scene of its own that learns its order in a first frame, so
    the later frames use the window class's default cooperative tier (two
    lanes per pixel at N = 2, four at N = 4, eight at N = 8).  The assembled
    frame of the third round equals the reference core's golden hashes."""
    import ctypes as C
    import json
    import os
    import torch
    gold = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "known_answers.json")))
    g = gold["smallpt"]["1920x1080_64spp_complex10k"]
    spheres, n, cam = rt.scenes.complex10k()
    w, h = 1920, 1080
    rt.scenes.update_camera(cam, w, h)
    dev = torch.device("cuda", 0)
    st = torch.cuda.current_stream(dev).cuda_stream
    L = rt.lib()
    seeds0 = torch.from_numpy(rt.scenes.seeds(w, h).view(np.int32)).to(dev)
    scenes = [rt.SmallptScene(spheres, n) for _ in range(nranks)]
    try:
        for _ in range(3):                     # learn, then the learnt order and its tiers
            col = torch.zeros(3 * w * h, dtype=torch.float32, device=dev)
            seeds = torch.zeros_like(seeds0)
            px = torch.zeros(w * h, dtype=torch.int32, device=dev)
            for k, sc in enumerate(scenes):
                rt.check(L.spt_scene_render_groups_async(sc.handle, C.byref(cam), col.data_ptr(), seeds0.data_ptr(),
                                                         seeds.data_ptr(), px.data_ptr(), w, h, k, nranks, 0, 64, 0,
                                                         None, st))
            torch.cuda.synchronize()
        got = (oracle.fnv1a64(col.cpu().numpy()), oracle.fnv1a64(px.cpu().numpy().view(np.uint32)),
               oracle.fnv1a64(seeds.cpu().numpy().view(np.uint32)))
        assert got == (g["colors"], g["pixels"], g["seeds"])
    finally:
        for sc in scenes:
            sc.close()


def test_async_device_paths(rt, oracle):
    """spt_scene_render_async and spt_render_async on device buffers, rows
    split in two calls, seeds_in != seeds_out."""
    import ctypes as C
    import torch
    w, h = 96, 64
    S, n = rt.scenes.cornell()
    cam = rt.scenes.cornell_camera(w, h)
    dev = torch.device("cuda", 0)
    seeds0 = torch.from_numpy(rt.scenes.seeds(w, h).view(np.int32)).to(dev)
    outs = []
    for use_scene in (True, False):
        col = torch.zeros(3 * w * h, dtype=torch.float32, device=dev)
        seeds = torch.zeros_like(seeds0)
        px = torch.zeros(w * h, dtype=torch.int32, device=dev)
        st = torch.cuda.current_stream(dev).cuda_stream
        if use_scene:
            sc = rt.SmallptScene(S, n)
            for r0, r1 in ((0, 40), (40, h)):
                rt.check(rt.lib().spt_scene_render_async(sc.handle, C.byref(cam), col.data_ptr(), seeds0.data_ptr(),
                                                         seeds.data_ptr(), px.data_ptr(), w, h, r0, r1, 0, 2, 0,
                                                         None, st))
        else:
            d_s = torch.frombuffer(bytearray(bytes(S)), dtype=torch.uint8).to(dev)
            for r0, r1 in ((0, 40), (40, h)):
                rt.check(rt.lib().spt_render_async(d_s.data_ptr(), n, C.byref(cam), col.data_ptr(), seeds0.data_ptr(),
                                                   seeds.data_ptr(), px.data_ptr(), w, h, r0, r1, 0, 2, 0, None, st))
        torch.cuda.synchronize()
        outs.append((col.cpu().numpy(), seeds.cpu().numpy().view(np.uint32), px.cpu().numpy().view(np.uint32)))
    ref = _oracle_frame(oracle, w, h, [2])
    for col, seeds, px in outs:
        assert (col.view(np.uint32) == ref[0].view(np.uint32)).all()
        assert (seeds == ref[1]).all() and (px == ref[2]).all()


def test_scene_cache_follows_the_array(rt, oracle):
    """spt_render / spt_render_async keep one prepared scene per device while
    the sphere array is unchanged; a changed array (same size, one sphere's
    colour and one's position edited in place) is prepared again: every frame
    equals the oracle's for the array it was given."""
    import ctypes as C
    import torch
    w, h = 64, 48
    S, n = rt.scenes.cornell()
    cam = rt.scenes.cornell_camera(w, h)
    T, _ = rt.scenes.cornell()
    T[7].c.x, T[8].p.y = 0.25, T[8].p.y + 3.0
    dev = torch.device("cuda", 0)
    seeds0 = torch.from_numpy(rt.scenes.seeds(w, h).view(np.int32)).to(dev)
    d_s = torch.frombuffer(bytearray(bytes(S)), dtype=torch.uint8).to(dev)
    st = torch.cuda.current_stream(dev).cuda_stream
    for arr in (S, S, T, S):
        ref_col, ref_seeds, ref_px, _ = _oracle_frame(oracle, w, h, [2], spheres=(arr, n), cam=cam)
        d_s.copy_(torch.frombuffer(bytearray(bytes(arr)), dtype=torch.uint8))     # same pointer, new contents
        col = torch.zeros(3 * w * h, dtype=torch.float32, device=dev)
        seeds = torch.zeros_like(seeds0)
        px = torch.zeros(w * h, dtype=torch.int32, device=dev)
        rt.check(rt.lib().spt_render_async(d_s.data_ptr(), n, C.byref(cam), col.data_ptr(), seeds0.data_ptr(),
                                           seeds.data_ptr(), px.data_ptr(), w, h, 0, h, 0, 2, 0, None, st))
        torch.cuda.synchronize()
        assert (col.cpu().numpy().view(np.uint32) == ref_col.view(np.uint32)).all()
        assert (seeds.cpu().numpy().view(np.uint32) == ref_seeds).all()
        f = rt.SmallptFrame(w, h, spheres=arr, nspheres=n, camera=cam)
        f.render(2, counters=False)
        assert (f.colors.view(np.uint32) == ref_col.view(np.uint32)).all() and (f.pixels == ref_px).all()


@pytest.mark.parametrize("walk", WALKS)
@pytest.mark.parametrize("sched", ["0", "1"])
def test_adaptive_group_order_is_exact(rt, monkeypatch, sched, walk):
    """Hierarchy scenes dispatch their tile groups heaviest-first once a
    launch has recorded the groups' wave times (SptSched): the 1st launch of a
    key records, the 2nd builds the order, the 3rd and later use it.  Every
    launch must give the same bits as the plain dispatch (RT_SPT_SCHED=0),
    counted and uncounted, full frame and a row window."""
    import ctypes as C
    import torch
    monkeypatch.setenv("RT_SPT_SCHED", sched)
    for k, v in walk.items():
        monkeypatch.setenv(k, v)
    w, h = 480, 270
    spheres, n, cam = rt.scenes.complex10k()
    rt.scenes.update_camera(cam, w, h)
    sc = rt.SmallptScene(spheres, n)
    dev = torch.device("cuda", 0)
    seeds0 = torch.from_numpy(rt.scenes.seeds(w, h).view(np.int32)).to(dev)
    st = torch.cuda.current_stream(dev).cuda_stream
    outs = []
    for r0, r1 in ((0, h), (0, h), (0, h), (0, h), (40, 200), (40, 200), (40, 200)):
        for counted in (False, True):
            col = torch.zeros(3 * w * h, dtype=torch.float32, device=dev)
            seeds = torch.zeros_like(seeds0)
            px = torch.zeros(w * h, dtype=torch.int32, device=dev)
            cnt = torch.zeros(4, dtype=torch.int64, device=dev)
            rt.check(rt.lib().spt_scene_render_async(sc.handle, C.byref(cam), col.data_ptr(), seeds0.data_ptr(),
                                                     seeds.data_ptr(), px.data_ptr(), w, h, r0, r1, 0, 3, 0,
                                                     cnt.data_ptr() if counted else None, st))
            torch.cuda.synchronize()
            outs.append(((r0, r1), col.cpu().numpy().view(np.uint32), seeds.cpu().numpy(), px.cpu().numpy(),
                         cnt.cpu().numpy() if counted else None))
    ref = {}
    for key, c, s_, p, k in outs:
        if key not in ref:
            ref[key] = (c, s_, p)
        rc, rs, rp = ref[key]
        assert (c == rc).all() and (s_ == rs).all() and (p == rp).all(), key
    full = [k for key, *_, k in outs if key == (0, h) and k is not None]
    assert all((k == full[0]).all() for k in full)


def test_graph_replay_survives_order_changes(rt):
    """A launch captured into a graph holds the learnt tile order's device
    buffer (SptSched): later uncaptured launches of other keys (window, spp)
    that learn and install new orders -- more tile slots, so a larger buffer
    -- must neither rewrite nor free it.  Capture a launch of a small window
    once its order is in use, run two larger keys until theirs are, replay:
    the bits equal an uncaptured launch of the small window."""
    import ctypes as C
    import torch
    w, h = 480, 270
    spheres, n, cam = rt.scenes.complex10k()
    rt.scenes.update_camera(cam, w, h)
    sc = rt.SmallptScene(spheres, n)
    dev = torch.device("cuda", 0)
    seeds0 = torch.from_numpy(rt.scenes.seeds(w, h).view(np.int32)).to(dev)

    def bufs():
        return (torch.zeros(3 * w * h, dtype=torch.float32, device=dev), torch.zeros_like(seeds0),
                torch.zeros(w * h, dtype=torch.int32, device=dev))

    def launch(r0, r1, spp, b, stream):
        col, seeds, px = b
        rt.check(rt.lib().spt_scene_render_async(sc.handle, C.byref(cam), col.data_ptr(), seeds0.data_ptr(),
                                                 seeds.data_ptr(), px.data_ptr(), w, h, r0, r1, 0, spp, 0, None,
                                                 stream))

    cur = torch.cuda.current_stream(dev).cuda_stream
    small = (96, 144, 2)
    for _ in range(3):                               # record, build the order, use it
        launch(*small, bufs(), cur)
    torch.cuda.synchronize()
    gb = bufs()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, capture_error_mode="relaxed"):
        launch(*small, gb, torch.cuda.current_stream(dev).cuda_stream)
    torch.cuda.synchronize()
    for key in ((0, h, 2), (0, h, 3)):               # new keys, larger order buffers
        for _ in range(3):
            launch(*key, bufs(), cur)
    torch.cuda.synchronize()
    for t in gb:
        t.zero_()
    g.replay()
    ref = bufs()
    launch(*small, ref, cur)
    torch.cuda.synchronize()
    for a, b in zip(gb, ref):
        assert (a.cpu().numpy().view(np.uint32) == b.cpu().numpy().view(np.uint32)).all()


def test_capture_limit_and_release(rt):
    """A hierarchy scene holds 64 work-counter entries and a captured launch
    keeps its entry for the graph's life: with 64 captured launches alive the
    next launch is refused (RT_ERR_INVALID, nothing launched); once the graph
    is destroyed spt_scene_release_captures hands the entries out again, and
    a new capture replays to the uncaptured frame's bits."""
    import ctypes as C
    import torch
    w, h = 64, 16
    spheres, n, cam = rt.scenes.complex10k()
    rt.scenes.update_camera(cam, w, h)
    sc = rt.SmallptScene(spheres, n)
    dev = torch.device("cuda", 0)
    seeds0 = torch.from_numpy(rt.scenes.seeds(w, h).view(np.int32)).to(dev)
    L = rt.lib()
    b = (torch.zeros(3 * w * h, dtype=torch.float32, device=dev), torch.zeros_like(seeds0),
         torch.zeros(w * h, dtype=torch.int32, device=dev))

    def launch(buf):
        return L.spt_scene_render_async(sc.handle, C.byref(cam), buf[0].data_ptr(), seeds0.data_ptr(),
                                        buf[1].data_ptr(), buf[2].data_ptr(), w, h, 0, h, 0, 1, 0, None,
                                        torch.cuda.current_stream(dev).cuda_stream)

    for _ in range(3):
        rt.check(launch(b))
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, capture_error_mode="relaxed"):
        rcs = [launch(b) for _ in range(64)]
    assert rcs == [0] * 64
    g2 = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g2, capture_error_mode="relaxed"):
        assert launch(b) == rt._lib.RT_ERR_INVALID
    assert launch(b) == rt._lib.RT_ERR_INVALID        # (uncaptured launches need an entry too)
    del g, g2
    torch.cuda.synchronize()
    rt.check(L.spt_scene_release_captures(sc.handle))
    gb = tuple(torch.zeros_like(t) for t in b)
    g3 = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g3, capture_error_mode="relaxed"):
        rt.check(launch(gb))
    g3.replay()
    ref = tuple(torch.zeros_like(t) for t in b)
    rt.check(launch(ref))
    torch.cuda.synchronize()
    for a, r in zip(gb, ref):
        assert torch.equal(a.view(torch.int32), r.view(torch.int32))


def _bvh_vs_scan(rt, monkeypatch, spheres, n, cam, w, h, spp, mode=0):
    """Renders with the 8-wide hierarchy, the binary hierarchy (RT_SPT_WIDE=0)
    and the full scan (RT_SPT_NO_BVH), each with and without the work
    counters (the uncounted kernels stop a shadow query at its first
    occluder): colours, seeds, pixels and counters must be identical bit for
    bit."""
    outs = []
    for env in ({}, {"RT_SPT_WIDE": "0"}, {"RT_SPT_NO_BVH": "1"}):
        for k in ("RT_SPT_WIDE", "RT_SPT_NO_BVH"):
            if k in env:
                monkeypatch.setenv(k, env[k])
            else:
                monkeypatch.delenv(k, raising=False)
        for counted in (True, False):
            f = rt.SmallptFrame(w, h, spheres=spheres, nspheres=n, camera=cam, mode=mode)
            f.render(spp, counters=counted)
            outs.append(f)
    a = outs[0]
    for b in outs[1:]:
        assert np.array_equal(a.colors.view(np.uint32), b.colors.view(np.uint32))
        assert np.array_equal(a.seeds, b.seeds) and np.array_equal(a.pixels, b.pixels)
    assert a.counters == outs[2].counters == outs[4].counters


def test_bvh_equals_full_scan_configs4(rt, monkeypatch):
    """configs[4] (10k spheres) at 1920x1080, 2 spp: hierarchy == full scan."""
    spheres, n, cam = rt.scenes.complex10k()
    rt.scenes.update_camera(cam, 1920, 1080)
    _bvh_vs_scan(rt, monkeypatch, spheres, n, cam, 1920, 1080, 2)


@pytest.mark.parametrize("seed,mode,far", [(1, 0, 0), (2, 0, 0), (3, 1, 0), (4, 0, 0),
                                           (5, 0, 3000), (6, 1, 20000)])
def test_bvh_equals_full_scan_random_scenes(rt, monkeypatch, seed, mode, far):
    """Random clouds of small spheres (some overlapping, some tiny, some far),
    a huge ground sphere and lights, camera inside the cloud: grazing and
    inside-sphere rays included.  far > 0: camera that far away with a
    narrow view of the cloud, where the culling margin (proportional to the
    origin's distance) is widest in absolute terms."""
    rng = np.random.default_rng(seed)
    n = 3000
    S = (rt.Sphere * n)()
    DIFF, SPEC, REFR = 0, 1, 2
    rt.scenes._sphere(S[0], 1e4, (0.0, -1e4 - 20.0, 0.0), (0, 0, 0), (0.7, 0.7, 0.7), DIFF)
    rt.scenes._sphere(S[1], 3.0, (0.0, 40.0, 0.0), (20, 20, 20), (0, 0, 0), DIFF)
    rt.scenes._sphere(S[2], 0.5, (10.0, 5.0, -5.0), (5, 3, 3), (0, 0, 0), DIFF)
    for i in range(3, n):
        scale = 10.0 ** rng.uniform(-2.5, 0.5)
        c = rng.uniform(-30, 30, 3)
        refl = int(rng.choice([DIFF, DIFF, DIFF, SPEC, REFR]))
        rt.scenes._sphere(S[i], scale, tuple(c), (0, 0, 0), tuple(rng.uniform(0.2, 0.9, 3)), refl)
    cam = rt.Camera()
    cam.orig = rt.Vec3(1.0, 2.0, 25.0) if not far else rt.Vec3(0.3 * far, 0.2 * far, far)
    cam.target = rt.Vec3(0.0, 0.0, 0.0)
    rt.scenes.update_camera(cam, 160, 120, fov_deg=45.0 if not far else 45.0 * 60.0 / far)
    _bvh_vs_scan(rt, monkeypatch, S, n, cam, 160, 120, 4, mode)


@pytest.mark.parametrize("seed", [11, 12, 13, 14, 15, 16])
def test_random_scenes_vs_oracle(rt, oracle, seed):
    """Random scenes (random sphere count, sizes, materials, lights, some
    overlapping, random camera) at ragged sizes, split progressive passes and
    both estimators, against the oracle: bit-exact HDR, seeds, pixels, counts."""
    rng = np.random.default_rng(seed)
    n = int(rng.integers(3, 40))
    S = (rt.Sphere * n)()
    for i in range(n):
        big = rng.random() < 0.2
        rad = float(10 ** rng.uniform(2, 4)) if big else float(10 ** rng.uniform(-1.5, 1.2))
        c = rng.uniform(-60, 60, 3)
        if big:
            ax = int(rng.integers(0, 3))
            c[ax] = np.sign(rng.standard_normal()) * (rad + rng.uniform(20, 80))
        light = rng.random() < 0.15 or i == 0
        e = tuple(rng.uniform(1, 15, 3)) if light else (0.0, 0.0, 0.0)
        refl = int(rng.choice([0, 0, 0, 1, 2]))
        rt.scenes._sphere(S[i], rad, tuple(c), e, tuple(rng.uniform(0.1, 0.95, 3)), refl)
    w, h = int(rng.integers(24, 90)), int(rng.integers(16, 70))
    cam = rt.Camera()
    cam.orig = rt.Vec3(*map(float, rng.uniform(-20, 20, 3)))
    cam.target = rt.Vec3(*map(float, rng.uniform(-20, 20, 3)))
    rt.scenes.update_camera(cam, w, h)
    mode = int(seed % 2)
    steps = [int(rng.integers(1, 4)), int(rng.integers(1, 4))]
    f = rt.SmallptFrame(w, h, spheres=S, nspheres=n, camera=cam, mode=mode)
    for k in steps:
        f.render(k)
    ref = _oracle_frame(oracle, w, h, steps, mode=mode, spheres=(S, n), cam=cam)
    _check((f.colors, f.seeds, f.pixels, f.counters), ref)
    g = rt.SmallptFrame(w, h, spheres=S, nspheres=n, camera=cam, mode=mode)
    for k in steps:
        g.render(k, counters=False)
    assert (g.colors.view(np.uint32) == f.colors.view(np.uint32)).all()
    assert (g.seeds == f.seeds).all() and (g.pixels == f.pixels).all()


@pytest.mark.parametrize("geo", ["lds", "global"])
def test_light_free_scene_vs_oracle(rt, oracle, geo, monkeypatch):
    """A scene with no emitter at all: render_kernel loads light 0's records
    unconditionally (discarded by selects), so the scene carries one zero
    record; the frame must still be the oracle's, bit for bit, on the LDS and
    the global-SoA paths, both estimators."""
    if geo == "global":
        monkeypatch.setenv("RT_SPT_GEO", "global")
    rng = np.random.default_rng(7)
    n = 12
    S = (rt.Sphere * n)()
    for i in range(n):
        rt.scenes._sphere(S[i], float(10 ** rng.uniform(-1, 1.2)), tuple(rng.uniform(-30, 30, 3)), (0.0, 0.0, 0.0),
                          tuple(rng.uniform(0.1, 0.95, 3)), int(rng.choice([0, 1, 2])))
    w, h = 40, 28
    cam = rt.Camera()
    cam.orig = rt.Vec3(0.0, 0.0, 80.0)
    cam.target = rt.Vec3(0.0, 0.0, 0.0)
    rt.scenes.update_camera(cam, w, h)
    for mode in (0, 1):
        f = rt.SmallptFrame(w, h, spheres=S, nspheres=n, camera=cam, mode=mode)
        f.render(3)
        _check((f.colors, f.seeds, f.pixels, f.counters),
               _oracle_frame(oracle, w, h, [3], mode=mode, spheres=(S, n), cam=cam))


def test_pack_pixels_matches_render(rt):
    """spt_pack_pixels_async (the repack after a multi-GPU colour all-gather)
    rebuilds exactly the pixels the render kernel wrote, for a row window."""
    import torch
    w, h = 320, 200
    f = rt.SmallptFrame(w, h)
    f.render(3)
    dev = torch.device("cuda", 0)
    col = torch.from_numpy(f.colors).to(dev)
    px = torch.zeros(w * h, dtype=torch.int32, device=dev)
    st = torch.cuda.current_stream(dev).cuda_stream
    rt.check(rt.lib().spt_pack_pixels_async(col.data_ptr(), px.data_ptr(), w, h, 0, h, st))
    torch.cuda.synchronize()
    assert (px.cpu().numpy().view(np.uint32) == f.pixels).all()
    px.zero_()
    rt.check(rt.lib().spt_pack_pixels_async(col.data_ptr(), px.data_ptr(), w, h, 50, 120, st))
    torch.cuda.synchronize()
    got = px.cpu().numpy().view(np.uint32).reshape(h, w)
    assert (got[50:120] == f.pixels.reshape(h, w)[50:120]).all() and not got[:50].any() and not got[120:].any()


@pytest.mark.parametrize("dual", ["0", "1"])
def test_one_and_two_query_iterations(rt, oracle, dual, monkeypatch):
    """Both forms of the single-light loop -- one ray query per iteration, and
    the two-query iteration (shadow ray + bounce ray together, which the
    library picks for every single-light scene) -- forced either way, against the
    oracle at a small size and the reference-core golden at 1920x1080x64."""
    import json
    import os
    monkeypatch.setenv("RT_SPT_DUAL", dual)
    w, h = 200, 150
    f = rt.SmallptFrame(w, h)
    f.render(3)
    f.render(2, counters=False)
    ref = _oracle_frame(oracle, w, h, [3, 2])
    assert (f.colors.view(np.uint32) == ref[0].view(np.uint32)).all()
    assert (f.seeds == ref[1]).all() and (f.pixels == ref[2]).all()
    g = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "known_answers.json")))
    g = g["smallpt"]["1920x1080_64spp"]
    f = rt.SmallptFrame(1920, 1080)
    f.render(64, counters=False)
    assert (oracle.fnv1a64(f.colors), oracle.fnv1a64(f.pixels), oracle.fnv1a64(f.seeds)) == \
        (g["colors"], g["pixels"], g["seeds"])
