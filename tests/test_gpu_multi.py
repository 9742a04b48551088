"""smallpt frames tiled over several GPUs behind the C-ABI (spt_render_multi,
spt_multi_*; SURVEY.md §8(b) "spt_render(..., ngpus)", §8(e) row bands).

A device may repeat in the device list, so the band / assemble code runs
with N bands on a one-GPU box exactly as it runs over N GPUs; with distinct
devices the gather is an RCCL group (RT_SPT_GATHER=rccl forces that path even
for one band).  Every result must equal the single-GPU frame bit for bit,
which the other GPU tests pin to the reference."""
import json
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "known_answers.json")


def _frame(rt, w, h, spp, devices=None, first=0, counters=True):
    f = rt.SmallptFrame(w, h)
    if first:
        f.render(first, counters=False)
    f.render(spp, counters=counters, devices=devices)
    return f


def _same(a, b):
    assert (a.colors.view(np.uint32) == b.colors.view(np.uint32)).all()
    assert (a.seeds == b.seeds).all() and (a.pixels == b.pixels).all()


def test_render_multi_one_device_equals_single(rt):
    a = _frame(rt, 320, 240, 4)
    b = _frame(rt, 320, 240, 4, devices=[0])
    _same(a, b)
    assert a.counters == b.counters


@pytest.mark.parametrize("nb,w,h", [(2, 320, 240), (3, 197, 241), (5, 64, 7), (7, 160, 120)])
def test_render_multi_repeated_device_bands(rt, nb, w, h):
    """nb bands on device 0 (ragged: h not a multiple of nb, bands of 1-2
    rows), continuing a progressive frame (first_sample > 0: the
    accumulator is uploaded per band too)."""
    a = _frame(rt, w, h, 3, first=2)
    b = _frame(rt, w, h, 3, devices=[0] * nb, first=2)
    _same(a, b)
    assert a.counters == b.counters


def _cache_info(rt):
    import ctypes as C
    out = (C.c_uint64 * 2)()
    rt.check(rt.lib().spt_multi_cache_info(out))
    return out[0], out[1]


def test_render_multi_reuses_its_band_context(rt, oracle):
    """spt_render_multi keeps its band context (scenes, buffers, streams)
    across calls: a second call with the same devices, size and spheres
    prepares nothing (contexts and scene preparations unchanged) and is
    bit-exact; an edited sphere array re-prepares only the scenes; another
    device list or frame size builds a new context -- every frame exact."""
    w, h = 160, 120
    _frame(rt, w, h, 2, devices=[0, 0])              # (context for [0, 0] at 160x120)
    c0, p0 = _cache_info(rt)
    a = _frame(rt, w, h, 2, devices=[0, 0])
    assert _cache_info(rt) == (c0, p0)                # reused: no scene preparation
    _same(a, _frame(rt, w, h, 2))
    S, n = rt.scenes.cornell()
    S[6].p.x += 1.0
    f = rt.SmallptFrame(w, h, spheres=S, nspheres=n)
    f.render(2, devices=[0, 0])
    assert _cache_info(rt) == (c0, p0 + 1)            # scenes re-prepared, same context
    g = rt.SmallptFrame(w, h, spheres=S, nspheres=n)
    g.render(2)
    _same(f, g)
    b = _frame(rt, w, h, 2, devices=[0, 0, 0])        # another device list: a new context
    assert _cache_info(rt)[0] == c0 + 1
    _same(b, _frame(rt, w, h, 2))
    c = _frame(rt, 96, 64, 3, devices=[0, 0, 0])      # another size: a new context
    assert _cache_info(rt)[0] == c0 + 2
    _same(c, _frame(rt, 96, 64, 3))


def test_render_multi_direct_lighting(rt):
    a = rt.SmallptFrame(160, 120, mode=rt.SPT_DIRECT_LIGHTING).render(3)
    b = rt.SmallptFrame(160, 120, mode=rt.SPT_DIRECT_LIGHTING).render(3, devices=[0, 0, 0])
    _same(a, b)


@pytest.mark.parametrize("gather", ["peer", "rccl"])
def test_multi_context_progressive_and_gather(rt, gather, monkeypatch):
    """Device-resident progressive passes on a band context, then the gather:
    every band's device then holds the whole frame (HDR + repacked RGBA8)."""
    w, h = 256, 192
    nb = 4 if gather == "peer" else 1          # RCCL needs distinct devices: one band here
    monkeypatch.setenv("RT_SPT_GATHER", gather)
    cam = rt.scenes.cornell_camera(w, h)
    m = rt.SmallptMulti(w, h, [0] * nb)
    assert m.rows[0] == 0 and m.rows[-1] == h and len(m.rows) == nb + 1
    seeds = rt.scenes.seeds(w, h)
    m.upload(seeds)
    for k in range(3):                          # three UpdateRenderingGPU-style passes
        m.render(cam, k, 1, counters=True)
    m.gather()
    m.sync()
    ref = _frame(rt, w, h, 3)
    for k in range(nb):
        col, px = m.read_frame(k)
        assert (col.view(np.uint32) == ref.colors.view(np.uint32)).all(), k
        assert (px == ref.pixels).all(), k
    col, sd, px = np.empty_like(ref.colors), np.empty_like(ref.seeds), np.empty_like(ref.pixels)
    m.download(col, sd, px)
    assert (col.view(np.uint32) == ref.colors.view(np.uint32)).all() and (sd == ref.seeds).all()
    assert (px == ref.pixels).all()
    assert m.counters() == ref.counters
    # a second frame after the gather (the peer copies are ordered before the
    # next render overwrites a band's rows)
    m.render(cam, 3, 2)
    m.gather()
    m.sync()
    ref.render(2)
    for k in range(nb):
        col, px = m.read_frame(k)
        assert (col.view(np.uint32) == ref.colors.view(np.uint32)).all() and (px == ref.pixels).all(), k
    m.close()


def test_multi_scene_update(rt):
    """spt_multi_set_scene (ReInitSceneGPU) re-uploads the edited scene to
    every band."""
    w, h = 160, 120
    S, n = rt.scenes.cornell()
    cam = rt.scenes.cornell_camera(w, h)
    m = rt.SmallptMulti(w, h, [0, 0], S, n)
    m.upload(rt.scenes.seeds(w, h))
    m.render(cam, 0, 2)
    S[6].p.x += 1.0
    m.set_scene(S, n)
    m.render(cam, 0, 2)
    col, px = np.empty(3 * w * h, np.float32), np.empty(w * h, np.uint32)
    m.download(col, None, px)
    f = rt.SmallptFrame(w, h)
    f.render(2)
    f.spheres = S
    f.current_sample = 0
    f.render(2)
    assert (col.view(np.uint32) == f.colors.view(np.uint32)).all() and (px == f.pixels).all()


def test_render_multi_full_frame_golden(rt, oracle):
    """BASELINE configs[3]'s frame (Cornell 1920x1080, 64 spp) in eight row
    bands on one device (the N = 8 decomposition), against the reference-
    core golden hashes."""
    ka = json.load(open(GOLDEN))["smallpt"]["1920x1080_64spp"]
    f = _frame(rt, 1920, 1080, 64, devices=[0] * 8, counters=False)
    assert oracle.fnv1a64(f.colors) == ka["colors"]
    assert oracle.fnv1a64(f.pixels) == ka["pixels"]
    assert oracle.fnv1a64(f.seeds) == ka["seeds"]


def test_multi_bad_arguments(rt):
    S, n = rt.scenes.cornell()
    with pytest.raises(rt.RTError):
        rt.SmallptMulti(64, 4, [0] * 5, S, n)       # more bands than rows
    with pytest.raises(rt.RTError):
        rt.SmallptMulti(64, 64, [rt.device_count()], S, n)


@pytest.mark.parametrize("ngroups,w,h,spp", [(2, 320, 240, 3), (3, 197, 241, 2), (4, 1920, 1080, 2), (8, 160, 60, 4)])
def test_interleaved_groups_partition_the_frame(rt, ngroups, w, h, spp):
    """spt_scene_render_groups_async for groups 0..ngroups-1 (the interleaved
    multi-GPU split of bench.py) into one device frame == one full-frame
    render, bit for bit, counters summed."""
    import ctypes as C
    import torch
    dev = torch.device("cuda", 0)
    S, n = rt.scenes.cornell()
    cam = rt.scenes.cornell_camera(w, h)
    sc = rt.SmallptScene(S, n)
    seeds0 = torch.from_numpy(rt.scenes.seeds(w, h).view(np.int32)).to(dev)
    L = rt.lib()
    st = torch.cuda.current_stream(dev)

    def buffers():
        return (torch.zeros(3 * w * h, dtype=torch.float32, device=dev), torch.empty_like(seeds0),
                torch.zeros(w * h, dtype=torch.int32, device=dev), torch.zeros(4, dtype=torch.int64, device=dev))

    c1, s1, p1, n1 = buffers()
    rt.check(L.spt_scene_render_async(sc.handle, C.byref(cam), c1.data_ptr(), seeds0.data_ptr(), s1.data_ptr(),
                                      p1.data_ptr(), w, h, 0, h, 0, spp, 0, n1.data_ptr(), st.cuda_stream))
    c2, s2, p2, n2 = buffers()
    for g in range(ngroups):
        rt.check(L.spt_scene_render_groups_async(sc.handle, C.byref(cam), c2.data_ptr(), seeds0.data_ptr(),
                                                 s2.data_ptr(), p2.data_ptr(), w, h, g, ngroups, 0, spp, 0,
                                                 n2.data_ptr(), st.cuda_stream))
    torch.cuda.synchronize()
    assert torch.equal(c1.view(torch.int32), c2.view(torch.int32))
    assert torch.equal(s1, s2) and torch.equal(p1, p2)
    assert n1.tolist() == n2.tolist()
    assert rt.lib().spt_scene_render_groups_async(sc.handle, C.byref(cam), c2.data_ptr(), seeds0.data_ptr(),
                                                  s2.data_ptr(), p2.data_ptr(), w, h, ngroups, ngroups, 0, 1, 0,
                                                  None, st.cuda_stream) == rt._lib.RT_ERR_INVALID
