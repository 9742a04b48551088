"""Explicit tile-group lists (spt_scene_render_list_async, the cost-balanced
multi-GPU split of configs[4]), the group pack / unpack of their exchange,
and the rays-only counter mode (SPT_COUNT_RAYS).

Every pixel is independent (own RNG words, own accumulator: smallptCPU.cpp:
84-123), so any partition of the frame's tile groups rendered list by list
must give the full-frame render's bits -- which the other GPU tests pin to
the reference (oracle, reference-core goldens)."""
import ctypes as C

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _scene(rt, kind, w, h):
    if kind == "cornell":
        S, n = rt.scenes.cornell()
        return S, n, rt.scenes.cornell_camera(w, h)
    S, n, cam = rt.scenes.complex10k()
    rt.scenes.update_camera(cam, w, h)
    return S, n, cam


class _Frame:
    def __init__(self, torch, dev, w, h, seeds0):
        self.col = torch.zeros(3 * w * h, dtype=torch.float32, device=dev)
        self.seeds = torch.zeros_like(seeds0)
        self.px = torch.zeros(w * h, dtype=torch.int32, device=dev)
        self.cnt = torch.zeros(4, dtype=torch.int64, device=dev)

    def same(self, o, torch):
        return (torch.equal(self.col.view(torch.int32), o.col.view(torch.int32)) and torch.equal(self.seeds, o.seeds)
                and torch.equal(self.px, o.px))


@pytest.mark.parametrize("kind,w,h,spp,env", [
    ("cornell", 200, 120, 3, {}),
    ("cornell", 197, 61, 2, {}),                          # ragged: groups straddle tile rows
    ("complex", 320, 180, 2, {}),                         # 8-wide hierarchy (persistent waves)
    ("complex", 320, 180, 2, {"RT_SPT_WIDE": "0"}),       # binary hierarchy (staged group stores)
    ("complex", 250, 130, 2, {"RT_SPT_WIDE": "0"}),
])
def test_lists_partition_the_frame(rt, monkeypatch, kind, w, h, spp, env):
    """A random partition of the frame's tile groups into 3 lists (random
    order within each), rendered list by list into one frame == one
    full-frame render: colours, seeds, pixels bit for bit, counters summed
    (full and rays-only).  Entries outside [0, groups) are skipped."""
    import torch
    from rtamd import dist as rd
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    S, n, cam = _scene(rt, kind, w, h)
    sc = rt.SmallptScene(S, n)
    dev = torch.device("cuda", 0)
    seeds0 = torch.from_numpy(rt.scenes.seeds(w, h).view(np.int32)).to(dev)
    st = torch.cuda.current_stream(dev).cuda_stream
    L = rt.lib()
    ng = L.spt_group_count(w, h)
    assert ng == rd.group_count(w, h)
    ref = _Frame(torch, dev, w, h, seeds0)
    rt.check(L.spt_scene_render_async(sc.handle, C.byref(cam), ref.col.data_ptr(), seeds0.data_ptr(),
                                      ref.seeds.data_ptr(), ref.px.data_ptr(), w, h, 0, h, 0, spp, 0,
                                      ref.cnt.data_ptr(), st))
    rng = np.random.default_rng(w + h)
    perm = rng.permutation(ng)
    cuts = sorted(rng.choice(np.arange(1, ng), 2, replace=False))
    lists = [perm[:cuts[0]], perm[cuts[0]:cuts[1]], perm[cuts[1]:]]
    for mode in (0, rt.SPT_COUNT_RAYS, rt.SPT_LIST_SET):
        got = _Frame(torch, dev, w, h, seeds0)
        got.cnt[2] = 12345                                 # rays-only leaves counters[2] untouched
        for i, lst in enumerate(lists):
            # out-of-range entries: skipped (SPT_LIST_SET: the caller promises none, and no dedup pass runs)
            lst = list(lst) + ([-7, ng, 1 << 30] if i == 1 and mode != rt.SPT_LIST_SET else [])
            d = torch.tensor(lst, dtype=torch.int32, device=dev)
            rt.check(L.spt_scene_render_list_async(sc.handle, C.byref(cam), got.col.data_ptr(), seeds0.data_ptr(),
                                                   got.seeds.data_ptr(), got.px.data_ptr(), w, h, d.data_ptr(),
                                                   len(lst), 0, spp, mode, got.cnt.data_ptr(), None, st))
        torch.cuda.synchronize()
        assert got.same(ref, torch), mode
        c, r = got.cnt.tolist(), ref.cnt.tolist()
        if mode == rt.SPT_COUNT_RAYS:
            assert (c[0], c[1], c[3]) == (r[0], r[1], r[3]) and c[2] == 12345, (c, r)
        else:
            assert c == [r[0], r[1], r[2] + 12345, r[3]], (c, r)


def test_list_costs_and_bad_arguments(rt):
    """d_group_cost gets a positive wave time for every listed group of a
    hierarchy scene and nothing for the others; a list longer than the
    frame's group count is refused."""
    import torch
    w, h = 320, 180
    S, n, cam = _scene(rt, "complex", w, h)
    sc = rt.SmallptScene(S, n)
    dev = torch.device("cuda", 0)
    seeds0 = torch.from_numpy(rt.scenes.seeds(w, h).view(np.int32)).to(dev)
    st = torch.cuda.current_stream(dev).cuda_stream
    L = rt.lib()
    ng = L.spt_group_count(w, h)
    f = _Frame(torch, dev, w, h, seeds0)
    lst = list(range(0, ng, 3))
    d = torch.tensor(lst, dtype=torch.int32, device=dev)
    cost = torch.zeros(ng, dtype=torch.int32, device=dev)
    for cbuf in (None, cost):                 # (a warm-up launch first: the timed ones compare)
        rt.check(L.spt_scene_render_list_async(sc.handle, C.byref(cam), f.col.data_ptr(), seeds0.data_ptr(),
                                               f.seeds.data_ptr(), f.px.data_ptr(), w, h, d.data_ptr(), len(lst), 0,
                                               2, 0, None, cbuf.data_ptr() if cbuf is not None else None, st))
    torch.cuda.synchronize()
    c = cost.cpu().numpy()
    mask = np.zeros(ng, bool)
    mask[lst] = True
    assert (c[mask] > 0).all() and (c[~mask] == 0).all()
    # SPT_COST_MAX: each listed group's longest tile instead of the sum of its
    # (up to four) tiles -- over all groups well below the sums and above a
    # quarter of them (two launches' wave times, so only in aggregate); the
    # same frame
    cmax = torch.zeros(ng, dtype=torch.int32, device=dev)
    f2 = _Frame(torch, dev, w, h, seeds0)
    rt.check(L.spt_scene_render_list_async(sc.handle, C.byref(cam), f2.col.data_ptr(), seeds0.data_ptr(),
                                           f2.seeds.data_ptr(), f2.px.data_ptr(), w, h, d.data_ptr(), len(lst), 0, 2,
                                           rt.SPT_COST_MAX, None, cmax.data_ptr(), st))
    torch.cuda.synchronize()
    m = cmax.cpu().numpy().astype(np.int64)
    assert (m[mask] > 0).all() and (m[~mask] == 0).all()
    ratio = m[mask].sum() / c[mask].sum()
    assert 0.15 < ratio < 0.9, ratio
    assert torch.equal(f2.col.view(torch.int32), f.col.view(torch.int32)) and torch.equal(f2.px, f.px)
    # Full counters (the refilling kernel: a lane's unit is a pixel): the sum
    # of each group's pixel durations, or with SPT_COST_MAX the longest one --
    # which no launch can exceed (100 MHz ticks against the launch's own
    # duration), while a sum over a group's pixels far exceeds its max.
    csum = torch.zeros(ng, dtype=torch.int32, device=dev)
    cmx = torch.zeros(ng, dtype=torch.int32, device=dev)
    cnt = torch.zeros(4, dtype=torch.int64, device=dev)
    for mode, cb in ((0, csum), (rt.SPT_COST_MAX, cmx)):
        f3 = _Frame(torch, dev, w, h, seeds0)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        rt.check(L.spt_scene_render_list_async(sc.handle, C.byref(cam), f3.col.data_ptr(), seeds0.data_ptr(),
                                               f3.seeds.data_ptr(), f3.px.data_ptr(), w, h, d.data_ptr(), len(lst), 0,
                                               2, mode, cnt.data_ptr(), cb.data_ptr(), st))
        e1.record()
        torch.cuda.synchronize()
        assert torch.equal(f3.col.view(torch.int32), f.col.view(torch.int32)) and torch.equal(f3.px, f.px)
    launch_ticks = e0.elapsed_time(e1) * 1e5
    s, mx = csum.cpu().numpy().astype(np.int64), cmx.cpu().numpy().astype(np.int64)
    assert (mx[mask] > 0).all() and (mx[~mask] == 0).all() and (s[mask] > 0).all()
    assert mx.max() <= 1.05 * launch_ticks + 1000, (mx.max(), launch_ticks)
    assert mx[mask].sum() < 0.5 * s[mask].sum(), (mx[mask].sum(), s[mask].sum())
    assert L.spt_scene_render_list_async(sc.handle, C.byref(cam), f2.col.data_ptr(), seeds0.data_ptr(),
                                         f2.seeds.data_ptr(), f2.px.data_ptr(), w, h, d.data_ptr(), len(lst), 0, 1,
                                         0x400, None, None, st) == rt._lib.RT_ERR_INVALID
    big = torch.zeros(ng + 1, dtype=torch.int32, device=dev)
    assert L.spt_scene_render_list_async(sc.handle, C.byref(cam), f.col.data_ptr(), seeds0.data_ptr(),
                                         f.seeds.data_ptr(), f.px.data_ptr(), w, h, big.data_ptr(), ng + 1, 0, 1, 0,
                                         None, None, st) == rt._lib.RT_ERR_INVALID


@pytest.mark.parametrize("kind", ["cornell", "complex"])
def test_list_repeated_entries_render_once(rt, kind):
    """A list naming groups more than once (and out-of-range entries) is
    taken as a set: the frame equals the same groups listed once (a group
    rendered twice with first_sample > 0 would fold its samples into the
    accumulator twice), so do the counters, and each group's wave time is
    added to its cost entry once (a repeat would roughly double it).  The
    whole frame as a list equals the full-frame render."""
    import torch
    w, h = 160, 96
    S, n, cam = _scene(rt, kind, w, h)
    sc = rt.SmallptScene(S, n)
    dev = torch.device("cuda", 0)
    seeds0 = torch.from_numpy(rt.scenes.seeds(w, h).view(np.int32)).to(dev)
    st = torch.cuda.current_stream(dev).cuda_stream
    L = rt.lib()
    ng = L.spt_group_count(w, h)

    def frame(lst, cost=None):
        f = _Frame(torch, dev, w, h, seeds0)
        if lst is None:
            rt.check(L.spt_scene_render_async(sc.handle, C.byref(cam), f.col.data_ptr(), seeds0.data_ptr(),
                                              f.seeds.data_ptr(), f.px.data_ptr(), w, h, 0, h, 0, 2, 0,
                                              f.cnt.data_ptr(), st))
            rt.check(L.spt_scene_render_async(sc.handle, C.byref(cam), f.col.data_ptr(), f.seeds.data_ptr(),
                                              f.seeds.data_ptr(), f.px.data_ptr(), w, h, 0, h, 2, 2, 0,
                                              f.cnt.data_ptr(), st))
        else:
            d = torch.tensor(lst, dtype=torch.int32, device=dev)
            rt.check(L.spt_scene_render_list_async(sc.handle, C.byref(cam), f.col.data_ptr(), seeds0.data_ptr(),
                                                   f.seeds.data_ptr(), f.px.data_ptr(), w, h, d.data_ptr(),
                                                   len(lst), 0, 2, 0, f.cnt.data_ptr(), None, st))
            rt.check(L.spt_scene_render_list_async(sc.handle, C.byref(cam), f.col.data_ptr(), f.seeds.data_ptr(),
                                                   f.seeds.data_ptr(), f.px.data_ptr(), w, h, d.data_ptr(),
                                                   len(lst), 2, 2, 0, f.cnt.data_ptr(),
                                                   cost.data_ptr() if cost is not None else None, st))
        torch.cuda.synchronize()
        return f

    ref = frame(None)
    rng = np.random.default_rng(5)
    base = [int(g) for g in rng.permutation(ng)]
    assert frame(base).same(ref, torch)
    cover = base[: ng // 2]                        # half the frame, then repeats (a list is <= ng long)
    lst = cover + [int(g) for g in rng.choice(cover, ng // 4)] + [-1, ng]
    rng.shuffle(lst)
    c1 = torch.zeros(ng, dtype=torch.int32, device=dev)
    c2 = torch.zeros(ng, dtype=torch.int32, device=dev)
    once = frame(cover, c1)
    got = frame(lst, c2)
    assert got.same(once, torch) and got.cnt.tolist() == once.cnt.tolist()
    if kind == "complex":                     # costs are recorded by the hierarchy kernels
        a, b = c1.cpu().numpy().astype(np.float64)[cover], c2.cpu().numpy().astype(np.float64)[cover]
        assert (a > 0).all() and (b > 0).all()
        assert np.median(b / a) < 1.5, np.median(b / a)


@pytest.mark.parametrize("w,h", [(1920, 1080), (197, 61), (33, 9)])
def test_groups_pack_unpack(rt, w, h):
    """spt_groups_pack_async == the host-side slot map (rtamd.dist.group_slots)
    with 0 for pixels outside the frame; unpacking into a cleared frame
    restores exactly the listed groups' slots and nothing else."""
    import torch
    from rtamd import dist as rd
    dev = torch.device("cuda", 0)
    st = torch.cuda.current_stream(dev).cuda_stream
    L = rt.lib()
    ng = rd.group_count(w, h)
    rng = np.random.default_rng(w)
    col = torch.from_numpy(rng.standard_normal(3 * w * h).astype(np.float32)).to(dev)
    lst = rng.permutation(ng)[: max(1, ng // 3)]
    d = torch.tensor(lst, dtype=torch.int32, device=dev)
    buf = torch.full((len(lst) * 768,), 7.0, dtype=torch.float32, device=dev)
    rt.check(L.spt_groups_pack_async(col.data_ptr(), w, h, d.data_ptr(), len(lst), buf.data_ptr(), st))
    torch.cuda.synchronize()
    slots = rd.group_slots(lst, w, h)                                    # [n, 256]
    c3 = col.cpu().numpy().reshape(-1, 3)
    want = np.where((slots >= 0)[..., None], c3[np.maximum(slots, 0)], 0).astype(np.float32)
    assert (buf.cpu().numpy().view(np.uint32) == want.reshape(-1).view(np.uint32)).all()
    out = torch.zeros_like(col)
    rt.check(L.spt_groups_unpack_async(out.data_ptr(), w, h, d.data_ptr(), len(lst), buf.data_ptr(), st))
    torch.cuda.synchronize()
    o3 = out.cpu().numpy().reshape(-1, 3)
    m = np.zeros(w * h, bool)
    m[slots[slots >= 0]] = True
    assert (o3[m].view(np.uint32) == c3[m].view(np.uint32)).all() and (o3[~m] == 0).all()


@pytest.mark.parametrize("kind,env", [("cornell", {}), ("complex", {}), ("complex", {"RT_SPT_WIDE": "0"})])
def test_count_rays_mode(rt, monkeypatch, kind, env):
    """SPT_COUNT_RAYS: the same frame, and Intersect / IntersectP calls and
    samples equal to the full counters (SURVEY §8(d)'s ray count), with the
    uncounted queries; counters[2] is left as it was."""
    import torch
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    w, h = 240, 136
    S, n, cam = _scene(rt, kind, w, h)
    sc = rt.SmallptScene(S, n)
    dev = torch.device("cuda", 0)
    seeds0 = torch.from_numpy(rt.scenes.seeds(w, h).view(np.int32)).to(dev)
    st = torch.cuda.current_stream(dev).cuda_stream
    L = rt.lib()
    fr = []
    for mode in (0, rt.SPT_COUNT_RAYS, rt.SPT_COUNT_RAYS | rt.SPT_DIRECT_LIGHTING, rt.SPT_DIRECT_LIGHTING):
        f = _Frame(torch, dev, w, h, seeds0)
        f.cnt[2] = -1
        rt.check(L.spt_scene_render_async(sc.handle, C.byref(cam), f.col.data_ptr(), seeds0.data_ptr(),
                                          f.seeds.data_ptr(), f.px.data_ptr(), w, h, 0, h, 0, 3, mode,
                                          f.cnt.data_ptr(), st))
        torch.cuda.synchronize()
        fr.append(f)
    for a, b in ((fr[0], fr[1]), (fr[3], fr[2])):
        assert a.same(b, torch)
        ca, cb = a.cnt.tolist(), b.cnt.tolist()
        assert (ca[0], ca[1], ca[3]) == (cb[0], cb[1], cb[3]) and cb[2] == -1 and ca[2] > 0, (ca, cb)
    assert L.spt_scene_render_async(sc.handle, C.byref(cam), fr[0].col.data_ptr(), seeds0.data_ptr(),
                                    fr[0].seeds.data_ptr(), fr[0].px.data_ptr(), w, h, 0, h, 0, 1, 0x400, None,
                                    st) == rt._lib.RT_ERR_INVALID      # (0x200 is SPT_COST_MAX)
