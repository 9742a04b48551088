"""smallpt frames over DISTINCT physical GPUs (BASELINE
configs[3] "tiled across 2/4/8", configs[4] "8xMI355X").

Every test here needs at least two visible gfx950 devices and skips
otherwise, so a one-GPU box reports them as skipped and the first box with
several GPUs runs the multi-device code automatically:

  * spt_render_multi over devices 0..N-1 (one host thread, one stream per
    device, row bands) against the reference-core golden of the full frame;
  * SmallptMulti with RT_SPT_GATHER=rccl: progressive passes per band, then
    the one in-place ncclAllGather of the padded bands (spt_multi.hip) --
    every device must then hold the single-GPU frame;
  * the tile-group-list split of configs[4] (spt_scene_render_list_async,
    one scene per device, lists from balanced_partition over a learning
    frame's measured costs) against the configs[4] golden;
  * one process per GPU over torch.distributed "nccl" (RCCL over xGMI):
    bench.py's interleaved split (GroupGather) and list split (ListGather)
    assembling the frame on every rank, checked against the goldens.

N = min(8, device count).  The one-GPU repeated-device forms of the same
code are in test_gpu_multi.py / test_gpu_lists.py."""
import ctypes as C
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
GOLDEN = json.load(open(os.path.join(HERE, "golden", "known_answers.json")))["smallpt"]


def _ndev(rt):
    n = min(8, rt.device_count())
    if n < 2:
        pytest.skip("needs >= 2 distinct GPUs (this box has %d)" % rt.device_count())
    return n


def test_render_multi_distinct_devices_golden(rt, oracle):
    """BASELINE configs[3]'s decomposition on real devices: the Cornell
    1920x1080 64-spp frame in N row bands on devices 0..N-1 (spt_render_multi)
    == the reference core's golden hashes (colours, pixels, seeds)."""
    n = _ndev(rt)
    g = GOLDEN["1920x1080_64spp"]
    f = rt.SmallptFrame(1920, 1080)
    f.render(64, counters=False, devices=list(range(n)))
    assert (oracle.fnv1a64(f.colors), oracle.fnv1a64(f.pixels), oracle.fnv1a64(f.seeds)) == \
        (g["colors"], g["pixels"], g["seeds"])


def test_multi_rccl_gather_distinct_devices(rt, monkeypatch):
    """spt_multi_* over N distinct devices with the RCCL gather: three
    progressive passes, the in-place all-gather of the ceil(h/N)-row padded
    bands, a second frame after it; every device's assembled frame (HDR +
    repacked RGBA8) == the one-GPU frame, and the counters sum to its
    counters.  h = 190 is not a multiple of N, so the last band is short."""
    n = _ndev(rt)
    monkeypatch.setenv("RT_SPT_GATHER", "rccl")
    w, h = 256, 190
    cam = rt.scenes.cornell_camera(w, h)
    m = rt.SmallptMulti(w, h, list(range(n)))
    B = -(-h // n)
    assert m.rows == [min(h, k * B) for k in range(n)] + [h]
    m.upload(rt.scenes.seeds(w, h))
    for k in range(3):
        m.render(cam, k, 1, counters=True)
    m.gather()
    m.sync()
    ref = rt.SmallptFrame(w, h).render(3)
    for k in range(n):
        col, px = m.read_frame(k)
        assert (col.view(np.uint32) == ref.colors.view(np.uint32)).all(), k
        assert (px == ref.pixels).all(), k
    assert m.counters() == ref.counters
    m.render(cam, 3, 2)
    m.gather()
    m.sync()
    ref.render(2)
    for k in range(n):
        col, px = m.read_frame(k)
        assert (col.view(np.uint32) == ref.colors.view(np.uint32)).all() and (px == ref.pixels).all(), k
    m.close()


def test_configs4_lists_distinct_devices_golden(rt, oracle):
    """BASELINE configs[4] (10k spheres, 1920x1080, 64 spp) split over N
    devices by measured cost, all devices rendering at once from one host
    thread: a learning frame of the interleaved group lists records each
    group's wave time, balanced_partition splits the groups, every device
    renders its list (heaviest first, cooperative heavy tiles), and the
    assembled frame == the reference core's golden."""
    import torch
    from rtamd import dist as rd
    n = _ndev(rt)
    g = GOLDEN["1920x1080_64spp_complex10k"]
    w, h = 1920, 1080
    S, ns, cam = rt.scenes.complex10k()
    rt.scenes.update_camera(cam, w, h)
    L = rt.lib()
    ng = rd.group_count(w, h)
    seeds_host = rt.scenes.seeds(w, h)
    per = []
    for k in range(n):
        rt.set_device(k)
        dev = torch.device("cuda", k)
        with torch.cuda.device(dev):
            per.append({"dev": dev, "sc": rt.SmallptScene(S, ns),
                        "seeds0": torch.from_numpy(seeds_host.view(np.int32)).to(dev),
                        "col": torch.zeros(3 * w * h, dtype=torch.float32, device=dev),
                        "px": torch.zeros(w * h, dtype=torch.int32, device=dev),
                        "cost": torch.zeros(ng, dtype=torch.int32, device=dev),
                        "st": torch.cuda.current_stream(dev)})
    for p in per:
        p["seeds"] = torch.empty_like(p["seeds0"])

    def render(k, lst, cost=None):
        p = per[k]
        rt.set_device(k)
        rt.check(L.spt_scene_render_list_async(p["sc"].handle, C.byref(cam), p["col"].data_ptr(),
                                               p["seeds0"].data_ptr(), p["seeds"].data_ptr(), p["px"].data_ptr(),
                                               w, h, lst.data_ptr(), lst.numel(), 0, 64, rt.SPT_PATH_TRACING, None,
                                               cost.data_ptr() if cost is not None else None,
                                               p["st"].cuda_stream))

    lists0 = [torch.tensor(rd.interleaved_groups(k, n, w, h), dtype=torch.int32, device=per[k]["dev"])
              for k in range(n)]
    for k in range(n):                                  # learning frame, all devices at once
        render(k, lists0[k], per[k]["cost"])
    costs = np.zeros(ng, np.int64)
    for k in range(n):
        torch.cuda.synchronize(per[k]["dev"])
        costs += per[k]["cost"].cpu().numpy().astype(np.int64)
    parts = rd.balanced_partition(costs, n)
    assert sorted(sum(parts, [])) == list(range(ng))
    lists = [torch.tensor(parts[k], dtype=torch.int32, device=per[k]["dev"]) for k in range(n)]
    for k in range(n):
        render(k, lists[k])
    col = np.zeros(3 * w * h, np.float32)
    seeds = np.zeros(2 * w * h, np.uint32)
    px = np.zeros(w * h, np.uint32)
    for k in range(n):
        torch.cuda.synchronize(per[k]["dev"])
        sl = rd.group_slots(parts[k], w, h)
        sl = sl[sl >= 0]                                # flipped slots (h-y-1)*w + x
        pi = (h - 1 - sl // w) * w + sl % w             # pixel index y*w + x
        c = per[k]["col"].cpu().numpy().reshape(-1, 3)
        s = per[k]["seeds"].cpu().numpy().view(np.uint32).reshape(-1, 2)
        p = per[k]["px"].cpu().numpy().view(np.uint32)
        col.reshape(-1, 3)[sl] = c[sl]
        seeds.reshape(-1, 2)[sl] = s[sl]
        px[pi] = p[pi]
    rt.set_device(0)
    assert (oracle.fnv1a64(col), oracle.fnv1a64(px), oracle.fnv1a64(seeds)) == (g["colors"], g["pixels"], g["seeds"])


WORKER = r'''
import ctypes as C, json, os, sys
sys.path[:0] = [%(pkg)r, %(tests)r]
import numpy as np, torch, torch.distributed as dist
import oracle_lib as O
import rtamd
from rtamd import dist as rd
rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
dev = torch.device("cuda", rank)
torch.cuda.set_device(dev)
dist.init_process_group("nccl", device_id=dev)
rtamd.set_device(rank)
L = rtamd.lib()
G = json.load(open(%(golden)r))["smallpt"]
W, H, SPP = 1920, 1080, 64
s = torch.cuda.current_stream(dev)
seeds0 = torch.from_numpy(rtamd.scenes.seeds(W, H).view(np.int32)).to(dev)
seeds = torch.empty_like(seeds0)
ok = True

def pack(col, px):
    return lambda: rtamd.check(L.spt_pack_pixels_async(col.data_ptr(), px.data_ptr(), W, H, 0, H,
                                                       torch.cuda.current_stream(dev).cuda_stream))

def check(col, px, key):
    torch.cuda.synchronize(dev)
    got = (O.fnv1a64(col.cpu().numpy()), O.fnv1a64(px.cpu().numpy()))
    return got == (G[key]["colors"], G[key]["pixels"])

# (1) Cornell, interleaved 8-row groups + GroupGather (bench.py's headline split)
S, n = rtamd.scenes.cornell()
cam = rtamd.scenes.cornell_camera(W, H)
sc = rtamd.SmallptScene(S, n)
col = torch.zeros(3 * W * H, dtype=torch.float32, device=dev)
px = torch.zeros(W * H, dtype=torch.int32, device=dev)
rtamd.check(L.spt_scene_render_groups_async(sc.handle, C.byref(cam), col.data_ptr(), seeds0.data_ptr(),
                                            seeds.data_ptr(), px.data_ptr(), W, H, rank, world, 0, SPP, 0, None,
                                            s.cuda_stream))
rd.GroupGather(col, px, rank, world, W, H, pack=pack(col, px)).gather()
ok = ok and check(col, px, "1920x1080_64spp")
print("RANK", rank, "groups", ok, flush=True)

# (2) configs[4], cost-balanced lists + ListGather (bench.py's configs4_tiled split)
S4, n4, cam4 = rtamd.scenes.complex10k()
rtamd.scenes.update_camera(cam4, W, H)
sc4 = rtamd.SmallptScene(S4, n4)
ng = rd.group_count(W, H)
cost = torch.zeros(ng, dtype=torch.int32, device=dev)
col.zero_(); px.zero_()

def render(lst, cost_buf=None):
    rtamd.check(L.spt_scene_render_list_async(sc4.handle, C.byref(cam4), col.data_ptr(), seeds0.data_ptr(),
                                              seeds.data_ptr(), px.data_ptr(), W, H, lst.data_ptr(), lst.numel(),
                                              0, SPP, 0, None, cost_buf.data_ptr() if cost_buf is not None else None,
                                              s.cuda_stream))

render(torch.tensor(rd.interleaved_groups(rank, world, W, H), dtype=torch.int32, device=dev), cost)
costs = cost.to(torch.int64)
dist.all_reduce(costs)
parts = rd.balanced_partition(costs.cpu().numpy(), world)
col.zero_(); px.zero_()
render(torch.tensor(parts[rank], dtype=torch.int32, device=dev))
pg = lambda c, g, k, b: rtamd.check(L.spt_groups_pack_async(c.data_ptr(), W, H, g.data_ptr(), k, b.data_ptr(),
                                                              torch.cuda.current_stream(dev).cuda_stream))
ug = lambda c, g, k, b: rtamd.check(L.spt_groups_unpack_async(c.data_ptr(), W, H, g.data_ptr(), k, b.data_ptr(),
                                                                torch.cuda.current_stream(dev).cuda_stream))
rd.ListGather(col, px, rank, world, W, H, parts, pack=pack(col, px), pack_groups=pg, unpack_groups=ug).gather()
ok4 = check(col, px, "1920x1080_64spp_complex10k")
print("RANK", rank, "lists", ok4, flush=True)
print("RANK", rank, "OK" if ok and ok4 else "MISMATCH", flush=True)
dist.destroy_process_group()
'''


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_nccl_ranks_assemble_golden_frames(rt, tmp_path):
    """One process per GPU over torch.distributed "nccl" (RCCL over xGMI),
    N = min(8, devices) ranks: the interleaved Cornell split (GroupGather)
    and the cost-balanced configs[4] list split (ListGather) must assemble
    the golden frames on every rank."""
    n = _ndev(rt)
    script = tmp_path / "w.py"
    script.write_text(WORKER % {"pkg": os.path.join(ROOT, "se-195-project-ray-tracer_amd"), "tests": HERE,
                                "golden": os.path.join(HERE, "golden", "known_answers.json")})
    port = _port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(n), LOCAL_RANK=str(r), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, "-u", str(script)], env=env, stdout=subprocess.PIPE,
                                      stderr=subprocess.STDOUT, text=True))
    try:
        outs = [p.communicate(timeout=100)[0] for p in procs]
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    for r, (p, o) in enumerate(zip(procs, outs)):
        assert p.returncode == 0, o
        assert "RANK %d OK" % r in o, o
