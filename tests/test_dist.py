"""Multi-rank sharding (rtamd.dist) on CPU with gloo, world sizes 2 to 8
(the 8-GPU node's rank count): each rank renders its share -- a row band,
its interleaved 8-row groups, or a cost-balanced tile-group list -- with the
CPU oracle, the shares are all-gathered, and the assembled frame must equal
a single-rank render bit for bit (tiles are disjoint, so sharding is exact).
Ragged frames (h not a multiple of 8 x world) leave ranks with short or
empty shares."""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)

WORKER = r'''
import os, sys
sys.path[:0] = [%(pkg)r, %(tests)r]
import numpy as np, torch, torch.distributed as dist
import oracle_lib as O
from rtamd import dist as rd
rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
dist.init_process_group("gloo")
w, h, spp = %(w)d, %(h)d, 3
S, n = O.cornell(); cam = O.cornell_camera(w, h)
col = np.zeros(3 * w * h, np.float32); seeds = O.seeds(w, h); px = np.zeros(w * h, np.uint32)
tc, tp, ts = torch.from_numpy(col), torch.from_numpy(px.view(np.int32)), torch.from_numpy(seeds.view(np.int32))
if %(mode)r == "bands":
    r0, r1 = rd.row_band(rank, world, h)
    O.smallpt_render(S, n, cam, col, seeds, px, w, h, 0, spp, row_begin=r0, row_end=r1)
    g = rd.FrameGather(tc, tp, rank, world, w, h)
    g.gather()
    rd.gather_seeds(ts, rank, world, w, h)
elif %(mode)r == "lists":
    # cost-balanced group lists (balanced_partition over made-up costs): each
    # rank keeps only its groups of an oracle frame, then ListGather (host
    # pack / unpack) must rebuild the whole accumulator on every rank
    O.smallpt_render(S, n, cam, col, seeds, px, w, h, 0, spp)
    costs = [(g * 7919) %% 13 + (g %% 5 == 0) * 40 for g in range(rd.group_count(w, h))]
    parts = rd.balanced_partition(costs, world)
    keep = np.zeros(w * h, bool)
    sl = rd.group_slots(parts[rank], w, h)
    keep[sl[sl >= 0]] = True
    col.reshape(-1, 3)[~keep] = 0.0
    g = rd.ListGather(tc, tp, rank, world, w, h, parts, pack=lambda: None)
    g.gather()
    c2 = np.zeros_like(col); s2 = O.seeds(w, h); p2 = np.zeros_like(px)
    O.smallpt_render(S, n, cam, c2, s2, p2, w, h, 0, spp)
    ok = (col.view(np.uint32) == c2.view(np.uint32)).all() and sorted(sum(parts, [])) == list(range(rd.group_count(w, h)))
    print("RANK", rank, "OK" if ok else "MISMATCH", flush=True)
    dist.destroy_process_group()
    sys.exit(0)
else:
    for g0 in range(rank, (h + 7) // 8, world):         # this rank's 8-row groups
        O.smallpt_render(S, n, cam, col, seeds, px, w, h, 0, spp, row_begin=8 * g0, row_end=min(8 * g0 + 8, h))
    g = rd.GroupGather(tc, tp, rank, world, w, h)
    g.gather()
    # seeds: the same interleaved gather on a seeds-shaped view (2 words per pixel)
    sg = rd.GroupGather(torch.zeros(3 * w * h), torch.zeros(w * h, dtype=torch.int32), rank, world, w, h)
    mine = sg.my_slots
    s2d = ts.view(h, 2 * w)
    send = torch.zeros(sg.maxr, 2 * w, dtype=torch.int32); send[:sg.n_mine] = s2d.index_select(0, mine)
    recv = torch.empty(world * sg.maxr, 2 * w, dtype=torch.int32)
    dist.all_gather_into_tensor(recv, send)
    s2d.index_copy_(0, sg.all_slots, recv.index_select(0, sg.valid))
c2 = np.zeros_like(col); s2 = O.seeds(w, h); p2 = np.zeros_like(px)
O.smallpt_render(S, n, cam, c2, s2, p2, w, h, 0, spp)
ok = (col.view(np.uint32) == c2.view(np.uint32)).all() and (px == p2).all() and (seeds == s2).all()
print("RANK", rank, "OK" if ok else "MISMATCH", flush=True)
dist.destroy_process_group()
'''


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("world,mode,w,h", [
    (2, "bands", 48, 32), (4, "bands", 48, 32), (8, "bands", 48, 32),
    (2, "groups", 48, 32), (3, "groups", 48, 32),
    (8, "groups", 48, 32),      # 4 groups: ranks 4..7 render nothing and still join the gather
    (8, "groups", 40, 70),      # ragged: 9 groups, the last 6 rows (h not a multiple of 8 x 8)
    (2, "lists", 48, 32), (3, "lists", 48, 32), (8, "lists", 48, 32), (8, "lists", 40, 70)])
def test_band_gather_is_exact(tmp_path, world, mode, w, h):
    script = tmp_path / "w.py"
    script.write_text(WORKER % {"pkg": os.path.join(ROOT, "se-195-project-ray-tracer_amd"),
                                "tests": HERE, "mode": mode, "w": w, "h": h})
    port = _port()
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), LOCAL_RANK=str(r))
        procs.append(subprocess.Popen([sys.executable, str(script)], env=env, stdout=subprocess.PIPE,
                                      stderr=subprocess.STDOUT, text=True))
    outs = [p.communicate(timeout=240)[0] for p in procs]
    for r, (p, o) in enumerate(zip(procs, outs)):
        assert p.returncode == 0, o
        assert "RANK %d OK" % r in o, o


def test_group_rows_partition():
    from rtamd import dist as rd
    for world in (1, 2, 3, 4, 8):
        rows = sorted(y for k in range(world) for y in rd.group_rows(k, world, 1080))
        assert rows == list(range(1080))
    assert rd.group_rows(1, 4, 1080)[:9] == [8, 9, 10, 11, 12, 13, 14, 15, 40]


def test_row_band_layout():
    from rtamd import dist as rd
    bands = [rd.row_band(k, 8, 1080) for k in range(8)]
    assert bands[0] == (945, 1080) and bands[-1] == (0, 135)
    covered = sorted(r for a, b in bands for r in range(a, b))
    assert covered == list(range(1080))
    with pytest.raises(ValueError):
        rd.row_band(0, 7, 1080)


def test_balanced_partition_properties():
    """Every group exactly once; each rank's list in decreasing cost; the
    heaviest `world` groups on distinct ranks; loads within the largest
    single cost of each other (the longest-first greedy bound)."""
    import numpy as np
    from rtamd import dist as rd
    rng = np.random.default_rng(3)
    for world in (1, 2, 3, 8):
        costs = rng.integers(1, 1000, 8100) * (rng.random(8100) < 0.3) + 1
        parts = rd.balanced_partition(costs, world)
        assert sorted(sum(parts, [])) == list(range(8100))
        for p in parts:
            assert all(costs[a] >= costs[b] for a, b in zip(p, p[1:]))
        top = np.argsort(-costs, kind="stable")[:world]
        owner = {g: r for r, p in enumerate(parts) for g in p}
        assert len({owner[g] for g in top}) == world
        loads = [int(costs[p].sum()) for p in parts]
        assert max(loads) - min(loads) <= costs.max()
    assert rd.interleaved_groups(1, 4, 1920, 1080)[:3] == [60, 61, 62]


def test_balanced_partition_order_key():
    """order_key (a group's longest tile) reorders each rank's list by
    decreasing key (ties: lower index) without changing which groups a rank
    gets -- the loads stay balanced by the costs."""
    import numpy as np
    from rtamd import dist as rd
    rng = np.random.default_rng(5)
    costs = rng.integers(1, 1000, 4000)
    keys = rng.integers(1, 300, 4000)
    keys[rng.random(4000) < 0.5] = 7                       # many ties
    for world in (1, 2, 4, 8):
        plain = rd.balanced_partition(costs, world)
        keyed = rd.balanced_partition(costs, world, order_key=keys)
        for p, q in zip(plain, keyed):
            assert sorted(p) == sorted(q)
            assert all((-keys[a], a) < (-keys[b], b) for a, b in zip(q, q[1:]))


def test_list_gather_refuses_overlapping_lists():
    """ListGather's lists must partition groups: a group in two ranks' lists
    (or twice in one), or outside the frame, is refused up front."""
    import torch
    from rtamd import dist as rd
    w, h = 48, 32
    col, px = torch.zeros(3 * w * h), torch.zeros(w * h, dtype=torch.int32)
    ng = rd.group_count(w, h)
    rd.ListGather(col, px, 0, 2, w, h, [list(range(0, ng, 2)), list(range(1, ng, 2))], pack=lambda: None)
    for bad in ([[0, 1], [1, 2]], [[0, 0], [1]], [[0], [ng]], [[0], [-1]], [[0]]):
        with pytest.raises(ValueError):
            rd.ListGather(col, px, 0, 2, w, h, bad, pack=lambda: None)
    assert sum(len(rd.interleaved_groups(k, 3, 197, 61)) for k in range(3)) == rd.group_count(197, 61)
