"""Row-band sharding of one smallpt frame over the ranks of a node.

SURVEY.md §8(e): every pixel is independent (own RNG words, own accumulator),
so a frame splits into row bands with no data-path exchange; the only
collective assembles the frame on every rank after a render call.  Splitting
samples of a pixel over GPUs is NOT done: it would break the per-pixel RNG
chain and the running-average order the parity contract pins.

Band layout: rank k owns the k-th contiguous chunk of the FLIPPED colour /
seed slots ((h-y-1)*w + x, smallptCPU.cpp:86), i.e. pixel rows
[h-(k+1)B, h-kB) with B = h/world.  Its HDR band is then chunk k, in rank
order, of the colour buffer, so the whole accumulator is assembled by ONE
in-place all-gather (RCCL over xGMI with backend "nccl", gloo on CPU).  The
RGBA8 frame is not sent at all: every rank rebuilds it from the gathered
colours with the same toInt pack the kernel ends with (pack callback:
spt_pack_pixels_async on the GPU), bit-identical to the bands the other ranks
wrote.  Without a pack callback (CPU tests) the pixel bands are all-gathered
too.

Interleaved layout (GroupGather, the default of bench.py for N > 1): rank k
renders the 8-row groups k, k + world, k + 2*world, ...
(spt_scene_render_groups_async).  Contiguous bands differ in cost with their
content (at N = 4 the band holding the glass sphere takes 5.8 ms, the others
5.2 ms); interleaved groups give every GPU the same mix.  The shares are
packed into one padded buffer each, all-gathered once, and scattered back
into the frame (exact copies).

Group lists (ListGather, bench.py's configs[4] line): rank k renders an
explicit list of tile groups (spt_scene_render_list_async), balanced on the
per-group wave times of one learning frame (balanced_partition); shares are
packed per group (spt_groups_pack_async), all-gathered once and unpacked.
"""
import torch
import torch.distributed as dist


def row_band(rank, world, h):
    """Rows [r0, r1) rendered by `rank` (h must divide by world)."""
    if h % world:
        raise ValueError("frame height %d does not split into %d equal bands" % (h, world))
    B = h // world
    r0 = h - (rank + 1) * B
    return r0, r0 + B


class FrameGather:
    """Assembles a full frame -- colors (float32[3*w*h]) and pixels
    (int32[w*h]) -- on every rank from the per-rank row bands."""

    def __init__(self, colors, pixels, rank, world, w, h, pack=None):
        self.rank, self.world, self.w, self.h = rank, world, w, h
        self.colors, self.pixels, self.pack = colors, pixels, pack
        B = h // world
        self.my_col = colors.view(world, 3 * B * w)[rank]
        self.px_parts = [pixels[(h - (k + 1) * B) * w:(h - k * B) * w] for k in range(world)]
        self.my_px = self.px_parts[rank]

    def gather(self, group=None):
        """Every rank ends with the whole frame."""
        if self.world == 1:
            return
        dist.all_gather_into_tensor(self.colors, self.my_col.clone(), group=group)
        if self.pack is not None:
            self.pack()
        else:
            dist.all_gather(self.px_parts, self.my_px.clone(), group=group)


def gather_seeds(seeds, rank, world, w, h, group=None):
    """All-gather the per-rank RNG bands (uint32 viewed as int32 [2*w*h]) --
    needed only to hand the full progressive state to another owner."""
    if world == 1:
        return
    B = h // world
    dist.all_gather_into_tensor(seeds, seeds.view(world, 2 * B * w)[rank].clone(), group=group)


def group_rows(rank, world, h):
    """Pixel rows of `rank` in the interleaved split: the 8-row groups g with
    g % world == rank (the window of spt_scene_render_groups_async)."""
    return [y for g in range(rank, (h + 7) // 8, world) for y in range(8 * g, min(8 * g + 8, h))]


class GroupGather:
    """FrameGather for the interleaved split: every rank ends with the whole
    frame -- colors (float32[3*w*h], flipped slots) and pixels (int32[w*h])."""

    def __init__(self, colors, pixels, rank, world, w, h, pack=None):
        self.rank, self.world, self.w, self.h = rank, world, w, h
        self.pack = pack
        dev = colors.device
        rows = [group_rows(k, world, h) for k in range(world)]
        self.maxr = max(len(r) for r in rows)
        self.col2d = colors.view(h, 3 * w)                 # row h-1-y holds pixel row y
        self.px2d = pixels.view(h, w)
        slot = lambda k: torch.tensor([h - 1 - y for y in rows[k]], dtype=torch.long, device=dev)  # noqa: E731
        self.my_slots = slot(rank)
        self.my_rows = torch.tensor(rows[rank], dtype=torch.long, device=dev)
        self.all_slots = torch.cat([slot(k) for k in range(world)])
        self.all_rows = torch.tensor([y for k in range(world) for y in rows[k]], dtype=torch.long, device=dev)
        self.valid = torch.tensor([k * self.maxr + j for k in range(world) for j in range(len(rows[k]))],
                                  dtype=torch.long, device=dev)
        self.n_mine = len(rows[rank])
        self.send = torch.zeros(self.maxr, 3 * w, dtype=colors.dtype, device=dev)
        self.recv = torch.empty(world * self.maxr, 3 * w, dtype=colors.dtype, device=dev)
        if pack is None:
            self.psend = torch.zeros(self.maxr, w, dtype=pixels.dtype, device=dev)
            self.precv = torch.empty(world * self.maxr, w, dtype=pixels.dtype, device=dev)

    def gather(self, group=None):
        if self.world == 1:
            return
        torch.index_select(self.col2d, 0, self.my_slots, out=self.send[:self.n_mine])
        dist.all_gather_into_tensor(self.recv, self.send, group=group)
        self.col2d.index_copy_(0, self.all_slots, self.recv.index_select(0, self.valid))
        if self.pack is not None:
            self.pack()
        else:
            torch.index_select(self.px2d, 0, self.my_rows, out=self.psend[:self.n_mine])
            dist.all_gather_into_tensor(self.precv, self.psend, group=group)
            self.px2d.index_copy_(0, self.all_rows, self.precv.index_select(0, self.valid))


# ---------------------------------------------------------------------------
# Explicit tile-group lists (spt_scene_render_list_async): a frame split by
# measured cost.  Group g = the 8x8 tiles 4g .. 4g+3 in row-major tile order
# (include/rt_hip.h spt_group_count).  Interleaved row groups balance a frame
# whose cost is spread evenly (Cornell), but a scene whose cost sits in a few
# tiles (configs[4]: per-tile work varies 6x, the heaviest tiles set the
# frame) leaves ranks unequal; one frame's per-group wave times, summed over
# the ranks, give every rank the same inputs for the same deterministic
# partition.

def group_count(w, h):
    """spt_group_count(w, h) without the library."""
    return ((w + 7) // 8 * ((h + 7) // 8) + 3) // 4


def interleaved_groups(rank, world, w, h):
    """Groups of the interleaved split (8-row groups rank, rank + world, ...)
    as a group list: the groups whose tiles lie in those rows.  With
    ceil(w/8) a multiple of 4 a group is one 32x8 strip of one 8-row group;
    otherwise a group straddling two rows goes to the owner of its first."""
    tx = (w + 7) // 8
    return [g for g in range(group_count(w, h)) if ((4 * g) // tx) % world == rank]


def balanced_partition(costs, world, order_key=None):
    """Deterministic longest-processing-time split of the groups over `world`
    ranks: groups in decreasing cost (ties: lower index first), each to the
    rank with the least total so far (ties: lower rank).  Returns per rank
    its groups in that order -- heaviest first, which is also the dispatch
    order spt_scene_render_list_async wants -- or, with `order_key` (per
    group, e.g. its longest tile: SPT_COST_MAX), each rank's groups sorted by
    decreasing key (ties: lower index first), so the groups holding the
    longest pixel chains take the list's heavy-tile slots.  Every rank
    computes the same lists from the same (all-reduced) costs."""
    import heapq
    order = sorted(range(len(costs)), key=lambda g: (-int(costs[g]), g))
    heap = [(0, r) for r in range(world)]
    parts = [[] for _ in range(world)]
    for g in order:
        load, r = heapq.heappop(heap)
        parts[r].append(g)
        heapq.heappush(heap, (load + int(costs[g]), r))
    if order_key is not None:
        parts = [sorted(p, key=lambda g: (-int(order_key[g]), g)) for p in parts]
    return parts


def group_slots(groups, w, h):
    """Accumulator slots ((h-y-1)*w + x, -1 outside the frame) of the listed
    groups, 256 per group in spt_groups_pack_async's order (CPU helper: the
    tests' host-side pack)."""
    import numpy as np
    tx = (w + 7) // 8
    g = np.asarray(groups, dtype=np.int64)[:, None]
    q = np.arange(256, dtype=np.int64)[None, :]
    tile = 4 * g + q // 64
    p = q % 64
    x = (tile % tx) * 8 + (p & 7)
    y = (tile // tx) * 8 + (p >> 3)
    ok = (x < w) & (y < h)
    return np.where(ok, (h - 1 - y) * w + x, -1)


class ListGather:
    """Assembles the whole frame on every rank when rank k rendered the
    groups lists[k] (spt_scene_render_list_async): each rank packs its
    groups' accumulator (768 floats a group), one all-gather of the shares
    padded to the longest list, every rank unpacks the others' shares, then
    repacks the RGBA8 frame from the colours (pack callback).

    pack / unpack: callables (colors, groups_tensor, n, buf) doing
    spt_groups_pack_async / spt_groups_unpack_async on the GPU; without them
    (CPU tensors, tests) torch index copies do the same."""

    def __init__(self, colors, pixels, rank, world, w, h, lists, pack=None, pack_groups=None,
                 unpack_groups=None):
        self.rank, self.world, self.w, self.h = rank, world, w, h
        self.colors, self.pixels, self.pack = colors, pixels, pack
        self.pack_groups, self.unpack_groups = pack_groups, unpack_groups
        if len(lists) != world:
            raise ValueError("ListGather: %d lists for %d ranks" % (len(lists), world))
        flat = [int(g) for x in lists for g in x]
        ng = group_count(w, h)
        if len(set(flat)) != len(flat) or any(not 0 <= g < ng for g in flat):
            # a group owned twice would be unpacked from two shares in rank
            # order: the frame would depend on which rank unpacks last
            raise ValueError("ListGather: the lists must be disjoint sets of groups in [0, %d)" % ng)
        dev = colors.device
        self.maxn = max(len(x) for x in lists)
        self.counts = [len(x) for x in lists]
        pad = [list(x) + [-1] * (self.maxn - len(x)) for x in lists]   # -1: skipped by pack / unpack
        self.all_groups = torch.tensor(pad, dtype=torch.int32, device=dev)   # [world, maxn]
        self.mine = self.all_groups[rank].contiguous()
        self.send = torch.zeros(self.maxn * 768, dtype=colors.dtype, device=dev)
        self.recv = torch.empty(world * self.maxn * 768, dtype=colors.dtype, device=dev)
        if pack_groups is None:
            import numpy as np
            sl = [group_slots(x, w, h) if len(x) else np.zeros((0, 256), np.int64) for x in lists]
            self._slots = [torch.from_numpy(s).to(dev) for s in sl]

    def _host_pack(self, k, buf):
        s = self._slots[k]
        if s.numel() == 0:
            return
        c3 = self.colors.view(-1, 3)
        v = torch.where((s >= 0)[..., None], c3[s.clamp(min=0)], torch.zeros((), dtype=self.colors.dtype))
        buf[:v.numel()] = v.reshape(-1)

    def _host_unpack(self, k, buf):
        s = self._slots[k]
        if s.numel() == 0:
            return
        c3 = self.colors.view(-1, 3)
        v = buf[:s.numel() * 3].view(-1, 256, 3)
        ok = s >= 0
        c3[s[ok]] = v[ok]

    def gather(self, group=None):
        if self.world == 1:
            return
        if self.pack_groups is not None:
            self.pack_groups(self.colors, self.mine, self.counts[self.rank], self.send)
        else:
            self._host_pack(self.rank, self.send)
        dist.all_gather_into_tensor(self.recv, self.send, group=group)
        parts = self.recv.view(self.world, self.maxn * 768)
        for k in range(self.world):
            if k == self.rank or self.counts[k] == 0:
                continue
            if self.unpack_groups is not None:
                self.unpack_groups(self.colors, self.all_groups[k], self.counts[k], parts[k])
            else:
                self._host_unpack(k, parts[k])
        if self.pack is not None:
            self.pack()
        else:
            raise RuntimeError("ListGather without a pixel pack callback: give pack=")
