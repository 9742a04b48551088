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
