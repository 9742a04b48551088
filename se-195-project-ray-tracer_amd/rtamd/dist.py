"""Row-band sharding of one smallpt frame over the ranks of a node.

SURVEY.md §8(e): every pixel is independent (own RNG words, own accumulator),
so a frame splits into row bands with no data-path exchange; the only
collective is the assembly of the HDR accumulator (12 B/px) and the RGBA8
frame (4 B/px) on every rank -- two all-gathers per frame (RCCL over xGMI
with backend "nccl", gloo on CPU for tests).  Splitting samples of a pixel
over GPUs is NOT done: it would break the per-pixel RNG chain and the
running-average order the parity contract pins.

Band layout: rank k owns the k-th contiguous chunk of the FLIPPED colour /
seed slots ((h-y-1)*w + x, smallptCPU.cpp:86), i.e. pixel rows
[h-(k+1)B, h-kB) with B = h/world, so its colour band is one contiguous
all-gather piece in rank order and its pixel band is contiguous too.
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
    """Views of a full-frame colors (float32[3*w*h]) / pixels (int32[w*h])
    pair for in-place all-gather of the per-rank bands."""

    def __init__(self, colors, pixels, rank, world, w, h):
        self.rank, self.world, self.w, self.h = rank, world, w, h
        B = h // world
        self.col_parts = list(colors.view(world, 3 * B * w).unbind(0))
        self.px_parts = [pixels[(h - (k + 1) * B) * w:(h - k * B) * w] for k in range(world)]
        self.my_col = self.col_parts[rank]
        self.my_px = self.px_parts[rank]

    def gather(self, group=None):
        """Every rank ends with the whole frame.  The own band is passed as a
        copy (the output list aliases it)."""
        if self.world == 1:
            return
        dist.all_gather(self.col_parts, self.my_col.clone(), group=group)
        dist.all_gather(self.px_parts, self.my_px.clone(), group=group)


def gather_seeds(seeds, rank, world, w, h, group=None):
    """All-gather the per-rank RNG bands (uint32 viewed as int32 [2*w*h]) --
    needed only to hand the full progressive state to another owner."""
    if world == 1:
        return
    B = h // world
    parts = list(seeds.view(world, 2 * B * w).unbind(0))
    dist.all_gather(parts, parts[rank].clone(), group=group)
