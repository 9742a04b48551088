"""Per-basic-block instruction mix of one kernel in a gfx950 .s file.

    python tools/isa_blocks.py FILE.s KERNEL_SUBSTRING [--top N] [--grep OPCODE_PREFIX]

FILE.s comes from `hipcc --cuda-device-only -S` with the Makefile's flags.
Prints, per basic block: its label, the loop nesting depth (count of backward
branches whose range covers it), instruction totals by class (VALU, SALU,
VMEM, LDS, SMEM, branch, writelane/readlane = SGPR spill traffic through VGPR
lanes, scratch = VGPR spill traffic) and the hipcc source line (`.loc`) that
most of its instructions come from.  Used to find where spills and copies
land (DESIGN.md §3 "instruction budget").
"""
import argparse
import collections
import re


def classify(op):
    if op.startswith("v_writelane") or op.startswith("v_readlane"):
        return "lane"
    if op.startswith("scratch_") or op.startswith("buffer_store") and "off" in op:
        return "scratch"
    if op.startswith("v_mov") or op.startswith("v_cndmask"):
        return "vmov"
    if op.startswith("v_"):
        return "valu"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith("global_") or op.startswith("buffer_") or op.startswith("flat_"):
        return "vmem"
    if op.startswith("s_load") or op.startswith("s_buffer_load"):
        return "smem"
    if op.startswith("s_cbranch") or op.startswith("s_branch"):
        return "branch"
    if op.startswith("s_waitcnt") or op.startswith("s_nop"):
        return "wait"
    if op.startswith("s_"):
        return "salu"
    return "other"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("file")
    ap.add_argument("kernel")
    ap.add_argument("--top", type=int, default=40)
    ap.add_argument("--grep", default=None, help="also count instructions starting with this prefix")
    a = ap.parse_args()
    lines = open(a.file).read().split("\n")
    start = next(i for i, l in enumerate(lines) if re.match(r"^\w*%s\w*:" % re.escape(a.kernel), l))
    end = next(i for i in range(start, len(lines)) if lines[i].startswith(".Lfunc_end"))
    blocks, cur, order = {}, None, []
    locs = collections.defaultdict(collections.Counter)
    label_pos, branches = {}, []
    loc = None
    idx = 0
    for l in lines[start:end]:
        s = l.strip()
        if not s or s.startswith(";") or s.startswith("//"):
            continue
        m = re.match(r"^(\.LBB\w+|_Z\w+):", s)
        if m:
            cur = m.group(1)
            blocks[cur] = collections.Counter()
            order.append(cur)
            label_pos[cur] = idx
            continue
        if s.startswith(".loc"):
            f = s.split()
            loc = "%s:%s" % (f[1], f[2])
            continue
        if s.startswith("."):
            continue
        op = s.split()[0]
        if cur is None:
            continue
        c = classify(op)
        blocks[cur][c] += 1
        blocks[cur]["all"] += 1
        if a.grep and op.startswith(a.grep):
            blocks[cur]["grep"] += 1
        if loc:
            locs[cur][loc] += 1
        if c == "branch":
            tgt = s.split()[-1]
            branches.append((idx, tgt))
        idx += 1
    depth = collections.Counter()
    for bi, tgt in branches:
        if tgt in label_pos and label_pos[tgt] <= bi:
            for b in order:
                if label_pos[tgt] <= label_pos[b] <= bi:
                    depth[b] += 1
    tot = collections.Counter()
    for b in order:
        tot.update(blocks[b])
    print("kernel lines %d..%d: %s" % (start, end, dict(tot)))
    keys = ["all", "valu", "vmov", "salu", "lds", "vmem", "smem", "lane", "scratch", "branch"] + (["grep"] if a.grep else [])
    print("%-14s %5s " % ("block", "loop") + " ".join("%6s" % k for k in keys) + "  main .loc")
    rows = sorted(order, key=lambda b: (-depth[b], -blocks[b]["all"]))
    for b in rows[:a.top]:
        ml = locs[b].most_common(1)[0][0] if locs[b] else ""
        print("%-14s %5d " % (b, depth[b]) + " ".join("%6d" % blocks[b][k] for k in keys) + "  " + ml)
    lane_in_loops = sum(blocks[b]["lane"] for b in order if depth[b] > 0)
    scr_in_loops = sum(blocks[b]["scratch"] for b in order if depth[b] > 0)
    print("writelane/readlane inside loops: %d of %d; scratch ops inside loops: %d of %d"
          % (lane_in_loops, tot["lane"], scr_in_loops, tot["scratch"]))


if __name__ == "__main__":
    main()
