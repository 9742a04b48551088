"""HBM traffic per frame from rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes
(FETCH_SIZE doubled: the gfx950 correction of MI355X_MICROARCH.md's HBM
section; kB units): sums every launch of the named kernel family, divided by
the frames rendered (root_kernel launches / SLABS).
Usage: SLABS=2 python tools/pmc_frame_sum.py <dir> [rt::whitted::]"""
import csv
import glob
import os
import sys
from collections import defaultdict

root = sys.argv[1]
fam = sys.argv[2] if len(sys.argv) > 2 else "rt::whitted::"
slabs = int(os.environ.get("SLABS", "2"))
tot = defaultdict(float)
roots = defaultdict(int)
per = defaultdict(lambda: defaultdict(float))
for f in sorted(glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True)):
    for r in csv.DictReader(open(f)):
        name = r["Kernel_Name"]
        if fam not in name:
            continue
        k = name.split("(")[0].replace("void ", "").replace(fam, "").split("<")[0]
        c, v = r["Counter_Name"], float(r["Counter_Value"])
        b = 2 * v * 1024 if c == "FETCH_SIZE" else v * 1024
        tot[c] += b
        per[k][c] += b
        if k == "root_kernel":
            roots[c] += 1
for c in sorted(tot):
    frames = max(1, roots[c] // slabs)
    print("%s: %.1f MB per frame (%d frames)" % (c, tot[c] / frames / 1e6, frames))
    for k in sorted(per):
        print("   %-16s %.1f MB" % (k, per[k][c] / frames / 1e6))
if len(tot) == 2:
    frames = {c: max(1, roots[c] // slabs) for c in tot}
    print("traffic: %.1f MB per frame" % sum(tot[c] / frames[c] / 1e6 for c in tot))
