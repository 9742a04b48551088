"""Sums rocprofv3 --pmc counter_collection CSVs per (variant, kernel) for the
render kernels: python tools/pmc_summary.py DIR (DIR/<variant>/<pass>/*counter_collection.csv)."""
import csv
import glob
import os
import sys
from collections import defaultdict

root = sys.argv[1]
res = defaultdict(lambda: defaultdict(float))
for f in sorted(glob.glob(os.path.join(root, "*", "*", "*counter_collection.csv"))):
    var = f.split(os.sep)[-3]
    for row in csv.DictReader(open(f)):
        if "render_kernel" not in row["Kernel_Name"]:
            continue
        kern = "smallpt" if "smallpt" in row["Kernel_Name"] else "whitted"
        res[(var, kern)][row["Counter_Name"]] += float(row["Counter_Value"])
for (var, kern), c in sorted(res.items()):
    print("== %s %s" % (var, kern))
    for k in sorted(c):
        print("  %-26s %16.0f" % (k, c[k]))
    w = c.get("SQ_WAVES", 0)
    if w:
        print("  VALU/wave %.0f  SALU/wave %.0f  branch/wave %.0f" % (
            c["SQ_INSTS_VALU"] / w, c["SQ_INSTS_SALU"] / w, c["SQ_INSTS_BRANCH"] / w))
    if c.get("SQ_ACTIVE_INST_VALU"):
        print("  lane util %.3f" % (c["SQ_THREAD_CYCLES_VALU"] / (64 * c["SQ_ACTIVE_INST_VALU"])))
