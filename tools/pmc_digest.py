"""Condenses a tools/prof_round.sh output directory into per-kernel averages
per launch (JSON on stdout): HBM traffic from FETCH_SIZE / WRITE_SIZE (kB;
FETCH_SIZE doubled per the gfx950 correction in MI355X_MICROARCH.md, HBM
section), VALU instruction counts, lane utilisation and VALU issue fraction.
Usage: python tools/pmc_digest.py gpurun_out/r01"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

SIMDS, CLOCK_HZ = 1024, 2.4e9        # 256 CUs x 4 SIMDs, MI355X_MICROARCH.md

root = sys.argv[1]
acc = defaultdict(lambda: defaultdict(list))
dur = defaultdict(list)
for f in sorted(glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True)):
    for r in csv.DictReader(open(f)):
        name = r["Kernel_Name"]
        if not any(t in name for t in ("rt::smallpt::", "rt::whitted::", "rt::queue::")):
            continue
        key = name.split("(")[0].replace("void ", "")
        acc[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
for f in sorted(glob.glob(os.path.join(root, "**", "*kernel_stats.csv"), recursive=True)):
    for r in csv.DictReader(open(f)):
        if any(t in r["Name"] for t in ("rt::smallpt::", "rt::whitted::", "rt::queue::")):
            dur[r["Name"].split("(")[0].replace("void ", "")].append(float(r["AverageNs"]))
out = {}
for k, c in acc.items():
    m = {n: sum(v) / len(v) for n, v in c.items()}   # per launch
    d = {"launches_sampled": max(len(v) for v in c.values())}
    if "FETCH_SIZE" in m:
        d["fetch_bytes"] = 2 * m["FETCH_SIZE"] * 1024
    if "WRITE_SIZE" in m:
        d["write_bytes"] = m["WRITE_SIZE"] * 1024
    if "fetch_bytes" in d and "write_bytes" in d:
        d["traffic_bytes"] = d["fetch_bytes"] + d["write_bytes"]
    for n in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR",
              "SQ_WAVES", "SQ_INSTS_VALU_TRANS_F32", "SQ_INSTS_VALU_FMA_F64", "SQ_INSTS_BRANCH"):
        if n in m:
            d[n] = m[n]
    if m.get("SQ_ACTIVE_INST_VALU"):
        d["lane_util"] = m["SQ_THREAD_CYCLES_VALU"] / (64 * m["SQ_ACTIVE_INST_VALU"])
    if k in dur and "SQ_INSTS_VALU" in m:
        t = min(dur[k]) * 1e-9
        d["kernel_ns"] = min(dur[k])
        # wave64 VALU op = 2 issue cycles on a SIMD32 (MI355X_MICROARCH.md)
        d["valu_issue_frac"] = m["SQ_INSTS_VALU"] * 2 / (SIMDS * CLOCK_HZ * t)
    out[k] = d
print(json.dumps(out, indent=1, sort_keys=True))
