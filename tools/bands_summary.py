"""Per-band render_kernel rows of a tools/prof_bands.sh stats file:
    python tools/bands_summary.py gpurun_out/r02/bands_kernel_stats.csv"""
import csv
import io
import sys

txt = open(sys.argv[1]).read().split("# band")
for part in txt[1:]:
    lines = part.splitlines()
    for r in csv.DictReader(io.StringIO("\n".join(lines[1:]))):
        if "render_kernel" in r["Name"]:
            print("band%s calls %s mean %.3f ms min %.3f ms" % (lines[0], r["Calls"], float(r["AverageNs"]) / 1e6,
                                                               float(r["MinNs"]) / 1e6))
