"""Timeline of the last Whitted frame from a rocprofv3 kernel trace
(`rocprofv3 --kernel-trace --output-format csv -d DIR -o w -- python3 tools/ab.py child`
with KERNEL=whitted): per stream (queue) the kernels in order with start
offsets and durations, the frame span and the time with 0 / 1 / 2 kernels
running.  Usage: python tools/wf_timeline.py DIR"""
import csv
import glob
import sys

f = glob.glob("%s/**/w_kernel_trace.csv" % sys.argv[1], recursive=True)[0]
rows = [r for r in csv.DictReader(open(f)) if "whitted" in r["Kernel_Name"]]
# the last frame: from the second-to-last pair of prep_kernels (two streams) on
sk = [j for j, r in enumerate(rows) if "prep_kernel" in r["Kernel_Name"]]
nstreams = 2 if len(sk) >= 2 and int(rows[sk[-1]]["Start_Timestamp"]) - int(rows[sk[-2]]["Start_Timestamp"]) < 50000 else 1
fr = rows[sk[-nstreams]:]
t0 = min(int(r["Start_Timestamp"]) for r in fr)
t1 = max(int(r["End_Timestamp"]) for r in fr)
key = "Queue_Id" if "Queue_Id" in fr[0] else "Stream_Id"
by = {}
for r in fr:
    by.setdefault(r.get(key, "?"), []).append(r)
for q, rs in by.items():
    print("queue", q, " ".join("%s@%.0f+%.0f" % (r["Kernel_Name"].split("(")[0].split("<")[0].split("::")[-1].replace("_kernel", ""),
                                                  (int(r["Start_Timestamp"]) - t0) / 1e3,
                                                  (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3) for r in rs))
ev = []
for r in fr:
    ev.append((int(r["Start_Timestamp"]), 1))
    ev.append((int(r["End_Timestamp"]), -1))
ev.sort()
busy = {0: 0, 1: 0, 2: 0}
cur, last = 0, t0
for t, d in ev:
    busy[min(cur, 2)] += t - last
    cur += d
    last = t
print("span %.0f us; 0 kernels %.0f us, 1 kernel %.0f us, >=2 kernels %.0f us" % (
    (t1 - t0) / 1e3, busy[0] / 1e3, busy[1] / 1e3, busy[2] / 1e3))
