#!/bin/bash
# Per-kernel times of the last Whitted 1080p frame for each environment
# variant in $VARS (space-separated NAME=VALUE, "-" = none), e.g.
#   VARS="RT_WHITTED_SLABS=1 RT_WHITTED_SLABS=2" bash tools/wf_env.sh
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
i=0
for v in $VARS; do
  i=$((i+1))
  ( [ "$v" != "-" ] && export "$v"; export KERNEL=whitted REPS=3
    timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/wfe/$i -o w \
      -- python3 tools/ab.py child > gpurun_out/wfe_$i.log 2>&1 )
  python3 - "$i" "$v" <<'PY'
import csv, glob, sys
f = glob.glob("gpurun_out/wfe/%s/**/w_kernel_trace.csv" % sys.argv[1], recursive=True)[0]
rows = [r for r in csv.DictReader(open(f)) if "whitted" in r["Kernel_Name"]]
# last frame: from the last scene_kernel on
k = max(j for j, r in enumerate(rows) if "scene_kernel" in r["Kernel_Name"])
fr = rows[k:]
t0 = int(fr[0]["Start_Timestamp"]); t1 = int(fr[-1]["End_Timestamp"])
out = []
for r in fr:
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000
    out.append("%s:%.0f" % (r["Kernel_Name"].split("(")[0].split("<")[0].split("::")[-1].replace("_kernel", ""), d))
busy = sum((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) for r in fr) / 1000
print("%s | span %.0f us busy %.0f us | %s" % (sys.argv[2], (t1 - t0) / 1000, busy, " ".join(out)))
PY
done
