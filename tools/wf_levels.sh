#!/bin/bash
# Per-launch kernel times of one Whitted frame for each build_ab variant in $LIBS.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for v in ${LIBS//,/ }; do
  export RT_HIP_LIB=$GRAFT_REPO_ROOT/build_ab/$v/librt_hip.so KERNEL=whitted REPS=2
  timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/wfl/$v -o w \
      -- python3 tools/ab.py child > /dev/null 2>&1
  python3 - "$v" <<'PY'
import csv, glob, sys
f = glob.glob("gpurun_out/wfl/%s/**/w_kernel_trace.csv" % sys.argv[1], recursive=True)[0]
rows = [r for r in csv.DictReader(open(f)) if "whitted" in r["Kernel_Name"]]
last = rows[-16:] if len(rows) >= 16 else rows
tot = 0
out = []
for r in rows[-14:]:
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000
    tot += d
    out.append("%s %.0f" % (r["Kernel_Name"].split("(")[0].split("::")[-1][:14], d))
print(sys.argv[1], "|", " ".join(out))
PY
done
