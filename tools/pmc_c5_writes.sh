#!/bin/bash
# HBM bytes of the configs[4] hierarchy kernel (one 64-spp frame, tools/c5_time.py)
# for each build_ab variant in $LIBS: FETCH_SIZE and WRITE_SIZE passes.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/pmcw
for v in ${LIBS//,/ }; do
  for c in FETCH_SIZE WRITE_SIZE; do
    RT_HIP_LIB=$GRAFT_REPO_ROOT/build_ab/$v/librt_hip.so SPP=64 REPS=1 timeout -k 10 120 \
      rocprofv3 --kernel-trace --output-format csv --pmc $c -d gpurun_out/pmcw/$v/$c -o p -- python3 tools/c5_time.py \
      > gpurun_out/pmcw/$v.$c.log 2>&1
    python3 - "$v" "$c" <<'PY'
import csv, glob, sys
v, c = sys.argv[1], sys.argv[2]
f = glob.glob("gpurun_out/pmcw/%s/%s/**/p_counter_collection.csv" % (v, c), recursive=True)[0]
rows = [r for r in csv.DictReader(open(f)) if "render_kernel" in r["Kernel_Name"]]
for r in rows:
    print(v, c, r["Kernel_Name"].split("(")[0][-40:], r.get("Counter_Value"), r.get("Dispatch_Id"))
PY
  done
done
