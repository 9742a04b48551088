#!/bin/bash
# Where the level-pass kernels' waves spend their cycles (Whitted 1080p frame,
# queue tracer 800x600): one rocprofv3 --pmc pass per workload with the SQ
# cycle buckets (WAIT_ANY = parked on s_waitcnt / barrier, WAIT_INST_ANY =
# issue stall, ACTIVE_INST_ANY = issuing; the three are disjoint and sum to
# WAVE_CYCLES, MI355X_MICROARCH.md) and the per-pipe active cycles.
#   gpurun -- bash tools/pmc_stalls.sh TAG
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${1:-stalls}
OUT=gpurun_out/$TAG
rm -rf "$OUT" && mkdir -p "$OUT"
SET=${SET:-"SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA"}
KERNEL=whitted REPS=3 timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv --pmc $SET -d "$OUT/whitted" -o p \
    -- python3 tools/ab.py child > "$OUT/whitted.log" 2>&1
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv --pmc $SET -d "$OUT/queue" -o p \
    -- python3 tools/queue_time.py 3 > "$OUT/queue.log" 2>&1
python3 - "$OUT" <<'PY' | tee "$OUT/summary.txt"
import csv, glob, collections, sys
out = sys.argv[1]
for wl in ("whitted", "queue"):
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    for f in glob.glob("%s/%s/**/*counter_collection.csv" % (out, wl), recursive=True):
        for r in csv.DictReader(open(f)):
            agg[r["Kernel_Name"].split("(")[0]][r["Counter_Name"]] += float(r["Counter_Value"])
    print("== %s" % wl)
    for k, v in sorted(agg.items(), key=lambda kv: -kv[1].get("SQ_WAVE_CYCLES", 0)):
        wc = v.get("SQ_WAVE_CYCLES", 0)
        if wc <= 0:
            continue
        print("%-45s wave_cyc %.3g  wait_any %.1f%%  wait_inst %.1f%% (lds %.1f%%)  active %.1f%%  "
              "[valu %.1f%% lds %.1f%% salu %.1f%%]" % (
                  k[:45], wc, 100 * v["SQ_WAIT_ANY"] / wc, 100 * v["SQ_WAIT_INST_ANY"] / wc,
                  100 * v["SQ_WAIT_INST_LDS"] / wc, 100 * v["SQ_ACTIVE_INST_ANY"] / wc,
                  100 * v["SQ_ACTIVE_INST_VALU"] / wc, 100 * v["SQ_ACTIVE_INST_LDS"] / wc,
                  100 * v["SQ_ACTIVE_INST_SCA"] / wc))
PY
