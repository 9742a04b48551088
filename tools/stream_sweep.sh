#!/bin/bash
# Slab / stream settings of the level-pass tracers, one child process each
# (env knobs RT_QUEUE_SLABS / RT_QUEUE_STREAMS, RT_WHITTED_SLABS /
# RT_WHITTED_STREAMS), interleaved ROUNDS times.  Output appended to $OUT.
#   OUT=gpurun_out/x/sweep.log ROUNDS=2 bash tools/stream_sweep.sh
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for r in $(seq 1 "${ROUNDS:-2}"); do
  for q in "-" "RT_QUEUE_STREAMS=2" "RT_QUEUE_STREAMS=2 RT_QUEUE_SLABS=4" "RT_QUEUE_SLABS=6" "RT_QUEUE_STREAMS=2 RT_QUEUE_SLABS=6"; do
    echo "--- queue [$q] round=$r" >> "$OUT"
    env ${q/-/} timeout -k 10 120 python -u tools/queue_time.py 20 2>&1 | grep -v amdgpu.ids >> "$OUT"
  done
  for wv in "-" "RT_WHITTED_SLABS=4" "RT_WHITTED_SLABS=6" "RT_WHITTED_STREAMS=1"; do
    echo "--- whitted [$wv] round=$r" >> "$OUT"
    env ${wv/-/} KERNEL=whitted LIBS=main ROUNDS=1 REPS=20 WARM=3 timeout -k 10 200 python -u tools/ab.py 2>&1 | grep -v amdgpu.ids >> "$OUT"
    env ${wv/-/} WH=640x480 KERNEL=whitted LIBS=main ROUNDS=1 REPS=20 WARM=3 timeout -k 10 200 python -u tools/ab.py 2>&1 | grep -v amdgpu.ids >> "$OUT"
  done
done
