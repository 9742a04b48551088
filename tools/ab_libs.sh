#!/bin/bash
# Interleaved A/B of library builds on the GPU box (each run a child process
# with RT_HIP_LIB): WHAT=queue (tools/queue_time.py), cornell (tools/ab.py
# KERNEL=smallpt), c4 (tools/c4_partition.py QUICK=1).  LIBS: names under
# build_ab/, "main" = the in-tree librt_hip.so.  Output appended to $OUT.
#   WHAT=queue LIBS=q0,main ROUNDS=2 OUT=gpurun_out/x/ab.log bash tools/ab_libs.sh
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
lib_path() { [ "$1" = main ] && echo "$PWD/se-195-project-ray-tracer_amd/librt_hip.so" || echo "$PWD/build_ab/$1/librt_hip.so"; }
for r in $(seq 1 "${ROUNDS:-2}"); do
  for lib in ${LIBS//,/ }; do
    echo "--- $WHAT lib=$lib round=$r" >> "$OUT"
    case "$WHAT" in
      queue) RT_HIP_LIB=$(lib_path $lib) timeout -k 10 120 python -u tools/queue_time.py "${REPS:-20}" 2>&1 | grep -v amdgpu.ids >> "$OUT" ;;
      cornell) KERNEL=smallpt LIBS=$lib ROUNDS=1 REPS=${REPS:-7} timeout -k 10 200 python -u tools/ab.py 2>&1 | grep -v amdgpu.ids >> "$OUT" ;;
      whitted) KERNEL=whitted LIBS=$lib ROUNDS=1 REPS=${REPS:-20} WARM=3 timeout -k 10 200 python -u tools/ab.py 2>&1 | grep -v amdgpu.ids >> "$OUT" ;;
      c4) RT_HIP_LIB=$(lib_path $lib) QUICK=1 NS=${NS:-4,8} timeout -k 10 400 python -u tools/c4_partition.py 2>&1 | grep -v amdgpu.ids >> "$OUT" ;;
    esac
  done
done
