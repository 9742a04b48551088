#!/bin/bash
# configs[4] per-rank time of interleaved groups (GROUP=k/N) and the full
# frame for the build_ab variants in $LIBS (tools/c5_time.py, 64 spp).
for r in 1 2; do for v in ${LIBS//,/ }; do for g in "" 0/4 0/8; do
  echo -n "$v group=$g: "
  RT_HIP_LIB=$GRAFT_REPO_ROOT/build_ab/$v/librt_hip.so GROUP=$g SPP=64 REPS=3 timeout -k 10 120 python tools/c5_time.py 2>&1 \
      | grep -v amdgpu.ids | sed 's/.*spheres=10000: //' | cut -c1-40
done; done; done
