#!/bin/bash
# A/B of build_ab variants in $LIBS on the three 1-GPU workloads: Cornell
# 1080p 64 spp and Whitted 1080p (tools/ab.py), configs[4] at 16 spp
# (tools/c5_time.py); two interleaved rounds.
for round in 1 2; do
  for v in ${LIBS//,/ }; do
    L=$GRAFT_REPO_ROOT/build_ab/$v/librt_hip.so
    RT_HIP_LIB=$L VARIANT=$v REPS=5 timeout -k 10 120 python tools/ab.py child 2>&1 | grep -v amdgpu.ids
    RT_HIP_LIB=$L VARIANT=$v KERNEL=whitted REPS=10 WARM=3 timeout -k 10 120 python tools/ab.py child 2>&1 | grep -v amdgpu.ids
    echo -n "$v: "; RT_HIP_LIB=$L SPP=16 REPS=5 timeout -k 10 120 python tools/c5_time.py 2>&1 | grep -v amdgpu.ids
  done
done
