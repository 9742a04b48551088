#!/bin/bash
# Priority-levelling schedules (RT_SPT_PRIO_SCHED=a,b,c in 1/256 of the
# samples) on the full frame ($FULL) and on the N=8 band 1/8 ($BAND8).
L=$GRAFT_REPO_ROOT/build_ab/${V:-ps}/librt_hip.so
for r in 1 2; do
  for sc in $FULL; do
    RT_SPT_PRIO_SCHED=$sc RT_HIP_LIB=$L VARIANT=$sc REPS=6 timeout -k 10 120 python tools/ab.py child 2>&1 | grep -v amdgpu.ids
  done
  for sc in $BAND8; do
    RT_SPT_PRIO_SCHED=$sc RT_HIP_LIB=$L BAND=1/8 VARIANT=$sc REPS=8 timeout -k 10 120 python tools/ab.py child 2>&1 | grep -v amdgpu.ids
  done
done
