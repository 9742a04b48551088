#!/bin/bash
# Priority-levelling schedule A/B (RT_SPT_PRIO_SCHED=64,128,192 vs 128,192,224) on the full frame and
# on one row band of N = 2/4/8 (tools/ab.py child; build_ab/$V).
L=$GRAFT_REPO_ROOT/build_ab/${V:-pl}/librt_hip.so
for r in 1 2; do
  for band in "" 1/2 1/4 1/8 3/8; do
    for late in 0 1; do
      echo -n "late=$late "
      RT_SPT_PRIO_SCHED=$([ $late = 1 ] && echo 128,192,224 || echo 64,128,192) RT_HIP_LIB=$L BAND=$band VARIANT=late$late REPS=8 timeout -k 10 120 python tools/ab.py child 2>&1 | grep -v amdgpu.ids
    done
  done
done
