#!/bin/bash
# configs[4] with the adaptive group order off / on (RT_SPT_SCHED=0/1): full
# frame twice, then row bands of N = 2/4/8 (tools/c5_time.py, 64 spp).
export RT_HIP_LIB=${RT_HIP_LIB:-$GRAFT_REPO_ROOT/build_ab/sched/librt_hip.so}
for r in 1 2; do for sch in 0 1; do
  echo -n "sched=$sch "; RT_SPT_SCHED=$sch SPP=64 REPS=3 timeout -k 10 120 python tools/c5_time.py 2>&1 | grep -v amdgpu.ids
done; done
for b in 1/2 1/4 1/8; do for sch in 0 1; do
  echo -n "sched=$sch "; RT_SPT_SCHED=$sch BAND=$b SPP=64 REPS=3 timeout -k 10 120 python tools/c5_time.py 2>&1 | grep -v amdgpu.ids
done; done
