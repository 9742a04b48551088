#!/bin/bash
# configs[4] with the adaptive order and RT_SPT_HEAVY groups kept at top
# priority ($HV list), full frame, two rounds (tools/c5_time.py, 64 spp).
export RT_HIP_LIB=${RT_HIP_LIB:-$GRAFT_REPO_ROOT/build_ab/hv/librt_hip.so}
for r in 1 2; do for hv in ${HV:-0 128 256 512 1024}; do
  echo -n "heavy=$hv "; RT_SPT_HEAVY=$hv SPP=64 REPS=4 timeout -k 10 120 python tools/c5_time.py 2>&1 | grep -v amdgpu.ids
done; done
