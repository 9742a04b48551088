#!/bin/bash
# configs[4] timing (tools/c5_time.py, SPP=4) for each build_ab variant in $LIBS.
for v in ${LIBS//,/ }; do
  echo -n "$v: "
  RT_HIP_LIB=$GRAFT_REPO_ROOT/build_ab/$v/librt_hip.so SPP=${SPP:-4} REPS=${REPS:-1} timeout -k 10 300 python tools/c5_time.py 2>&1 | grep -v amdgpu.ids
done
