#!/bin/bash
# VALU instruction mix of one smallpt launch (tools/ab.py child, REPS=1) for
# the build_ab variants in $LIBS.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export REPS=1
mkdir -p gpurun_out/pmc_mix
for v in ${LIBS//,/ }; do
  export RT_HIP_LIB=$GRAFT_REPO_ROOT/build_ab/$v/librt_hip.so VARIANT=$v
  timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv \
      --pmc SQ_INSTS_VALU SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_CVT SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_MUL_F64 \
      -d gpurun_out/pmc_mix/$v -o p -- python3 tools/ab.py child > gpurun_out/pmc_mix/$v.log 2>&1
done
python3 tools/pmc_summary.py gpurun_out/pmc_mix
