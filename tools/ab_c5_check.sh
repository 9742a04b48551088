#!/bin/bash
# Exactness of build_ab variant $CHECK (smallpt GPU tests), then configs[4]
# timings of the variants in $LIBS (tools/ab_c5.sh), two rounds.
set -o pipefail
RT_HIP_LIB=$GRAFT_REPO_ROOT/build_ab/$CHECK/librt_hip.so timeout -k 10 300 python -u -m pytest tests/test_gpu_smallpt.py \
    -x -q --timeout 120 --timeout-method thread > gpurun_out/ab_check.log 2>&1
tail -2 gpurun_out/ab_check.log
LIBS=$LIBS,$LIBS bash tools/ab_c5.sh
