#!/bin/bash
# Builds an A/B variant of librt_hip.so from the working tree into
# build_ab/<name>/ (timed by tools/ab.py).  Usage: tools/build_variants.sh NAME [hipcc flags...]
set -e
cd "$(dirname "$0")/.."
NAME=$1; shift
P=se-195-project-ray-tracer_amd
SRCS="$P/csrc/rt_api.hip $P/csrc/whitted.hip $P/csrc/smallpt.hip $P/csrc/spt_multi.hip $P/csrc/queue.hip"
mkdir -p build_ab/$NAME
/opt/rocm/bin/hipcc --offload-arch=${ARCH:-gfx950} -O3 -std=c++17 -fPIC -ffp-contract=off -fno-slp-vectorize -fno-gpu-rdc -shared -w "$@" \
    -o build_ab/$NAME/librt_hip.so $SRCS
