#!/bin/bash
# Builds A/B variants of librt_hip.so into build_ab/<name>/ (see tools/ab_smallpt.py).
set -e
cd "$(dirname "$0")/.."
P=se-195-project-ray-tracer_amd
SRCS="$P/csrc/rt_api.hip $P/csrc/whitted.hip $P/csrc/smallpt.hip"
FLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-gpu-rdc -shared -w"
build() { mkdir -p build_ab/$1; /opt/rocm/bin/hipcc $FLAGS $2 -o build_ab/$1/librt_hip.so $SRCS & }
build base ""
build w5 "-DRT_SPT_MINWAVES=5"
build w6 "-DRT_SPT_MINWAVES=6"
build w8 "-DRT_SPT_MINWAVES=8"
build branchy "-DRT_SPT_BRANCHY"
build branchy_w6 "-DRT_SPT_BRANCHY -DRT_SPT_MINWAVES=6"
wait
ls -la build_ab/*/librt_hip.so
