# Whitted: root kernel at occupancy 7 (r7: 72 VGPRs, 28 B scratch) vs 6 (base)
# exactness, frame times, PMC traffic per frame
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r03ah; mkdir -p $O
RT_HIP_LIB=$GRAFT_REPO_ROOT/build_ab/r7/librt_hip.so timeout -k 10 400 python -u -m pytest tests/test_gpu_whitted.py -x -q --timeout 120 --timeout-method thread > $O/t_whitted.log 2>&1
LIBS=base,r7 KERNEL=whitted ROUNDS=4 REPS=20 WARM=3 timeout -k 10 300 python -u tools/ab.py > $O/ab.log 2>&1
WH=640x480 LIBS=base,r7 KERNEL=whitted ROUNDS=4 REPS=20 WARM=3 timeout -k 10 300 python -u tools/ab.py >> $O/ab.log 2>&1
