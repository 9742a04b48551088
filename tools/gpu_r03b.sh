set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r03b; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_smallpt.py -x -v --timeout 120 --timeout-method thread > $O/t_smallpt.log 2>&1
echo "== wide (default)" > $O/c5.log
SPP=64 REPS=5 timeout -k 10 120 python tools/c5_time.py >> $O/c5.log 2>&1
echo "== wide, GROUP=3/8" >> $O/c5.log
GROUP=3/8 SPP=64 REPS=5 timeout -k 10 120 python tools/c5_time.py >> $O/c5.log 2>&1
echo "== binary" >> $O/c5.log
RT_SPT_WIDE=0 SPP=64 REPS=5 timeout -k 10 120 python tools/c5_time.py >> $O/c5.log 2>&1
echo "== wide, wpb 8, 2 blocks/CU" >> $O/c5.log
RT_WIDE_WPB=8 RT_WIDE_BLOCKS=512 SPP=64 REPS=5 timeout -k 10 120 python tools/c5_time.py >> $O/c5.log 2>&1
echo "== wide static (no persist)" >> $O/c5.log
RT_HIP_LIB=$GRAFT_REPO_ROOT/build_ab/wide_np/librt_hip.so SPP=64 REPS=5 timeout -k 10 120 python tools/c5_time.py >> $O/c5.log 2>&1
RT_HIP_LIB=$GRAFT_REPO_ROOT/build_ab/trace/librt_hip.so N=8 K=3 timeout -k 10 200 python tools/c5_phase.py > $O/phase_n8.log 2>&1
RT_HIP_LIB=$GRAFT_REPO_ROOT/build_ab/trace/librt_hip.so N=1 K=0 timeout -k 10 200 python tools/c5_phase.py > $O/phase_n1.log 2>&1
