set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r03e; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_smallpt.py tests/test_gpu_multi.py -x -q --timeout 120 --timeout-method thread > $O/t_smallpt.log 2>&1
for opt in 16,16,32 24,16,32 16,8,32 16,16,24 12,16,32 20,16,40 16,16,16; do
  echo "== opts $opt" >> $O/c5.log
  RT_WIDE_OPTS=$opt SPP=64 REPS=3 timeout -k 10 120 python tools/c5_time.py 2>&1 | grep -v amdgpu >> $O/c5.log
  RT_WIDE_OPTS=$opt GROUP=3/8 SPP=64 REPS=3 timeout -k 10 120 python tools/c5_time.py 2>&1 | grep -v amdgpu >> $O/c5.log
done
echo "== binary" >> $O/c5.log
RT_SPT_WIDE=0 SPP=64 REPS=3 timeout -k 10 120 python tools/c5_time.py 2>&1 | grep -v amdgpu >> $O/c5.log
RT_SPT_WIDE=0 GROUP=3/8 SPP=64 REPS=3 timeout -k 10 120 python tools/c5_time.py 2>&1 | grep -v amdgpu >> $O/c5.log
RT_HIP_LIB=$GRAFT_REPO_ROOT/build_ab/trace/librt_hip.so N=8 K=0,1,2,3,4,5,6,7 timeout -k 10 200 python tools/c5_phase.py > $O/phase_n8.log 2>&1
timeout -k 10 120 tests/native/smallpt_dropin_bench 1920 1080 3.0 > $O/dropin.log 2>&1
RT_SPT_SHIM_BATCH=1 timeout -k 10 120 tests/native/smallpt_dropin_bench 1920 1080 3.0 >> $O/dropin.log 2>&1
