set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r03d; mkdir -p $O
for opt in 16,16,0 8,16,0 4,16,0 32,16,0 16,16,32 16,16,48 32,16,32 8,8,0 16,32,0 12,16,0 64,16,32; do
  echo "== opts $opt" >> $O/c5.log
  RT_WIDE_OPTS=$opt SPP=64 REPS=3 timeout -k 10 120 python tools/c5_time.py 2>&1 | grep -v amdgpu >> $O/c5.log
  RT_WIDE_OPTS=$opt GROUP=3/8 SPP=64 REPS=3 timeout -k 10 120 python tools/c5_time.py 2>&1 | grep -v amdgpu >> $O/c5.log
done
for opt in 4,16,0 16,16,32; do
RT_WIDE_OPTS=$opt RT_HIP_LIB=$GRAFT_REPO_ROOT/build_ab/trace/librt_hip.so N=8 K=3 timeout -k 10 200 python tools/c5_phase.py > $O/phase_n8_$opt.log 2>&1
done
