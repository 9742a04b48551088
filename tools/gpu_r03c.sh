set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r03c; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_smallpt.py -x -q --timeout 120 --timeout-method thread > $O/t_smallpt.log 2>&1
for k in 0 1 2 3; do
  echo "== split $k" >> $O/c5.log
  RT_SPT_SPLIT=$k SPP=64 REPS=5 timeout -k 10 120 python tools/c5_time.py >> $O/c5.log 2>&1
  RT_SPT_SPLIT=$k GROUP=3/8 SPP=64 REPS=5 timeout -k 10 120 python tools/c5_time.py >> $O/c5.log 2>&1
done
for k in 0 2 3; do
RT_SPT_SPLIT=$k RT_HIP_LIB=$GRAFT_REPO_ROOT/build_ab/trace/librt_hip.so N=8 K=3 timeout -k 10 200 python tools/c5_phase.py > $O/phase_n8_s$k.log 2>&1
done
