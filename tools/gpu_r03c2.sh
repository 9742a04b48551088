# coop walk: phase trace at N=8 and heavy-count sweeps at N=1/2/4/8 windows
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r03c2; mkdir -p $O
RT_HIP_LIB=build_ab/trace/librt_hip.so RT_SPT_SPLIT=3 RT_WIDE_HEAVY=512 N=8 K=0,3 timeout -k 10 120 python -u tools/c5_phase.py > $O/phase_coop.log 2>&1
for g in 0/4 1/4 0/2 ""; do
  for h in 0 64 128 256 512 1024; do
    echo "split=3 heavy=$h group=$g" >> $O/ab.log
    SPP=64 RT_SPT_SPLIT=3 RT_WIDE_HEAVY=$h GROUP=$g REPS=5 timeout -k 10 120 python -u tools/c5_time.py >> $O/ab.log 2>&1
  done
done
