# coop walk: N=4 phase trace; heavy sub-item waves per block (RT_WIDE_HEAVY_WAVES) sweep
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r03c4; mkdir -p $O
RT_HIP_LIB=build_ab/trace/librt_hip.so RT_SPT_SPLIT=3 RT_WIDE_HEAVY=512 N=4 K=0 timeout -k 10 120 python -u tools/c5_phase.py > $O/phase_n4.log 2>&1
for g in 0/4 0/8 3/8 0/2; do
  for cfg in "main 512 0" "main 512 8" "main 512 4" "main 1024 8" "g4 1024 0" "g4 1024 8" "g4 2048 8"; do
    set -- $cfg
    lib=build_ab/$1/librt_hip.so; [ $1 = main ] && lib=se-195-project-ray-tracer_amd/librt_hip.so
    echo "$1 heavy=$2 hw=$3 group=$g" >> $O/ab.log
    RT_HIP_LIB=$lib SPP=64 RT_SPT_SPLIT=3 RT_WIDE_HEAVY=$2 RT_WIDE_HEAVY_WAVES=$3 GROUP=$g REPS=5 timeout -k 10 120 python -u tools/c5_time.py 2>&1 | grep c5 >> $O/ab.log
  done
  echo "base group=$g" >> $O/ab.log
  SPP=64 GROUP=$g REPS=5 timeout -k 10 120 python -u tools/c5_time.py 2>&1 | grep c5 >> $O/ab.log
done
