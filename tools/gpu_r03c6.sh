# coop walk: 4 leaves per pass (nl4) A/B; coop tiles / heavy waves at N=2 and N=4
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r03c6; mkdir -p $O
RT_HIP_LIB=build_ab/nl4/librt_hip.so timeout -k 10 300 python -u -m pytest tests/test_gpu_smallpt.py -x -q --timeout 120 --timeout-method thread -k "cooperative or adaptive" > $O/t_nl4.log 2>&1
M=se-195-project-ray-tracer_amd/librt_hip.so
for rnd in 1 2; do
for g in 0/8 3/8 5/8 0/4; do
  for v in main nl4; do
    lib=build_ab/$v/librt_hip.so; [ $v = main ] && lib=$M
    echo "$v group=$g" >> $O/nl.log
    RT_HIP_LIB=$lib SPP=64 GROUP=$g REPS=5 timeout -k 10 120 python -u tools/c5_time.py 2>&1 | grep c5 >> $O/nl.log
  done
done
done
for cfg in "0/2 64 2" "0/2 128 4" "0/2 256 8" "0/2 0 0" "0/4 256 8" "0/4 384 12" "0/4 768 16" "0/4 0 0"; do
  set -- $cfg
  echo "group=$1 heavy=$2 hw=$3" >> $O/hw.log
  if [ $2 = 0 ]; then
    RT_SPT_SPLIT=0 SPP=64 GROUP=$1 REPS=5 timeout -k 10 120 python -u tools/c5_time.py 2>&1 | grep c5 >> $O/hw.log
  else
    RT_SPT_SPLIT=3 RT_WIDE_HEAVY=$2 RT_WIDE_HEAVY_WAVES=$3 SPP=64 GROUP=$1 REPS=5 timeout -k 10 120 python -u tools/c5_time.py 2>&1 | grep c5 >> $O/hw.log
  fi
done
