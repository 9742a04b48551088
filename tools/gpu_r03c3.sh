# coop walk v2 (leaf children tested at their parent) and G=4: exactness, then A/B vs v1
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r03c3; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_smallpt.py -x -q --timeout 120 --timeout-method thread -k "cooperative" > $O/t_coop.log 2>&1
RT_SPT_SPLIT=3 timeout -k 10 300 python -u -m pytest tests/test_gpu_smallpt.py -x -q --timeout 120 --timeout-method thread -k "adaptive or bvh_equals" > $O/t_adapt.log 2>&1
RT_HIP_LIB=build_ab/g4/librt_hip.so timeout -k 10 300 python -u -m pytest tests/test_gpu_smallpt.py -x -q --timeout 120 --timeout-method thread -k "cooperative" > $O/t_coop_g4.log 2>&1
RT_HIP_LIB=build_ab/trace/librt_hip.so RT_SPT_SPLIT=3 RT_WIDE_HEAVY=512 N=8 K=0 timeout -k 10 120 python -u tools/c5_phase.py > $O/phase_coop.log 2>&1
for rnd in 1 2; do
for g in 0/8 3/8 0/4; do
  for v in v1 main g4; do
    lib=build_ab/$v/librt_hip.so; [ $v = main ] && lib=se-195-project-ray-tracer_amd/librt_hip.so
    for h in 512 1024; do
      echo "$v heavy=$h group=$g" >> $O/ab.log
      RT_HIP_LIB=$lib SPP=64 RT_SPT_SPLIT=3 RT_WIDE_HEAVY=$h GROUP=$g REPS=5 timeout -k 10 120 python -u tools/c5_time.py 2>&1 | grep c5 >> $O/ab.log
    done
  done
done
done
for v in v1 main g4; do
  lib=build_ab/$v/librt_hip.so; [ $v = main ] && lib=se-195-project-ray-tracer_amd/librt_hip.so
  for h in 64 256; do
    echo "$v heavy=$h group=full" >> $O/ab.log
    RT_HIP_LIB=$lib SPP=64 RT_SPT_SPLIT=3 RT_WIDE_HEAVY=$h REPS=5 timeout -k 10 120 python -u tools/c5_time.py 2>&1 | grep c5 >> $O/ab.log
  done
done
