# three-tier dispatch (cooperative, routed heavy, rest): exactness, then sweeps at N=8/4/2
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r03c7; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_smallpt.py -x -q --timeout 120 --timeout-method thread -k "cooperative or adaptive or bvh_equals or configs4" > $O/t_tiers.log 2>&1
REPEAT=2 N=40 SEED=13 timeout -k 10 300 python -u tools/bvh_stress.py > $O/bvh_stress.log 2>&1
run() { echo "$1" >> $O/ab.log; shift; env "$@" SPP=64 REPS=5 timeout -k 10 120 python -u tools/c5_time.py 2>&1 | grep c5 >> $O/ab.log; }
for rnd in 1 2; do
  for g in 0/8 3/8; do
    run "default g=$g" GROUP=$g
    run "n2=0 g=$g" GROUP=$g RT_WIDE_HEAVY=0
  done
  for g in 0/4 1/4; do
    run "default g=$g" GROUP=$g
    run "n2=0 g=$g" GROUP=$g RT_WIDE_HEAVY=0
    run "n1=256 hw=8 g=$g" GROUP=$g RT_WIDE_COOP=256 RT_WIDE_HEAVY_WAVES=8
    run "n1=768 hw=12 g=$g" GROUP=$g RT_WIDE_COOP=768 RT_WIDE_HEAVY_WAVES=12
  done
  run "default g=0/2" GROUP=0/2
  run "n1=64 hw=2 g=0/2" GROUP=0/2 RT_WIDE_COOP=64 RT_WIDE_HEAVY_WAVES=2
  run "n1=128 hw=4 g=0/2" GROUP=0/2 RT_WIDE_COOP=128 RT_WIDE_HEAVY_WAVES=4
  run "n1=256 hw=8 g=0/2" GROUP=0/2 RT_WIDE_COOP=256 RT_WIDE_HEAVY_WAVES=8
done
run "default full" GROUP=
timeout -k 10 300 python -u -m pytest tests/test_gpu_queue.py -x -q --timeout 120 --timeout-method thread > $O/t_queue.log 2>&1
for r in 1 2 3; do
  for v in main fr32; do
    lib=build_ab/$v/librt_hip.so; [ $v = main ] && lib=se-195-project-ray-tracer_amd/librt_hip.so
    echo "lib=$v" >> $O/queue_ab.log
    RT_HIP_LIB=$lib timeout -k 10 120 python -u tools/queue_time.py 20 2>&1 | grep -v amdgpu >> $O/queue_ab.log
  done
done
