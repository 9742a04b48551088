# default coop policy + queue gather fold: full GPU suite, queue A/B, configs[4] windows, stress
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r03c5; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_queue.py -x -q --timeout 120 --timeout-method thread > $O/t_queue.log 2>&1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gputests.log 2>&1
for r in 1 2 3; do
  for v in main qg0; do
    lib=build_ab/$v/librt_hip.so; [ $v = main ] && lib=se-195-project-ray-tracer_amd/librt_hip.so
    echo "lib=$v" >> $O/queue_ab.log
    RT_HIP_LIB=$lib timeout -k 10 120 python -u tools/queue_time.py 20 2>&1 | grep -v amdgpu >> $O/queue_ab.log
  done
done
for g in "" 0/2 0/4 1/4 0/8 3/8 5/8; do
  echo "default group=$g" >> $O/c4.log
  SPP=64 GROUP=$g REPS=5 timeout -k 10 120 python -u tools/c5_time.py 2>&1 | grep c5 >> $O/c4.log
done
REPEAT=2 N=60 SEED=11 timeout -k 10 400 python -u tools/bvh_stress.py > $O/bvh_stress_coop.log 2>&1
