# coop walk: DPP-folded integer reductions (main) vs v2 (fminf); exactness + N=8/N=4 A/B
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r03c11; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_smallpt.py -x -q --timeout 120 --timeout-method thread -k "cooperative or adaptive or configs4 or bvh_equals" > $O/t_smallpt.log 2>&1
REPEAT=2 N=40 SEED=17 timeout -k 10 300 python -u tools/bvh_stress.py > $O/bvh_stress.log 2>&1
M=se-195-project-ray-tracer_amd/librt_hip.so
for rnd in 1 2 3; do
for g in 0/8 3/8 5/8 0/4; do
  for v in main v2; do
    lib=build_ab/$v/librt_hip.so; [ $v = main ] && lib=$M
    echo "$v group=$g" >> $O/ab.log
    RT_HIP_LIB=$lib SPP=64 GROUP=$g REPS=5 timeout -k 10 120 python -u tools/c5_time.py 2>&1 | grep c5 >> $O/ab.log
  done
done
done
