set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r03w; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_smallpt.py -x -q --timeout 120 --timeout-method thread > $O/t_smallpt.log 2>&1
N=200 SEED=11 timeout -k 10 300 python -u tools/bvh_stress.py > $O/bvh_stress.log 2>&1
for r in 1 2; do
for v in f8 f16; do
  for g in "" 3/8 0/8; do
    echo "lib=$v group=$g" >> $O/f16.log
    RT_HIP_LIB=$GRAFT_REPO_ROOT/build_ab/$v/librt_hip.so SPP=64 GROUP=$g REPS=5 timeout -k 10 120 python -u tools/c5_time.py >> $O/f16.log 2>&1
  done
  echo "lib=$v counted" >> $O/f16.log
  RT_HIP_LIB=$GRAFT_REPO_ROOT/build_ab/$v/librt_hip.so COUNTED=1 SPP=64 REPS=3 timeout -k 10 120 python -u tools/c5_time.py >> $O/f16.log 2>&1
done
done
