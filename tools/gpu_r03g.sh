set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r03g; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_smallpt.py -x -q --timeout 120 --timeout-method thread > $O/t_smallpt.log 2>&1
for c in 0 1; do
  COUNTED=$c SPP=64 REPS=3 timeout -k 10 120 python tools/c5_time.py 2>&1 | grep -v amdgpu >> $O/c5.log
  RT_SPT_WIDE=0 COUNTED=$c SPP=64 REPS=3 timeout -k 10 120 python tools/c5_time.py 2>&1 | grep -v amdgpu >> $O/c5.log
done
N=200 timeout -k 10 300 python tools/bvh_stress.py > $O/bvh_stress.log 2>&1
