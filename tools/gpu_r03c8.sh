# Whitted: unequal two-stream slab split sweep (RT_WHITTED_SPLIT), exactness
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r03c8; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_whitted.py -x -q --timeout 120 --timeout-method thread > $O/t_whitted.log 2>&1
for r in 1 2 3; do
  for sp in 1,1 9,7 5,4 4,3 3,2 5,3; do
    KERNEL=whitted VARIANT=split$sp RT_WHITTED_SPLIT=$sp REPS=20 WARM=3 timeout -k 10 120 python -u tools/ab.py child 2>&1 | grep whitted >> $O/split.log
  done
done
timeout -k 10 300 python -u -m pytest tests/test_gpu_smallpt.py -x -q --timeout 120 --timeout-method thread -k "cooperative or adaptive or configs4 or bvh_equals" > $O/t_smallpt.log 2>&1
for g in 0/8 3/8 0/4 1/4 0/2 ""; do
  echo "default g=$g" >> $O/c4.log
  SPP=64 GROUP=$g REPS=5 timeout -k 10 120 python -u tools/c5_time.py 2>&1 | grep c5 >> $O/c4.log
done
