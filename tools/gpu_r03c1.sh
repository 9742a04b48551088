# cooperative 8-lanes-per-pixel walk for heavy tiles: exactness, then A/B
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r03c1; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_smallpt.py -x -v --timeout 120 --timeout-method thread -k "cooperative" > $O/t_coop.log 2>&1
RT_SPT_SPLIT=3 timeout -k 10 300 python -u -m pytest tests/test_gpu_smallpt.py -x -q --timeout 120 --timeout-method thread -k "adaptive" > $O/t_adapt.log 2>&1
for g in "" 3/8 0/8; do
  echo "split=0 group=$g" >> $O/ab.log
  SPP=64 GROUP=$g REPS=5 timeout -k 10 120 python -u tools/c5_time.py >> $O/ab.log 2>&1
  for h in 256 512 1024 2048; do
    echo "split=3 heavy=$h group=$g" >> $O/ab.log
    SPP=64 RT_SPT_SPLIT=3 RT_WIDE_HEAVY=$h GROUP=$g REPS=5 timeout -k 10 120 python -u tools/c5_time.py >> $O/ab.log 2>&1
  done
done
