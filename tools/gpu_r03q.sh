set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r03q; mkdir -p $O
for r in 1 2; do
for lf in 8 5 6; do
  for g in "" 3/8 0/8; do
    echo "leaf=$lf group=$g" >> $O/leaf.log
    RT_SPT_WIDE_LEAF=$lf SPP=64 GROUP=$g REPS=5 timeout -k 10 120 python -u tools/c5_time.py >> $O/leaf.log 2>&1
  done
done
done
